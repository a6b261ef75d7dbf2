# host-buffer path timeline (tools/host_path_trace.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $R/gpurun_out/hp -o run -- python3 $R/tools/host_path_trace.py > $R/gpurun_out/hp.log 2>&1 || { tail $R/gpurun_out/hp.log; exit 1; }
cd $R && grep "host wall" gpurun_out/hp.log && python3 tools/host_path_trace.py --report gpurun_out/hp > gpurun_out/hp_report.txt && tail -60 gpurun_out/hp_report.txt
