# Round 5: where a host-buffer gate batch's time goes (1,024 NAND, 128-bit): plain-context wall
# times, the single-process multi-device line, the device-resident line, and the rocprofv3
# timeline of the plain-context calls (tools/host_path_trace.py).   bash tools/gpu_r05hp.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r05hp}
cd $R
mkdir -p gpurun_out
timeout -k 10 200 python tools/host_path_trace.py > gpurun_out/$TAG.plain.txt 2>&1 && grep "host wall" gpurun_out/$TAG.plain.txt || exit 1
timeout -k 10 200 python bench.py --single-process --gpus 1 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG.sp1.json 2>/dev/null || exit 2
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('single-process 1 device', d['value'], d['ms_per_step'])" gpurun_out/$TAG.sp1.json
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/$TAG.bench.json 2>/dev/null || exit 3
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('device-resident', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])" gpurun_out/$TAG.bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $R/gpurun_out/$TAG.trace -o run -- python3 $R/tools/host_path_trace.py > $R/gpurun_out/$TAG.trace.log 2>&1 || exit 4
cd $R && python3 tools/host_path_trace.py --report gpurun_out/$TAG.trace > gpurun_out/$TAG.report.txt 2>&1; tail -40 gpurun_out/$TAG.report.txt
