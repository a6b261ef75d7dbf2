# BASELINE configs 3-5 lines + kernel stats of the LUT and mixed workloads
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_workloads.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_lut -o lut -- python3 $R/bench.py --workload lut --batch 4096 --steps 3 --warmup 1 > $R/gpurun_out/prof_lut.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_mixed -o mixed -- python3 $R/bench.py --workload mixed --batch 8192 --steps 3 --warmup 1 > $R/gpurun_out/prof_mixed.log 2>&1 || exit 1
