# proxy re-encryption workload: bench lines + kernel time
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload reenc --batch 16384 --steps 5 --warmup 1 > gpurun_out/wl_reenc16k.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_reenc -o reenc -- python3 bench.py --workload reenc --batch 16384 --steps 5 --warmup 1 > gpurun_out/prof_reenc.log 2>&1 || exit 1
