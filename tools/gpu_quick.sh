# quick GPU iteration: parity tests (not slow) + 1-GPU bench + kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${1:-q}
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "not slow" > gpurun_out/$TAG.pytest.log 2>&1; rc=$?; echo "pytest exit $rc" >> gpurun_out/$TAG.pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG.bench.log 2>&1 || exit 2
TFHE_BR_KERNEL=split timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG.bench_split.log 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG.prof -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/$TAG.prof.log 2>&1 || exit 3
