# Iteration check: GPU parity tests (optionally -k EXPR), the default bench without the CPU
# baseline, and rocprof kernel stats of the bench.  bash tools/gpu_iter.sh TAG [pytest -k expr]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-iter}
K=${2:-}
cd $R
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/$TAG.gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/$TAG.gpu_tests.log; exit 1; }
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG.gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/$TAG.gpu_tests.log; exit 1; }
fi
tail -2 gpurun_out/$TAG.gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || { echo "bench failed"; tail -20 gpurun_out/$TAG.bench.err; exit 1; }
cat gpurun_out/$TAG.bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG.prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/$TAG.prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
head -4 $R/gpurun_out/$TAG.prof/run_kernel_stats.csv
