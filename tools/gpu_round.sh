# Full round check on one GPU: all GPU tests (incl. slow), smoke, default bench (with CPU baseline),
# rocprofv3 kernel stats of the bench, FETCH/WRITE PMC passes of the blind rotation.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/$TAG.gpu_tests.log 2>&1; rc=$?; echo "pytest exit $rc" >> gpurun_out/$TAG.gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG.smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/$TAG.bench.log 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG.prof -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/$TAG.prof.log 2>&1 || exit 3
cd $R && bash tools/pmc_br.sh $TAG.pmc
