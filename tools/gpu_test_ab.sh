# GPU tests (optionally -k EXPR) then an alternating A/B of tools/bin/lib_<name>.so builds.
#   bash tools/gpu_test_ab.sh TAG ROUNDS "pytest -k expr or ''" name1 name2 ...
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; ROUNDS=$2; K=$3; shift 3
cd $R
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${KARG[@]}" > gpurun_out/$TAG.gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/$TAG.gpu_tests.log; exit 1; }
tail -2 gpurun_out/$TAG.gpu_tests.log
[ $# -gt 0 ] && bash tools/gpu_ab_libs.sh $TAG $ROUNDS "$@"
exit 0
