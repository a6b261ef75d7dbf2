# Knock-out timing (tools/ko_libs.sh builds; wrong results by design): bash tools/ko_bench.sh [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
for f in tools/bin/libko_*.so; do
  TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$PWD/$f timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/ko_b.log 2>&1 || exit 1
  echo "$f $* $(grep -o '"kernel_avg_ms": [0-9.]*' gpurun_out/ko_b.log)"
done
