# Alternating timing of several library builds: tools/ab_multi.sh name1 name2 ... (tools/bin/lib_<name>.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for v in "$@"; do
    TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$PWD/tools/bin/lib_$v.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/abm_$v$r.log 2>&1 || exit 1
    echo "$v $(grep -o '"kernel_avg_ms": [0-9.]*' gpurun_out/abm_$v$r.log) $(grep -o '"value": [0-9.]*' gpurun_out/abm_$v$r.log)"
  done
done
