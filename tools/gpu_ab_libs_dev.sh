# Alternating timing of the product default against A/B libraries and forms given as NAME:FORM
# (tools/bin/lib_ab_NAME.so, or lib_ab.so for NAME "-"), 1,024-gate NAND line.
#   bash tools/gpu_ab_libs_dev.sh ROUNDS NAME:FORM...
set -o pipefail
R=$GRAFT_REPO_ROOT
N=$1; shift
cd $R
line() { python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['kernel'].split(' (')[0], d['decrypt_check'], d['margin_guard']['recomputed_items'])" "$1"; }
for r in $(seq $N); do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 2>/dev/null | line "product" || exit 2
  for e in "$@"; do
    name=${e%%:*}; f=${e##*:}
    lib=$R/tools/bin/lib_ab${name/#-/}.so; [ "$name" = "-" ] || lib=$R/tools/bin/lib_ab_$name.so
    timeout -k 10 200 env TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$lib python bench.py --no-cpu-baseline --steps 30 --opt br_form=$f 2>/dev/null | line "$name:$f" || exit 2
  done
done
