# Alternating timing of the product default against A/B-library forms (tools/bin/lib_ab.so,
# TFHE_OPT_BR_FORM n) on the 1,024-gate NAND bench line.   bash tools/gpu_ab_dev.sh ROUNDS FORM...
set -o pipefail
R=$GRAFT_REPO_ROOT
N=$1; shift
cd $R
AB="env TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$R/tools/bin/lib_ab.so"
line() { python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['kernel'].split(' (')[0], d['decrypt_check'], d['margin_guard']['recomputed_items'])" "$1"; }
for r in $(seq $N); do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 2>/dev/null | line "product" || exit 2
  for f in "$@"; do
    timeout -k 10 200 $AB python bench.py --no-cpu-baseline --steps 30 --opt br_form=$f 2>/dev/null | line "form $f" || exit 2
  done
done
