# Alternating timing of library builds tools/bin/lib_<name>.so on the NAND batch with
# one blind-rotation form: bash tools/gpu_ab_form.sh TAG ROUNDS FORM name1 name2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; R=$2; F=$3; shift 3
for r in $(seq 1 $R); do
  for v in "$@"; do
    TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$PWD/tools/bin/lib_$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --opt br_form=$F > gpurun_out/${T}_$v$r.json 2> gpurun_out/${T}_$v$r.err || { echo "$v failed"; tail -5 gpurun_out/${T}_$v$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_avg_ms'], d['decrypt_check'])" gpurun_out/${T}_$v$r.json "$v r$r"
  done
done
