# A/B timing of library builds in alternation: bash tools/gpu_ab_libs.sh TAG ROUNDS name1 name2 ...
# (tools/bin/lib_<name>.so, selected through TFHE_GPU_LIB)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; R=$2; shift 2
for r in $(seq 1 $R); do
  for v in "$@"; do
    TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$PWD/tools/bin/lib_$v.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_$v$r.json 2> gpurun_out/${T}_$v$r.err || { echo "$v failed"; tail -5 gpurun_out/${T}_$v$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_avg_ms'], d['key_switch']['avg_ms'], d['decrypt_check'])" gpurun_out/${T}_$v$r.json "$v r$r"
  done
done
