# Alternating timing of library builds x option sets: tools/ab_libs_opts.sh ROUNDS "lib1 lib2" "opts1" "opts2" ...
# (tools/bin/lib_<name>.so; options are bench.py arguments, e.g. "--opt br_form=pair")
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$1; LIBS=$2; shift 2
for r in $(seq 1 $R); do
  for v in $LIBS; do
    for o in "$@"; do
      TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$PWD/tools/bin/lib_$v.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $o > gpurun_out/abl.json 2> gpurun_out/abl.err || { echo "$v [$o] failed"; tail -5 gpurun_out/abl.err; exit 1; }
      python -c "import json,sys; d=json.loads(open('gpurun_out/abl.json').read().splitlines()[-1]); print(sys.argv[1], d['value'], d['roofline']['kernel_avg_ms'], d['roofline']['kernel'])" "$v r$r [$o]"
    done
  done
done
