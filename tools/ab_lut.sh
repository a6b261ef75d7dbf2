# Alternating timing of library builds on the UINT4 LUT workload (BASELINE config 5):
#   bash tools/ab_lut.sh ROUNDS "lib1 lib2"   (tools/bin/lib_<name>.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$1; LIBS=$2
for r in $(seq 1 $R); do
  for v in $LIBS; do
    TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$PWD/tools/bin/lib_$v.so timeout -k 10 200 python bench.py --workload lut --batch 4096 --steps 5 --warmup 1 > gpurun_out/abl.json 2> gpurun_out/abl.err || { echo "$v failed"; tail -5 gpurun_out/abl.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/abl.json').read().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['kernels'], d['decrypt_check'])" "$v r$r"
  done
done
