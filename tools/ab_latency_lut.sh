set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do for v in ldsex regex; do
  TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$PWD/tools/bin/lib_$v.so timeout -k 10 200 python bench.py --workload adder --batch 1 --steps 3 --warmup 1 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v adder1', d['ms_per_adder_circuit'], d['kernels'])" || exit 1
  TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$PWD/tools/bin/lib_$v.so timeout -k 10 200 python bench.py --workload lut --batch 4096 --steps 3 --warmup 1 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v lut', d['value'])" || exit 1
done; done
