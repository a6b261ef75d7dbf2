# Round-5 per-process rehearsal of the driver's 8-GPU SCALE run on the one card: bench.py
# --gpus 8 over gloo (8 ranks share device 0), for config 2 (NAND), config 4 (65,536 mixed
# gates, strong scaling) and config 5 (4,096 UINT4 LUTs, strong scaling).
#   bash tools/gpu_r05b.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r05b}
cd $R
mkdir -p gpurun_out
for w in "nand" "mixed --global-batch 65536" "lut --global-batch 4096"; do
  set -- $w
  timeout -k 10 400 python bench.py --gpus 8 --dist-backend gloo --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG.gloo8_$1.json 2> gpurun_out/$TAG.gloo8_$1.err || { echo "gloo 8 $w failed"; tail -30 gpurun_out/$TAG.gloo8_$1.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['n_gpus'], d['value'], d['ms_per_step'], d.get('decrypt_check', d.get('sums_check')), d['scaling'])" gpurun_out/$TAG.gloo8_$1.json $1
done
