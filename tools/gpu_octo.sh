# Octo form vs whole form: device-resident NAND batches (128-bit) of 2,048 / 4,096 / 8,192 and the
# UINT4 LUT workload at 4,096, alternating.  bash tools/gpu_octo.sh TAG ROUNDS
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-octo}; ROUNDS=${2:-2}
cd $R
for r in $(seq 1 $ROUNDS); do
  for B in 2048 4096 8192; do
    for f in whole octo; do
      timeout -k 10 200 python bench.py --batch $B --steps 6 --warmup 1 --no-cpu-baseline --opt br_form=$f > gpurun_out/${TAG}_${f}_$B_$r.json 2> gpurun_out/${TAG}.err || { echo "bench $f $B failed"; tail -5 gpurun_out/${TAG}.err; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_avg_ms'], d['decrypt_check'], d['margin_guard']['recomputed_items'])" gpurun_out/${TAG}_${f}_$B_$r.json "r$r B=$B $f"
    done
  done
  for f in whole octo; do
    timeout -k 10 200 python bench.py --workload lut --batch 4096 --steps 6 --warmup 1 --opt br_form=$f > gpurun_out/${TAG}_lut_${f}_$r.json 2> gpurun_out/${TAG}.err || { echo "lut $f failed"; tail -5 gpurun_out/${TAG}.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['decrypt_check'], d['kernels'])" gpurun_out/${TAG}_lut_${f}_$r.json "r$r lut4096 $f"
  done
done
