# guard accumulator A/B, LUT whole vs octo (host path, pipeline off), single-process host path
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_ab_libs.sh r03e 3 noguard guard4 guard || exit 1
for r in 1 2; do
  for f in whole octo; do
    timeout -k 10 200 python bench.py --workload lut --batch 4096 --steps 6 --warmup 1 --opt br_form=$f > gpurun_out/r03e_lut_${f}_$r.json 2> gpurun_out/r03e.err || { echo "lut $f failed"; tail -5 gpurun_out/r03e.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['decrypt_check'])" gpurun_out/r03e_lut_${f}_$r.json "r$r lut4096 $f"
  done
  timeout -k 10 200 python bench.py --single-process --gpus 1 --steps 10 --warmup 2 > gpurun_out/r03e_sp_$r.json 2>/dev/null || { echo "single-process failed"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['decrypt_check'])" gpurun_out/r03e_sp_$r.json "r$r single-process host buffers"
done
