# flipped-digit tmp words: full GPU tests, A/B vs the previous build, L=1 octo dispatch by batch
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03g_tests.txt 2>&1 || { tail -40 gpurun_out/r03g_tests.txt; exit 1; }
tail -2 gpurun_out/r03g_tests.txt
bash tools/gpu_ab_libs.sh r03g 3 prev flip || exit 1
for b in 1024 2048 2348 3548 4096 8192; do
  for f in auto whole; do
    o=""; [ $f = whole ] && o="--opt br_form=whole"
    timeout -k 10 200 python bench.py --workload lut --batch $b --steps 5 --warmup 1 --no-cpu-baseline $o > gpurun_out/r03g_lut_${f}_$b.json 2> gpurun_out/r03g.err || { echo "lut $f $b failed"; tail -5 gpurun_out/r03g.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['decrypt_check'], d['kernels'][:40])" gpurun_out/r03g_lut_${f}_$b.json "lut $b $f"
  done
done
