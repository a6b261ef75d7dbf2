# four-chain guard default + L=1 octo dispatch: GPU tests for the touched paths, LUT batches auto vs whole
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lut or blind_rotate or margin_guard or idle_slot" > gpurun_out/r03f_tests.txt 2>&1 || { tail -30 gpurun_out/r03f_tests.txt; exit 1; }
tail -3 gpurun_out/r03f_tests.txt
for b in 1024 2048 2348 3548 4096 8192; do
  for f in auto whole; do
    o=""; [ $f = whole ] && o="--opt br_form=whole"
    timeout -k 10 200 python bench.py --workload lut --batch $b --steps 5 --warmup 1 $o > gpurun_out/r03f_lut_${f}_$b.json 2> gpurun_out/r03f.err || { echo "lut $f $b failed"; tail -5 gpurun_out/r03f.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['decrypt_check'], d['kernels'])" gpurun_out/r03f_lut_${f}_$b.json "lut $b $f"
  done
done
timeout -k 10 200 python bench.py --steps 10 --warmup 2 > gpurun_out/r03f_nand.json 2> gpurun_out/r03f.err || exit 1
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('nand', d['value'], d['ms_per_step'], d['margin_guard'])" gpurun_out/r03f_nand.json
