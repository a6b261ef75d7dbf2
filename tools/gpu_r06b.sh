# Round 6: half-wave pair layout A/B and the 1/8 guard's recompute rate
# (item 3), plus the new product GPU tests.  Libraries built on the CPU beforehand:
# tools/bin/lib_ab_hw.so (tools/ab_forms.sh, NAME=hw), tools/bin/lib_ab_g8.so (-DTFHE_GUARD_EIGHTH).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06b}
cd $R
mkdir -p gpurun_out
AB="env TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$R/tools/bin/lib_ab_hw.so"
G8="env TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$R/tools/bin/lib_ab_g8.so"
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_multi_device.py::test_host_staging_modes_same_words tests/test_gpu_parity.py::test_worst_admitted_key_under_the_product_guard > gpurun_out/$TAG.newtests.log 2>&1 || { tail -30 gpurun_out/$TAG.newtests.log; exit 1; }
tail -1 gpurun_out/$TAG.newtests.log
for f in 26 27; do
  timeout -k 10 300 $AB FORM=$f python tools/ab_assist_check.py parity > gpurun_out/$TAG.parity$f.log 2>&1 || { echo "form $f parity failed"; tail -20 gpurun_out/$TAG.parity$f.log; exit 2; }
  echo "form $f: $(tail -2 gpurun_out/$TAG.parity$f.log | head -1)"
done
for r in 1 2 3; do for f in 9 26 27 19; do
  timeout -k 10 200 $AB BR_FORM=$f python tools/ab_assist_check.py time 40 2>/dev/null | tail -1 | cut -c1-110 || exit 3
done; done | tee gpurun_out/$TAG.hw_ab.txt
timeout -k 10 600 python tools/guard_rate.py 150 > gpurun_out/$TAG.guard4.json 2>gpurun_out/$TAG.guard.err || { tail gpurun_out/$TAG.guard.err; exit 4; }
cat gpurun_out/$TAG.guard4.json
timeout -k 10 600 $G8 python tools/guard_rate.py 150 > gpurun_out/$TAG.guard8.json 2>>gpurun_out/$TAG.guard.err || { tail gpurun_out/$TAG.guard.err; exit 4; }
cat gpurun_out/$TAG.guard8.json
timeout -k 10 300 $G8 python -u -m pytest -q -x --timeout 200 --timeout-method thread -s tests/test_gpu_parity.py::test_worst_admitted_key_under_the_product_guard tests/test_gpu_parity.py::test_margin_guard_recomputes_near_ties > gpurun_out/$TAG.g8tests.log 2>&1 || { tail -30 gpurun_out/$TAG.g8tests.log; exit 5; }
grep -E "worst admitted|passed|failed" gpurun_out/$TAG.g8tests.log
# the latency form with row counters (A/B form 30): parity, then the 16-bit adder alternating
timeout -k 10 300 $AB FORM=30 python tools/ab_assist_check.py parity > gpurun_out/$TAG.parity30.log 2>&1 || { echo "form 30 parity failed"; tail -20 gpurun_out/$TAG.parity30.log; exit 6; }
echo "form 30: $(tail -2 gpurun_out/$TAG.parity30.log | head -1)"
for r in 1 2 3; do for f in 0 30; do
  timeout -k 10 300 $AB python bench.py --workload adder --batch 1 --steps 5 --warmup 1 --opt br_form=$f > gpurun_out/$TAG.adder_f${f}_$r.json 2>gpurun_out/$TAG.adder.err || { tail -5 gpurun_out/$TAG.adder.err; exit 7; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('adder form', sys.argv[2], d['ms_per_step'], d['sums_check'], d['kernels'])" gpurun_out/$TAG.adder_f${f}_$r.json $f
done; done | tee gpurun_out/$TAG.adder_ab.txt
