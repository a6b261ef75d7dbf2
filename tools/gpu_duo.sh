# Duo-form iteration: its parity tests, then the NAND batch on the whole and
# duo forms in alternation.  bash tools/gpu_duo.sh TAG [rounds]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-duo}
N=${2:-2}
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "duo" > gpurun_out/$TAG.tests.log 2>&1 || { echo "duo tests failed"; tail -40 gpurun_out/$TAG.tests.log; exit 1; }
tail -2 gpurun_out/$TAG.tests.log
for r in $(seq 1 $N); do
  for f in whole duo; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --opt br_form=$f > gpurun_out/${TAG}_$f$r.json 2> gpurun_out/${TAG}_$f$r.err || { echo "$f bench failed"; tail -5 gpurun_out/${TAG}_$f$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_avg_ms'], d['roofline']['kernel'], d['decrypt_check'], d['margin_guard']['recomputed_items'])" gpurun_out/${TAG}_$f$r.json "$f r$r"
  done
done
