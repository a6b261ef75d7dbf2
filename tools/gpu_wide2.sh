# Split-transform latency form: its parity tests, then the 16-bit adder (config 3)
# with the split form and the round-3 form in alternation.  bash tools/gpu_wide2.sh TAG [rounds]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-wide2}
N=${2:-2}
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_circuit.py -x -q --timeout 200 --timeout-method thread -k "wide or adder or latency or options or ragged" > gpurun_out/$TAG.tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/$TAG.tests.log; exit 1; }
tail -2 gpurun_out/$TAG.tests.log
for r in $(seq 1 $N); do
  for f in wide wide2; do
    timeout -k 10 200 python bench.py --workload adder --batch 1 --steps 5 --warmup 1 --no-cpu-baseline --opt br_form=$f > gpurun_out/${TAG}_$f$r.json 2> gpurun_out/${TAG}_$f$r.err || { echo "$f bench failed"; tail -5 gpurun_out/${TAG}_$f$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d.get('ms_per_step'), d.get('config',{}).get('workload','')[:60])" gpurun_out/${TAG}_$f$r.json "$f r$r"
  done
done
