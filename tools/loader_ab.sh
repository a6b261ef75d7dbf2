# Whole form with loader waves (--opt br_loader=1) vs without: parity tests, then alternating benches
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_circuit.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/loader_tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --opt br_loader=$v > gpurun_out/loader_b$v.$r.log 2>&1 || exit 1
    echo "loader=$v run $r $(grep -o '"value": [0-9.]*' gpurun_out/loader_b$v.$r.log | head -1) $(grep -o '"kernel_avg_ms": [0-9.]*' gpurun_out/loader_b$v.$r.log)"
  done
done
