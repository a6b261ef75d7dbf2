# Whole form with loader waves (TFHE_BR_LOADER=1) vs without: parity tests, then alternating benches
set -o pipefail
cd $GRAFT_REPO_ROOT
TFHE_BR_LOADER=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_circuit.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/loader_tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in 0 1; do
    TFHE_BR_LOADER=$v timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/loader_b$v.$r.log 2>&1 || exit 1
    echo "loader=$v run $r $(grep -o '"value": [0-9.]*' gpurun_out/loader_b$v.$r.log | head -1) $(grep -o '"kernel_avg_ms": [0-9.]*' gpurun_out/loader_b$v.$r.log)"
  done
done
