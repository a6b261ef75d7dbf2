# latency form: flipped-digit A/B on the 16-bit adder (config 3), after the form's parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_circuit.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wide or blind_rotate or margin or adder or circuit" > gpurun_out/wide_tests.txt 2>&1 || { tail -30 gpurun_out/wide_tests.txt; exit 1; }
tail -1 gpurun_out/wide_tests.txt
for r in 1 2 3; do for v in widebase wideflip; do
  TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$PWD/tools/bin/lib_$v.so timeout -k 10 200 python bench.py --workload adder --batch 1 --steps 4 --warmup 1 > gpurun_out/wide_$v$r.json 2> gpurun_out/wide.err || { echo "$v failed"; tail -5 gpurun_out/wide.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/wide_$v$r.json "$v r$r"
done; done
