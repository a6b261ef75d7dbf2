# gemm key switch generalised (n_in, t): key-switch + re-encryption tests, reenc workload A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_proxy_reenc.py -m gpu -x -q --timeout 120 --timeout-method thread -k "key_switch or reenc or options" > gpurun_out/ksg3_tests.txt 2>&1 || { tail -30 gpurun_out/ksg3_tests.txt; exit 1; }
tail -1 gpurun_out/ksg3_tests.txt
for f in 0 3; do
  timeout -k 10 200 python bench.py --workload reenc --batch 16384 --steps 8 --warmup 2 --opt ks_form=$f > gpurun_out/ksg3_reenc_$f.json 2> gpurun_out/ksg3.err || { echo "reenc $f failed"; tail -5 gpurun_out/ksg3.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['decrypt_check'])" gpurun_out/ksg3_reenc_$f.json "reenc ks_form=$f"
done
timeout -k 10 200 python bench.py --workload adder --batch 1 --steps 3 --warmup 1 > gpurun_out/ksg3_adder1.json 2> gpurun_out/ksg3.err || exit 1
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('adder1', d['value'], d['ms_per_step'])" gpurun_out/ksg3_adder1.json
