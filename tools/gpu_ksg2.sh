# gemm vs lane key switch by batch (bench's key_switch avg_ms), then the GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 64 128 256 512 1024 4096; do
  for f in 0 2; do
    timeout -k 10 200 python bench.py --batch $b --steps 6 --warmup 2 --no-cpu-baseline --opt ks_form=$f > gpurun_out/ksb_${f}_$b.json 2> gpurun_out/ksb.err || { echo "bench $b $f failed"; tail -5 gpurun_out/ksb.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['key_switch'], d['decrypt_check'])" gpurun_out/ksb_${f}_$b.json "B=$b ks_form=$f"
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ksg2_tests.txt 2>&1 || { tail -30 gpurun_out/ksg2_tests.txt; exit 1; }
tail -1 gpurun_out/ksg2_tests.txt
