# gemm key switch at basebit 5 (UINT4): tests, LUT 4,096 ring vs gemm
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_proxy_reenc.py -m gpu -x -q --timeout 120 --timeout-method thread -k "key_switch or reenc or options or lut" > gpurun_out/ksg4_tests.txt 2>&1 || { tail -30 gpurun_out/ksg4_tests.txt; exit 1; }
tail -1 gpurun_out/ksg4_tests.txt
for r in 1 2; do for f in 0 2; do
  timeout -k 10 200 python bench.py --workload lut --batch 4096 --steps 6 --warmup 2 --no-cpu-baseline --opt ks_form=$f > gpurun_out/ksg4_lut_$f$r.json 2> gpurun_out/ksg4.err || { echo "lut $f failed"; tail -5 gpurun_out/ksg4.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['decrypt_check'], d['kernels'])" gpurun_out/ksg4_lut_$f$r.json "lut4096 ks_form=$f r$r"
done; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ksg4.prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload lut --batch 4096 --steps 4 --warmup 1 --no-cpu-baseline --opt ks_form=2 > $GRAFT_REPO_ROOT/gpurun_out/ksg4.prof.log 2>&1 || exit 2
grep -E "key_switch|reduce|ksk_to|blind" $GRAFT_REPO_ROOT/gpurun_out/ksg4.prof/run_kernel_stats.csv | cut -c1-160
