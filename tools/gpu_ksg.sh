# gemm key switch: parity tests, then alternating bench A/B (lanes vs gemm), LUT untouched
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "key_switch" > gpurun_out/ksg_tests.txt 2>&1 || { tail -30 gpurun_out/ksg_tests.txt; exit 1; }
tail -1 gpurun_out/ksg_tests.txt
for r in 1 2 3; do
  for f in 0 2; do
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --opt ks_form=$f > gpurun_out/ksg_$f$r.json 2> gpurun_out/ksg.err || { echo "bench ks_form=$f failed"; tail -5 gpurun_out/ksg.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_avg_ms'], d['key_switch'], d['decrypt_check'])" gpurun_out/ksg_$f$r.json "ks_form=$f r$r"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ksg.prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --opt ks_form=2 > $GRAFT_REPO_ROOT/gpurun_out/ksg.prof.log 2>&1 || exit 2
grep -E "key_switch|reduce|ksk_to" $GRAFT_REPO_ROOT/gpurun_out/ksg.prof/run_kernel_stats.csv | cut -c1-200
