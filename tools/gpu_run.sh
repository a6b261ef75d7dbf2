# One parametrised GPU-box script for the round's measurements (replaces the per-round
# tools/gpu_r0x*.sh one-offs).  Every step has its own time limit; the first failing step
# ends the call (nothing more runs on the GPU after a fault, abort or timeout).
#   bash tools/gpu_run.sh TAG step[,step...]
# steps:
#   tests     pytest -m gpu (whole suite)          smoke   __graft_entry__.smoke()
#   prof      rocprofv3 --kernel-trace --stats of a 50-step bench -> rocprof record (warm-up
#             excluded by position) + the blind-rotation PMC passes (with the GRBM clock pass)
#   clock     tools/bin/clock_probe (core clock per wave, no phase marks) -> clock-probe record
#   bench     the default bench line (CPU baseline included), with the records just measured
#   bench2k   a 2,048-gate line                    arith1  the headline config under --opt arith=1
#   copy      tools/bin/copy_bw (host copy rates, per-shard staging)
#   sp8       single-process 8 shards on device 0, host_staging 0 / 1 alternating (3 rounds each)
#   wl        BASELINE configs 3-5 + re-encryption workload lines
#   adder     config 3 (one 16-bit adder) only     hp      single-process one-device host path
# Everything lands under gpurun_out/<TAG>*; copy what is judged into profiles/.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:?tag}
STEPS=${2:-tests,smoke,prof,bench}
cd $R
mkdir -p gpurun_out
last() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], *[d.get(k) for k in sys.argv[3:]])" "$@"; }
for S in ${STEPS//,/ }; do
  echo "== $S"
  case $S in
  tests)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/$TAG.gpu_tests.log 2>&1 || { tail -40 gpurun_out/$TAG.gpu_tests.log; exit 1; }
    tail -1 gpurun_out/$TAG.gpu_tests.log ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG.smoke.log 2>&1 || { tail gpurun_out/$TAG.smoke.log; exit 1; }
    cat gpurun_out/$TAG.smoke.log ;;
  prof)
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG.prof -o run -- python3 $R/bench.py --steps 50 --warmup 3 --no-cpu-baseline > $R/gpurun_out/$TAG.prof.log 2>&1 ) || exit 3
    ks=$(find gpurun_out/$TAG.prof -name run_kernel_stats.csv -print -quit)
    kt=$(find gpurun_out/$TAG.prof -name run_kernel_trace.csv -print -quit)
    [ -n "$ks" ] && [ -n "$kt" ] || { echo "no kernel stats / trace"; exit 3; }
    cp "$ks" gpurun_out/${TAG}_kernel_stats.csv
    python tools/trace_excerpt.py "$kt" gpurun_out/${TAG}_kernel_trace_br.csv || exit 3
    python tools/rocprof_record.py gpurun_out/${TAG}_kernel_stats.csv gpurun_out/${TAG}_rocprof_blind_rotate.json gpurun_out/${TAG}_kernel_trace_br.csv 3 || exit 3
    bash tools/pmc_br.sh $TAG.pmc 1024 "" gpurun_out/${TAG}_pmc_blind_rotate.json || exit 4
    cp gpurun_out/${TAG}_rocprof_blind_rotate.json profiles/rocprof_blind_rotate.json
    cp gpurun_out/${TAG}_pmc_blind_rotate.json profiles/pmc_blind_rotate.json ;;
  clock)
    timeout -k 10 120 tools/bin/clock_probe 1024 whole > gpurun_out/$TAG.clock_probe.txt 2>&1 || { tail gpurun_out/$TAG.clock_probe.txt; exit 1; }
    python tools/clock_probe_record.py gpurun_out/$TAG.clock_probe.txt --out gpurun_out/${TAG}_clock_probe.json || exit 1
    cp gpurun_out/${TAG}_clock_probe.json profiles/clock_probe.json ;;
  bench)
    timeout -k 10 600 python bench.py > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || { tail gpurun_out/$TAG.bench.err; exit 2; }
    last gpurun_out/$TAG.bench.json bench value ms_per_step ;;
  bench2k)
    timeout -k 10 300 python bench.py --no-cpu-baseline --batch 2048 --steps 25 > gpurun_out/$TAG.bench2048.json 2> gpurun_out/$TAG.bench.err || { tail gpurun_out/$TAG.bench.err; exit 2; }
    last gpurun_out/$TAG.bench2048.json bench2048 value ms_per_step ;;
  arith1)
    timeout -k 10 600 python bench.py --opt arith=1 --steps 20 --cpu-seconds 5 > gpurun_out/$TAG.arith1.json 2> gpurun_out/$TAG.arith1.err || { tail gpurun_out/$TAG.arith1.err; exit 2; }
    last gpurun_out/$TAG.arith1.json arith1 value ms_per_step decrypt_check ;;
  copy)
    timeout -k 10 200 tools/bin/copy_bw > gpurun_out/$TAG.copy_bw.txt 2>&1 || { tail gpurun_out/$TAG.copy_bw.txt; exit 6; }
    tail -12 gpurun_out/$TAG.copy_bw.txt ;;
  sp8)
    for r in 1 2 3; do for st in 0 1; do
      timeout -k 10 300 python bench.py --single-process --gpus 8 --devices 0,0,0,0,0,0,0,0 --steps 5 --warmup 1 --no-cpu-baseline --opt host_staging=$st > gpurun_out/$TAG.sp8_st${st}_$r.json 2> gpurun_out/$TAG.sp8.err || { tail gpurun_out/$TAG.sp8.err; exit 7; }
      last gpurun_out/$TAG.sp8_st${st}_$r.json "sp8 staging=$st" value ms_per_step words_equal_one_device
    done; done ;;
  wl)
    for w in "adder 1 5" "adder 256 3" "mixed 65536 3" "lut 4096 8" "reenc 16384 8"; do
      set -- $w
      timeout -k 10 300 python bench.py --workload $1 --batch $2 --steps $3 --warmup 1 > gpurun_out/$TAG.wl_$1_$2.json 2> gpurun_out/$TAG.wl.err || { echo "workload $w failed"; tail -5 gpurun_out/$TAG.wl.err; exit 5; }
      last gpurun_out/$TAG.wl_$1_$2.json "$w" value unit ms_per_step decrypt_check
    done ;;
  adder)
    timeout -k 10 300 python bench.py --workload adder --batch 1 --steps 5 --warmup 1 > gpurun_out/$TAG.wl_adder_1.json 2> gpurun_out/$TAG.wl.err || { tail -5 gpurun_out/$TAG.wl.err; exit 5; }
    last gpurun_out/$TAG.wl_adder_1.json adder value ms_per_step sums_check ;;
  hp)
    timeout -k 10 200 python bench.py --single-process --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG.single_process.json 2>/dev/null || exit 6
    last gpurun_out/$TAG.single_process.json single-process value ms_per_step ;;
  *) echo "unknown step $S"; exit 9 ;;
  esac
done
