# Round-5 measurement set: GPU tests, smoke, rocprofv3 kernel stats of a 50-step bench,
# blind-rotation PMC passes, then the default bench (CPU baseline) with both records in
# place, BASELINE configs 3-5 workload lines and the single-process host path.
# Everything lands under gpurun_out/<TAG>*; copy what is judged into profiles/.
#   bash tools/gpu_r05_final.sh TAG [skip_tests]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r05f}
cd $R
mkdir -p gpurun_out
if [ -z "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.gpu_tests.log 2>&1 || { tail -30 gpurun_out/$TAG.gpu_tests.log; exit 1; }
  tail -1 gpurun_out/$TAG.gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG.smoke.log 2>&1 || { tail gpurun_out/$TAG.smoke.log; exit 1; }
  cat gpurun_out/$TAG.smoke.log
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG.prof -o run -- python3 $R/bench.py --steps 50 --warmup 3 --no-cpu-baseline > $R/gpurun_out/$TAG.prof.log 2>&1 || exit 3
cd $R
ks=$(find gpurun_out/$TAG.prof -name run_kernel_stats.csv -print -quit)
[ -n "$ks" ] || { echo "no kernel stats"; exit 3; }
cp "$ks" gpurun_out/${TAG}_kernel_stats.csv
python tools/rocprof_record.py gpurun_out/${TAG}_kernel_stats.csv gpurun_out/${TAG}_rocprof_blind_rotate.json || exit 3
bash tools/pmc_br.sh $TAG.pmc 1024 "" gpurun_out/${TAG}_pmc_blind_rotate.json || exit 4
# the bench reads its records from profiles/: point it at this build's files for the default line
cp gpurun_out/${TAG}_rocprof_blind_rotate.json profiles/rocprof_blind_rotate.json
cp gpurun_out/${TAG}_pmc_blind_rotate.json profiles/pmc_blind_rotate.json
timeout -k 10 600 python bench.py > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || { tail gpurun_out/$TAG.bench.err; exit 2; }
tail -1 gpurun_out/$TAG.bench.json | cut -c1-300
timeout -k 10 300 python bench.py --no-cpu-baseline --batch 2048 --steps 25 > gpurun_out/$TAG.bench2048.json 2> gpurun_out/$TAG.bench.err || { tail gpurun_out/$TAG.bench.err; exit 2; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench 2048', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])" gpurun_out/$TAG.bench2048.json
for w in "adder 1 5" "adder 256 3" "mixed 65536 3" "lut 4096 8" "reenc 16384 8"; do
  set -- $w
  timeout -k 10 300 python bench.py --workload $1 --batch $2 --steps $3 --warmup 1 > gpurun_out/$TAG.wl_$1_$2.json 2> gpurun_out/$TAG.wl.err || { echo "workload $w failed"; tail -5 gpurun_out/$TAG.wl.err; exit 5; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'], d.get('decrypt_check'))" gpurun_out/$TAG.wl_$1_$2.json "$w"
done
timeout -k 10 200 python bench.py --single-process --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG.single_process.json 2>/dev/null || exit 6
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('single-process', d['value'], d['ms_per_step'])" gpurun_out/$TAG.single_process.json
