# Round-3 measurement set: GPU tests, smoke, default bench (CPU baseline), rocprofv3 kernel stats,
# blind-rotation PMC passes, BASELINE configs 3-5 workload lines, single-process host path.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03j}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/$TAG.gpu_tests.log 2>&1 || { tail -30 gpurun_out/$TAG.gpu_tests.log; exit 1; }
tail -1 gpurun_out/$TAG.gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG.smoke.log 2>&1 || { tail gpurun_out/$TAG.smoke.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || { tail gpurun_out/$TAG.bench.err; exit 2; }
tail -1 gpurun_out/$TAG.bench.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG.prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/$TAG.prof.log 2>&1 || exit 3
cd $R && bash tools/pmc_br.sh $TAG.pmc 1024 "" gpurun_out/$TAG.pmc_blind_rotate.json || exit 4
for w in "adder 1 3" "adder 256 3" "mixed 65536 3" "lut 4096 8" "reenc 16384 8"; do
  set -- $w
  timeout -k 10 300 python bench.py --workload $1 --batch $2 --steps $3 --warmup 1 > gpurun_out/$TAG.wl_$1_$2.json 2> gpurun_out/$TAG.wl.err || { echo "workload $w failed"; tail -5 gpurun_out/$TAG.wl.err; exit 5; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'], d.get('decrypt_check'))" gpurun_out/$TAG.wl_$1_$2.json "$w"
done
timeout -k 10 200 python bench.py --single-process --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG.single_process.json 2>/dev/null || exit 6
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('single-process', d['value'], d['ms_per_step'])" gpurun_out/$TAG.single_process.json
