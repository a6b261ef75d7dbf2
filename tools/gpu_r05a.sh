# Round-5 check after the product/A-B split: GPU tests, smoke, the default bench (timed region
# without per-launch events) at 1,024 and 2,048 gates, and the single-process 8-shard rehearsals
# (device 0 listed eight times) of configs 2, 4 (components and forced level split) and 5.
#   bash tools/gpu_r05a.sh TAG [skip_tests]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r05a}
cd $R
mkdir -p gpurun_out
if [ -z "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG.gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/$TAG.gpu_tests.log; exit 1; }
  tail -2 gpurun_out/$TAG.gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG.smoke.log 2>&1 || { tail gpurun_out/$TAG.smoke.log; exit 1; }
  cat gpurun_out/$TAG.smoke.log
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || { echo "bench failed"; tail -20 gpurun_out/$TAG.bench.err; exit 2; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['decrypt_check'])" gpurun_out/$TAG.bench.json
timeout -k 10 300 python bench.py --no-cpu-baseline --batch 2048 --steps 25 > gpurun_out/$TAG.bench2048.json 2> gpurun_out/$TAG.bench.err || { echo "bench 2048 failed"; tail -20 gpurun_out/$TAG.bench.err; exit 2; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench 2048', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['decrypt_check'])" gpurun_out/$TAG.bench2048.json
D8=0,0,0,0,0,0,0,0
for w in "nand --batch 1024 --steps 5" "mixed --global-batch 65536 --steps 2" "mixed --global-batch 65536 --steps 2 --opt circuit_split=2" "lut --global-batch 4096 --steps 3"; do
  set -- $w
  name=sp8_$1$(echo "$w" | grep -q circuit_split && echo _levels)
  timeout -k 10 400 python bench.py --single-process --gpus 8 --devices $D8 --workload $w --warmup 1 > gpurun_out/$TAG.$name.json 2> gpurun_out/$TAG.sp.err || { echo "single-process $w failed"; tail -20 gpurun_out/$TAG.sp.err; exit 3; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['n_gpus'], d['value'], d['ms_per_step'], d['decrypt_check'], d['words_equal_one_device'], d['bootstraps_per_device_per_step'], d.get('level_issue_us'))" gpurun_out/$TAG.$name.json $name
done
