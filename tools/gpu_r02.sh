# Round-2 GPU check: GPU tests, smoke, the default bench (CPU baseline), rocprof
# kernel stats of the bench, PMC passes of the blind rotation, and the --gpus 2
# spawn path (gloo, two ranks sharing the one GPU).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r02}
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG.gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/$TAG.gpu_tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG.smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 4 --warmup 1 > gpurun_out/$TAG.bench2.json 2> gpurun_out/$TAG.bench2.err || { echo "bench --gpus 2 failed"; tail -20 gpurun_out/$TAG.bench2.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG.prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/$TAG.prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
cd $R && bash tools/pmc_br.sh $TAG.pmc 1024
