# dispatch plans (blind_rotate_plan): full GPU tests, UINT4 LUT batches auto and forced forms
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03h_tests.txt 2>&1 || { tail -40 gpurun_out/r03h_tests.txt; exit 1; }
tail -2 gpurun_out/r03h_tests.txt
run() {  # batch form
  o=""; [ $2 != auto ] && o="--opt br_form=$2"
  timeout -k 10 200 python bench.py --workload lut --batch $1 --steps 5 --warmup 1 --no-cpu-baseline $o > gpurun_out/r03h_lut_$2_$1.json 2> gpurun_out/r03h.err || { echo "lut $2 $1 failed"; tail -5 gpurun_out/r03h.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['decrypt_check'], d['kernels'][:44])" gpurun_out/r03h_lut_$2_$1.json "lut $1 $2"
}
run 256 wide && run 256 whole && run 512 wide && run 512 whole && run 768 wide && \
for b in 256 512 1024 2048 2348 3548 4096 8192; do run $b auto || exit 1; done
