# Round-5 check of the loader-assist default (L = 3 whole form): GPU tests, then alternating
# timing against round 4's whole form (A/B library, TFHE_OPT_BR_FORM 8) at 1,024 NAND (128-bit),
# 1,024 NAND (80-bit) and 4,096 NAND, and the config-4 workload line.   bash tools/gpu_r05c.sh TAG [skip_tests]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r05c}
cd $R
mkdir -p gpurun_out
if [ -z "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG.gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/$TAG.gpu_tests.log; exit 1; }
  tail -1 gpurun_out/$TAG.gpu_tests.log
fi
AB="env TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$R/tools/bin/lib_ab.so"
line() { python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['kernels'].split(' (')[0] if 'kernels' in d else d['roofline']['kernel'].split(' (')[0], d['decrypt_check'])" "$1"; }
for r in 1 2 3; do
  for cfg in "--params 128" "--params 80" "--batch 4096 --steps 12"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 $cfg 2>/dev/null | line "assist $cfg" || exit 2
    timeout -k 10 200 $AB python bench.py --no-cpu-baseline --steps 30 $cfg --opt br_form=8 2>/dev/null | line "plain  $cfg" || exit 2
  done
done
timeout -k 10 300 python bench.py --workload mixed --global-batch 65536 --steps 3 --warmup 1 > gpurun_out/$TAG.wl_mixed.json 2>/dev/null || exit 3
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('mixed 65536', d['value'], d['unit'], d['ms_per_step'], d.get('decrypt_check'))" gpurun_out/$TAG.wl_mixed.json
