# Parity (tools/ab_assist_check.py parity: oracle, round 4's whole form at every idle-slot count,
# 1,024 mixed gates) of A/B-library forms, then their alternating timing against the product.
#   bash tools/gpu_ab_dev_parity.sh ROUNDS FORM...
set -o pipefail
R=$GRAFT_REPO_ROOT
N=$1; shift
cd $R
mkdir -p gpurun_out
for f in "$@"; do
  timeout -k 10 150 env TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$R/tools/bin/lib_ab.so FORM=$f python tools/ab_assist_check.py parity > gpurun_out/dev$f.parity.log 2>&1 || { echo "form $f parity failed"; tail -20 gpurun_out/dev$f.parity.log; exit 1; }
  echo "form $f: $(grep -c "" gpurun_out/dev$f.parity.log) lines, $(grep -v amdgpu.ids gpurun_out/dev$f.parity.log | tr '\n' ' ' | cut -c1-300)"
done
bash tools/gpu_ab_dev.sh $N "$@"
