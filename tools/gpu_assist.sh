# A/B of the loader-assist whole form (tools/ab/tfhe_ab_assist.hip, TFHE_OPT_BR_FORM 8 in
# tools/bin/lib_ab.so): parity first (bounded waits), then alternating timing against the
# product library's default whole form.   bash tools/gpu_assist.sh TAG [rounds]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-assist}
N=${2:-3}
cd $R
mkdir -p gpurun_out
AB="env TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$R/tools/bin/lib_ab.so"
timeout -k 10 120 $AB python tools/ab_assist_check.py parity > gpurun_out/$TAG.parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/$TAG.parity.log; exit 1; }
cat gpurun_out/$TAG.parity.log | grep -v amdgpu.ids
for r in $(seq $N); do
  timeout -k 10 120 python tools/ab_assist_check.py time 40 2>/dev/null | tail -1 || exit 2
  timeout -k 10 120 env BR_FORM=assist $AB python tools/ab_assist_check.py time 40 2>/dev/null | tail -1 || exit 2
done
