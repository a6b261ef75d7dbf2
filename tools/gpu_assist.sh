# A/B of whole-form variants built as tools/bin/lib_ab_<variant>.so (tools/ab_forms.sh NAME=...):
# parity of the first variant's whole form against round 4's (A/B form 8 "plain") and the oracle
# (bounded waits), then alternating timing of every variant's whole form against the product
# library's default.  (Round 5 used it for the loader-assist form before it became the default.)
#   bash tools/gpu_assist.sh TAG ROUNDS VARIANT...
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; N=$2; shift 2
cd $R
mkdir -p gpurun_out
ab() { echo "env TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$R/tools/bin/lib_ab_$1.so"; }
timeout -k 10 120 $(ab $1) python tools/ab_assist_check.py parity > gpurun_out/$TAG.parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/$TAG.parity.log; exit 1; }
grep -v amdgpu.ids gpurun_out/$TAG.parity.log
for r in $(seq $N); do
  timeout -k 10 120 python tools/ab_assist_check.py time 40 2>/dev/null | tail -1 | cut -c1-90 || exit 2
  for v in "$@"; do
    echo -n "$v: "; timeout -k 10 120 env BR_FORM=whole $(ab $v) python tools/ab_assist_check.py time 40 2>/dev/null | tail -1 | cut -c1-90 || exit 2
  done
done
# phase profiles (s_memtime marks; tools/phase_prof.hip built with -DTFHE_PHASE_PROF)
if [ -x tools/bin/phase_prof ] && [ -z "$NOPROF" ]; then
  timeout -k 10 120 tools/bin/phase_prof 1024 whole 2>&1 | tail -16
  timeout -k 10 120 tools/bin/phase_prof 1024 assist 2>&1 | tail -16
fi
