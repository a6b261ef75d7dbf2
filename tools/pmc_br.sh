# rocprofv3 --pmc passes over br_only.py (one B=1024 NAND batch), one counter
# group per pass (gfx950 block limits: <= 8 SQ, FETCH_SIZE alone, WRITE_SIZE alone).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-pmc_br}
B=${2:-1024}
FORM=${3:-}
cd /tmp && export TMPDIR=/tmp
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $R/gpurun_out/$TAG/p$i -o run -- python3 $R/tools/br_only.py $B 1 $FORM > $R/gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i ($CTRS) failed"; exit 1; }
done
# clock pass: GRBM_GUI_ACTIVE (summed over the 8 XCDs) with the dispatch's own duration from the
# kernel trace of the same run -> effective clock = GRBM_GUI_ACTIVE / 8 / duration (MI355X_MICROARCH.md, DVFS);
# four launches, the first (cold: code-object load, caches) excluded
i=$((i+1))
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $R/gpurun_out/$TAG/p$i -o run -- python3 $R/tools/br_only.py $B 4 $FORM > $R/gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i (GRBM clock) failed"; exit 1; }
cd $R && python3 tools/pmc_traffic.py gpurun_out/$TAG $B 128 ${4:-profiles/pmc_blind_rotate.json} > gpurun_out/${TAG}_summary.json
