# Round 5, VERDICT r04 item 4: the latency form's PMC (one gate, tools/pmc_br.sh passes) and its
# per-phase timing (tools/bin/phase_prof 1 wide) on the current build.   bash tools/gpu_r05w.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r05w}
cd $R
mkdir -p gpurun_out
bash tools/pmc_br.sh $TAG.pmc 1 wide gpurun_out/${TAG}_pmc_wide.json || exit 1
python -c "import json; d=json.load(open('gpurun_out/${TAG}_pmc_wide.json')); print({k: v for k, v in d.items() if k != 'raw_per_launch'})"
timeout -k 10 120 tools/bin/phase_prof 1 wide > gpurun_out/$TAG.phase_wide.txt 2>&1 || exit 2
tail -16 gpurun_out/$TAG.phase_wide.txt
