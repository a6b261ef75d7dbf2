# Round 6: phase profiles and PMC of the half-wave layout (A/B VAR 18 = form 27) against the
# control copy (VAR 0 = form 9), phase profiles of the latency form with and without row counters,
# and the worst admitted key's recompute count under the product guard.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06c}
cd $R
mkdir -p gpurun_out
for f in dev0 dev18 dev17 wide widerc; do
  timeout -k 10 120 tools/bin/phase_prof 1024 $f > gpurun_out/$TAG.phase_$f.txt 2>&1 || { echo "phase $f failed"; tail gpurun_out/$TAG.phase_$f.txt; exit 1; }
  echo "== $f"; tail -n +$(grep -n "rep 1" gpurun_out/$TAG.phase_$f.txt | cut -d: -f1) gpurun_out/$TAG.phase_$f.txt
done
export TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$R/tools/bin/lib_ab_hw.so
for f in 9 27; do
  bash tools/pmc_br.sh $TAG.pmc$f 1024 $f gpurun_out/${TAG}_pmc_form$f.json > /dev/null || exit 2
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['raw_per_launch']; print('form', sys.argv[2], 'VALU/item/CMUX', d['valu_insts_per_item_per_cmux'], 'LDS', d['lds_insts_per_item_per_cmux'], 'bank conflicts', r.get('SQ_LDS_BANK_CONFLICT'), 'wait_inst_lds', round(r['SQ_WAIT_INST_LDS']/r['SQ_WAVE_CYCLES'],4), 'clock', d.get('clock_ghz'))" gpurun_out/${TAG}_pmc_form$f.json $f
done
unset TFHE_ALLOW_AB_BUILD TFHE_GPU_LIB
timeout -k 10 300 python -u -m pytest -q -x -s --timeout 200 --timeout-method thread tests/test_gpu_parity.py::test_worst_admitted_key_under_the_product_guard > gpurun_out/$TAG.worst.log 2>&1 || { tail -20 gpurun_out/$TAG.worst.log; exit 3; }
grep -E "worst admitted|passed" gpurun_out/$TAG.worst.log
