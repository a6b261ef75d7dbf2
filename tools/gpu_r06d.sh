# Round 6: the row-counter latency form (A/B form 30) against the product latency form at the
# batch sizes the latency form serves: phase profiles at 1 and 256 gates, 256 adders side by
# side (config 3's batch line), and 256 / 512-gate NAND batches; alternating, one call.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06d}
cd $R
mkdir -p gpurun_out
for b in 1 256; do for f in wide widerc; do
  timeout -k 10 120 tools/bin/phase_prof $b $f > gpurun_out/$TAG.phase_${f}_$b.txt 2>&1 || { echo "phase $f $b failed"; tail gpurun_out/$TAG.phase_${f}_$b.txt; exit 1; }
  echo "== $f B=$b"; tail -n +$(grep -n "rep 1" gpurun_out/$TAG.phase_${f}_$b.txt | cut -d: -f1) gpurun_out/$TAG.phase_${f}_$b.txt
done; done
AB="env TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$R/tools/bin/lib_ab_hw.so"
for r in 1 2; do for f in 0 30; do
  timeout -k 10 300 $AB python bench.py --workload adder --batch 256 --steps 3 --warmup 1 --opt br_form=$f > gpurun_out/$TAG.adder256_f${f}_$r.json 2>gpurun_out/$TAG.err || { tail -5 gpurun_out/$TAG.err; exit 2; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('256 adders form', sys.argv[2], d['value'], d['ms_per_step'], d['sums_check'])" gpurun_out/$TAG.adder256_f${f}_$r.json $f
  for b in 256 512; do
    timeout -k 10 300 $AB python bench.py --batch $b --steps 20 --warmup 2 --no-cpu-baseline --opt br_form=$f > gpurun_out/$TAG.nand${b}_f${f}_$r.json 2>gpurun_out/$TAG.err || { tail -5 gpurun_out/$TAG.err; exit 3; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('NAND', sys.argv[2], 'form', sys.argv[3], d['value'], d['ms_per_step'], d['decrypt_check'], d['roofline']['kernel'])" gpurun_out/$TAG.nand${b}_f${f}_$r.json $b $f
  done
done; done | tee gpurun_out/$TAG.wide_rc_ab.txt
