# A/B of bench variants in alternation: bash tools/gpu_ab.sh TAG ROUNDS "opts A" "opts B" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; R=$2; shift 2
for r in $(seq 1 $R); do
  i=0
  for o in "$@"; do
    i=$((i+1))
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 $o > gpurun_out/${T}_v${i}_r$r.json 2> gpurun_out/${T}_v${i}_r$r.err || { echo "variant $i failed"; tail -5 gpurun_out/${T}_v${i}_r$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_avg_ms'], d['roofline']['kernel'])" gpurun_out/${T}_v${i}_r$r.json "v$i r$r [$o]"
  done
done
