set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do for f in 3 0; do
timeout -k 10 200 python bench.py --workload adder --batch 1 --steps 5 --warmup 1 --no-cpu-baseline --opt ks_form=$f > gpurun_out/ksa_$f$r.json 2>/dev/null || exit 1
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['kernels'][:120])" gpurun_out/ksa_$f$r.json "ks_form=$f r$r"
done; done
