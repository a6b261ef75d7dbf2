# UINT4 LUT workload with 1, 2, 4 item groups per key-switch block (--opt ks_item_groups), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for g in 1 4 8; do
    timeout -k 10 200 python bench.py --workload lut --batch 4096 --steps 5 --warmup 1 --opt ks_item_groups=$g > gpurun_out/gw$g.$r.log 2>&1 || exit 1
    echo "gw=$g $(grep -o '"value": [0-9.]*' gpurun_out/gw$g.$r.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/gw$g.$r.log)"
  done
done
