# BASELINE configs 3-5 on one GPU (each its own JSON line)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --workload adder --batch 1 --steps 2 --warmup 1 > gpurun_out/wl_adder1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload adder --batch 256 --steps 2 --warmup 1 > gpurun_out/wl_adder256.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload mixed --batch 8192 --steps 3 --warmup 1 > gpurun_out/wl_mixed.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload lut --batch 4096 --steps 3 --warmup 1 > gpurun_out/wl_lut.log 2>&1 || exit 1
