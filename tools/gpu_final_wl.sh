# Final BASELINE configs 3-5 lines (more steps for stable numbers) + 2-rank gloo rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --workload adder --batch 1 --steps 3 --warmup 1 > gpurun_out/fw_adder1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload adder --batch 256 --steps 3 --warmup 1 > gpurun_out/fw_adder256.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload mixed --batch 8192 --steps 5 --warmup 1 > gpurun_out/fw_mixed.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload lut --batch 4096 --steps 8 --warmup 2 > gpurun_out/fw_lut.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload reenc --batch 16384 --steps 8 --warmup 2 > gpurun_out/fw_reenc.log 2>&1 || exit 1
