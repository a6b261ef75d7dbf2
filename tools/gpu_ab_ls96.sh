# A/B of two library builds (tools/bin/lib_<A>.so, lib_<B>.so) on the NAND batch at 1,024 and 4,096 gates,
# the 80-bit set and the 65,536-gate circuit, then the GPU tests on build B: bash tools/gpu_ab_ls96.sh A B
set -o pipefail
cd $GRAFT_REPO_ROOT
A=${1:-new}; B=${2:-cur}
bash tools/gpu_ab_libs_wl.sh s1k 2 "--steps 10 --warmup 2 --no-cpu-baseline" $A $B || exit 1
bash tools/gpu_ab_libs_wl.sh s80 2 "--params 80 --steps 10 --warmup 2 --no-cpu-baseline" $A $B || exit 1
bash tools/gpu_ab_libs_wl.sh s4k 2 "--batch 4096 --steps 5 --warmup 1 --no-cpu-baseline" $A $B || exit 1
bash tools/gpu_ab_libs_wl.sh smx 2 "--workload mixed --batch 65536 --steps 2 --warmup 1" $A $B || exit 1
TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$PWD/tools/bin/lib_$B.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
