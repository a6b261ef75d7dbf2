# Builds tools/bin/lib_ab.so: the product sources compiled as an A/B build
# (TFHE_AB_BUILD) plus tools/ab/tfhe_ab_forms.hip (the duo and split-transform
# latency forms, TFHE_OPT_BR_FORM 6 and 7; round 4's whole form at L = 3 without
# the loader assist, 8; development copies of the assist form, 9 + VAR, tools/ab/tfhe_ab_assist_dev.hip).  tfhe_gpu_create refuses it unless
# TFHE_ALLOW_AB_BUILD=1; select it with TFHE_GPU_LIB:
#   [NAME=x] [ABD_SCHED="..."] bash tools/ab_forms.sh [extra hipcc flags]   (NAME: tools/bin/lib_ab_x.so;
#   ABD_SCHED: the scheduler flags of the assist-form copies, default max-memory-clause)
#   TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=$PWD/tools/bin/lib_ab.so python bench.py --opt br_form=6 ...
set -e
cd "$(dirname "$0")/.."
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Izig-tfhe_amd/csrc -DTFHE_AB_BUILD $*"
O=tools/bin/ab_obj${NAME:+_$NAME}
mkdir -p $O
$H -c -o $O/k.o zig-tfhe_amd/csrc/tfhe_kernels.hip &
$H -mllvm -amdgpu-sched-strategy=max-memory-clause -c -o $O/w.o zig-tfhe_amd/csrc/tfhe_kernels_whole.hip &
$H -mllvm -amdgpu-sched-strategy=max-memory-clause -c -o $O/ab.o tools/ab/tfhe_ab_forms.hip &
$H ${ABD_SCHED--mllvm -amdgpu-sched-strategy=max-memory-clause} -c -o $O/abd.o tools/ab/tfhe_ab_assist_dev.hip &
$H -x hip -c -o $O/g.o zig-tfhe_amd/csrc/tfhe_gpu.cpp &
wait
printf 'extern "C" const char *tfhe_gpu_build_id(void) { return "ab-%s"; }\n' "$(cat $O/k.o $O/w.o $O/ab.o $O/abd.o | sha256sum | cut -c1-13)" > $O/id.cpp
g++ -O2 -fPIC -c -o $O/id.o $O/id.cpp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/bin/lib_ab${NAME:+_$NAME}.so $O/k.o $O/w.o $O/ab.o $O/abd.o $O/g.o $O/id.o
echo "tools/bin/lib_ab${NAME:+_$NAME}.so"
