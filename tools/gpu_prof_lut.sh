# Kernel stats of the config-5 (UINT4 LUT, 4096) workload: bash tools/gpu_prof_lut.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-lut}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$T -o lut -- python3 $R/bench.py --workload lut --batch 4096 --steps 3 --warmup 1 > $R/gpurun_out/$T.log 2>&1 || exit 1
