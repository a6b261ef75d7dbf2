# rocprofv3 kernel statistics of the config-3 workload (one 16-bit adder per step):
# where a level's time goes besides the latency-form blind rotation.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-adder_prof}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG -o run -- python3 $R/bench.py --workload adder --batch 1 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/$TAG.log 2>&1 || exit 1
cd $R && f=$(find gpurun_out/$TAG -name run_kernel_stats.csv -print -quit) && cp "$f" gpurun_out/${TAG}_kernel_stats.csv && cut -d, -f1-8 gpurun_out/${TAG}_kernel_stats.csv | head -12
