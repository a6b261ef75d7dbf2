# rocprofv3 kernel statistics of the config-4 and config-5 workload lines (final build).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-wlstats}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_mixed -o run -- python3 $R/bench.py --workload mixed --batch 65536 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/${TAG}_mixed.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_lut -o run -- python3 $R/bench.py --workload lut --batch 4096 --steps 8 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${TAG}_lut.log 2>&1 || exit 1
cd $R
for w in mixed lut; do f=$(find gpurun_out/${TAG}_$w -name run_kernel_stats.csv -print -quit) && cp "$f" gpurun_out/${TAG}_${w}_kernel_stats.csv; done
