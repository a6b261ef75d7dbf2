set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/gpu3.log 2>&1; echo "pytest exit $?" >> gpurun_out/gpu3.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke3.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/bench3.log 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof3 -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof3.log 2>&1 || exit 3
