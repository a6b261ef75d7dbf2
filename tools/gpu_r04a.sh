# Round-4 diagnostics: the default bench on this box, then PMC passes of the
# octo form (B = 8,192) and the pair form (B = 1,024), the two forms that run
# two computing waves per SIMD.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04a.bench.json 2> gpurun_out/r04a.bench.err || { echo "bench failed"; tail -20 gpurun_out/r04a.bench.err; exit 1; }
tail -1 gpurun_out/r04a.bench.json | cut -c1-400
bash tools/pmc_br.sh r04a_pmc_octo 8192 octo gpurun_out/r04a_pmc_octo.json || exit 1
bash tools/pmc_br.sh r04a_pmc_pair 1024 pair gpurun_out/r04a_pmc_pair.json || exit 1
bash tools/pmc_br.sh r04a_pmc_whole 1024 whole gpurun_out/r04a_pmc_whole.json || exit 1
ls gpurun_out
