set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for G in 8 16 32; do
  TFHE_KS_G=$G timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ks$G -o run -- python $R/tools/ks_tune.py 128 > $R/gpurun_out/ks$G.log 2>&1 || exit 1
done
TFHE_KS_G=16 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ksu4 -o run -- python $R/tools/ks_tune.py uint4 > $R/gpurun_out/ksu4.log 2>&1 || exit 1
