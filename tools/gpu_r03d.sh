# Round-3 check: full GPU tests, host pipeline, guard breakdown A/B, octo vs whole
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_pipe.sh r03d 2 noguard nomin guard || exit 1
bash tools/gpu_octo.sh r03d_octo 2 || exit 1
