# Host-buffer pipeline check: GPU tests, copy rates, and the single-process host-buffer bench
# with the pipeline on / off in alternation vs the device-resident bench.  bash tools/gpu_pipe.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-pipe}
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG.gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/$TAG.gpu_tests.log; exit 1; }
tail -2 gpurun_out/$TAG.gpu_tests.log
timeout -k 10 60 tools/bin/copy_bw > gpurun_out/$TAG.copy_bw.txt 2>&1 || { echo "copy_bw failed"; exit 1; }
cat gpurun_out/$TAG.copy_bw.txt
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_dev$r.json 2>/dev/null || { echo "bench failed"; exit 1; }
  for pl in 1 0; do
    timeout -k 10 200 python bench.py --single-process --gpus 1 --steps 10 --warmup 2 --opt host_pipeline=$pl > gpurun_out/${TAG}_sp${pl}_$r.json 2>/dev/null || { echo "single-process bench failed"; exit 1; }
  done
  python - <<PY
import json
d=json.load(open("gpurun_out/${TAG}_dev$r.json"))
a=json.load(open("gpurun_out/${TAG}_sp1_$r.json")); b=json.load(open("gpurun_out/${TAG}_sp0_$r.json"))
print("r$r device-resident", d["value"], d["ms_per_step"], "| host pipeline", a["value"], a["ms_per_step"], a["decrypt_check"], "| host plain", b["value"], b["ms_per_step"], b["decrypt_check"], "| pipeline/device %.3f" % (a["value"]/d["value"]))
PY
done
[ -n "$2" ] && bash tools/gpu_ab_libs.sh ${TAG}_ab $2 ${@:3}
exit 0
