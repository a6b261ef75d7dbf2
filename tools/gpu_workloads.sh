# BASELINE configs 3-5 (+ re-encryption, the single-process multi-device mode and the
# latency table) on one GPU, each its own JSON line.   bash tools/gpu_workloads.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-wl}
run() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { echo "$name failed"; tail -5 gpurun_out/${T}_$name.err; exit 1; }; tail -1 gpurun_out/${T}_$name.json; }
run adder1 --workload adder --batch 1 --steps 2 --warmup 1
run adder256 --workload adder --batch 256 --steps 2 --warmup 1
run mixed --workload mixed --batch 8192 --steps 3 --warmup 1
run mixed_nopack --workload mixed --batch 8192 --steps 3 --warmup 1 --no-pack
run lut --workload lut --batch 4096 --steps 3 --warmup 1
run reenc --workload reenc --batch 16384 --steps 3 --warmup 1
run single_process --single-process --gpus 1 --steps 5 --warmup 1
run single_process2 --single-process --gpus 2 --devices 0,0 --steps 5 --warmup 1
timeout -k 10 300 python tools/latency.py > gpurun_out/${T}_latency.txt 2>&1 || { echo "latency failed"; exit 1; }
cat gpurun_out/${T}_latency.txt
