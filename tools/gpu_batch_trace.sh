# Kernel trace of the NAND bench at one batch size: gaps between a step's kernels.
#   bash tools/gpu_batch_trace.sh TAG BATCH
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-bt}
B=${2:-2048}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$TAG -o run -- python3 $R/bench.py --batch $B --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/$TAG.log 2>&1 || exit 1
cd $R && f=$(find gpurun_out/$TAG -name run_kernel_trace.csv -print -quit) && python3 - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
prev = None
for r in rows[-16:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0
    print(f'{r["Kernel_Name"][:50]:50s} dur {(e - s) / 1e3:9.1f} us  gap {gap:9.1f} us')
    prev = e
PY
