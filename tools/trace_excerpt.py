"""Blind-rotation rows of a rocprofv3 run_kernel_trace.csv (the record's per-launch
durations, small enough to commit beside the stats csv).

    python tools/trace_excerpt.py run_kernel_trace.csv out.csv
"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_blind_rotate" in r["Kernel_Name"]]
if not rows:
    raise SystemExit(f"no blind-rotation launches in {sys.argv[1]}")
keep = ["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp", "VGPR_Count", "LDS_Block_Size", "Grid_Size_X"]
with open(sys.argv[2], "w", newline="") as f:
    w = csv.DictWriter(f, fieldnames=keep, extrasaction="ignore")
    w.writeheader()
    w.writerows(rows)
print(f"{len(rows)} blind-rotation launches -> {sys.argv[2]}")
