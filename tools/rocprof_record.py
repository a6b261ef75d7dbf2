"""rocprofv3 --kernel-trace --stats summary -> profiles/rocprof_blind_rotate.json.

Takes the blind-rotation row of a run_kernel_stats.csv (copied under profiles/),
tags it with the loaded library's kernel build id, and writes the record that
bench.py reports as roofline.kernel_avg_ms_rocprof beside its HIP-event average
(only while the build id matches).

    python tools/rocprof_record.py profiles/<tag>_kernel_stats.csv [out.json]
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    src = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "rocprof_blind_rotate.json")
    rows = [r for r in csv.DictReader(open(src)) if "k_blind_rotate" in r["Name"]]
    if not rows:
        raise SystemExit(f"no blind-rotation row in {src}")
    r = max(rows, key=lambda r: float(r["TotalDurationNs"]))  # the main launch, not the guard's recompute
    import bench  # noqa: E402
    calls = int(r["Calls"])
    rec = {"kernel": r["Name"].split("(")[0], "kernel_build_id": bench.kernel_build_id(),
           "launches": calls, "avg_ms": round(float(r["AverageNs"]) / 1e6, 4),
           "min_ms": round(float(r["MinNs"]) / 1e6, 4), "max_ms": round(float(r["MaxNs"]) / 1e6, 4),
           "avg_ms_without_max": round((float(r["TotalDurationNs"]) - float(r["MaxNs"])) / max(1, calls - 1) / 1e6, 4),
           "source": os.path.relpath(src, ROOT)}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
