"""rocprofv3 --kernel-trace --stats summary -> profiles/rocprof_blind_rotate.json.

Takes the blind-rotation row of a run_kernel_stats.csv (copied under profiles/),
tags it with the loaded library's kernel build id, and writes the record that
bench.py reports as roofline.kernel_avg_ms_rocprof beside its HIP-event average
(only while the build id matches).

    python tools/rocprof_record.py profiles/<tag>_kernel_stats.csv [out.json] [kernel_trace.csv warmup]

With the run's kernel trace, the record also carries the average over the launches after
the first `warmup` ones BY POSITION (dispatch order): the warm-up steps of bench.py, whatever
their durations (dropping the slowest launch would also drop a real outlier).
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
    if len(sys.argv) > 4:
        trace, warm = sys.argv[3], int(sys.argv[4])
        name = r["Name"].split("(")[0]
        ds = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"]) - int(x["Start_Timestamp"]))
                    for x in csv.DictReader(open(trace)) if x["Kernel_Name"].split("(")[0] == name)
        if len(ds) != calls:
            raise SystemExit(f"kernel trace has {len(ds)} launches of {name}, the stats row {calls}")
        kept = [d for _, d in ds[warm:]]
        rec["avg_ms_excl_warmup"] = round(sum(kept) / len(kept) / 1e6, 4)
        rec["warmup_launches_excluded"] = warm
        rec["trace"] = os.path.relpath(trace, ROOT)
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
