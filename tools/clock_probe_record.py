"""Clock-probe output (tools/bin/clock_probe, i.e. tools/phase_prof.hip built with
-DTFHE_PHASE_PROF=2) -> profiles/clock_probe.json.

The probe runs the product's blind-rotation kernel with two timer reads per wave
(s_memtime: core clock; s_memrealtime: 100 MHz) and no phase marks, six launches
back to back.  Per launch it prints the HIP-event kernel time, the mean wave span
and the core clock the waves held.  The record keeps every launch and the
kernel's cycle count per launch (event time x clock, launches after the clock has
settled), which is what bench.py divides by its own in-run kernel time to state
the clock of that run.

    python tools/clock_probe_record.py gpurun_out/r06h.clock_whole.txt [--out profiles/clock_probe.json]
"""
import argparse
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LINE = re.compile(r"rep (\d+): ([\d.]+) ms \((\d+) gates, (\w+)\); clock probe over (\d+) waves: "
                  r"mean wave span ([\d.]+) ms .*core clock ([\d.]+) GHz")
SETTLED_FROM = 3  # launches 0-2 ramp the clock up (1.88 -> 2.20 GHz on the round-6 box)


def parse(text):
    reps = []
    for m in LINE.finditer(text):
        reps.append({"launch": int(m.group(1)), "kernel_ms": float(m.group(2)), "batch": int(m.group(3)),
                     "form": m.group(4), "waves": int(m.group(5)), "wave_span_ms": float(m.group(6)),
                     "clock_ghz": float(m.group(7))})
    return reps


def record(reps, source, build_id):
    if len(reps) <= SETTLED_FROM:
        raise SystemExit(f"need more than {SETTLED_FROM} launches, got {len(reps)}")
    for r in reps:
        r["cycles_per_launch_m"] = round(r["kernel_ms"] * r["clock_ghz"], 4)  # ms x GHz = M cycles
        r["cycles_per_wave_span_m"] = round(r["wave_span_ms"] * r["clock_ghz"], 4)
    settled = reps[SETTLED_FROM:]
    per_launch = [r["cycles_per_launch_m"] for r in settled]
    per_span = [r["cycles_per_wave_span_m"] for r in reps]
    return {
        "kernel": "void tfhe::k_blind_rotate_assist<true>" if reps[0]["form"] == "whole" else reps[0]["form"],
        "batch": reps[0]["batch"], "params": "128",
        "kernel_build_id": build_id,
        "probe": ("tools/phase_prof.hip built with -DTFHE_PHASE_PROF=2 (tools/bin/clock_probe): the product "
                  "kernel source plus one s_memtime / s_memrealtime pair per wave at the start and the end of "
                  "its step loop; random operands, 6 launches back to back"),
        "launches": reps,
        "cycles_per_launch": round(statistics.mean(per_launch) * 1e6),
        "cycles_per_launch_spread": round((max(per_launch) - min(per_launch)) / 2 * 1e6),
        "cycles_per_launch_basis": (f"HIP-event kernel time x core clock, mean of launches {SETTLED_FROM}-"
                                    f"{len(reps) - 1} (after the clock ramp)"),
        "cycles_per_wave_span": round(statistics.mean(per_span) * 1e6),
        "cycles_per_wave_span_spread": round((max(per_span) - min(per_span)) / 2 * 1e6),
        "note": ("the wave span's cycle count is the same at every clock the launches held, so the kernel's "
                 "time is its cycle count over the core clock: no part of it waits on a clock-independent "
                 "latency"),
        "source": source,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "clock_probe.json"))
    ap.add_argument("--source", default=None, help="path recorded as the source (default: the log path)")
    a = ap.parse_args()
    import bench  # the product library's build id (the probe compiles the same kernel source)
    rec = record(parse(open(a.log).read()), a.source or os.path.relpath(a.log, ROOT), bench.kernel_build_id())
    json.dump(rec, open(a.out, "w"), indent=1)
    print(json.dumps({k: rec[k] for k in ("cycles_per_launch", "cycles_per_launch_spread", "cycles_per_wave_span",
                                          "cycles_per_wave_span_spread")}))


if __name__ == "__main__":
    main()
