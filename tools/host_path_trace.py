"""Timeline of host-buffer gate batches (tfhe_gpu_gate_batch, 1,024 NAND gates):
run under rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace and
print per call the copies, kernels and gaps.

    rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \\
        -d gpurun_out/hp -o run -- python3 tools/host_path_trace.py
    python3 tools/host_path_trace.py --report gpurun_out/hp
"""
import csv
import glob
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run():
    sys.path.insert(0, os.path.join(ROOT, "zig-tfhe_amd"))
    import numpy as np
    import tfhe_amd
    c = tfhe_amd.Context("128", 0)
    sk, _ = c.keygen(42, 43)
    g = np.random.default_rng(0)
    A = sk.encrypt_bool(g.integers(0, 2, 1024).astype(np.uint8), seed0=1)
    B = sk.encrypt_bool(g.integers(0, 2, 1024).astype(np.uint8), seed0=9999)
    ops = np.zeros(1024, np.uint8)
    for _ in range(3):
        c.gate_batch(ops, A, B)
    ts = []
    for _ in range(8):
        t0 = time.perf_counter()
        c.gate_batch(ops, A, B)
        ts.append(time.perf_counter() - t0)
    print("host wall ms per call:", " ".join(f"{t * 1e3:.3f}" for t in ts))


def report(d):
    rows = []
    for f in glob.glob(f"{d}/**/run_kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append(("K " + r["Kernel_Name"].split("(")[0].replace("void tfhe::", ""), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for f in glob.glob(f"{d}/**/run_memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append(("C " + r.get("Direction", r.get("Operation", "?")) + f" {int(r.get('Bytes', 0) or 0)}",
                         int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    api = []
    for f in glob.glob(f"{d}/**/run_hip_api_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            api.append(("A " + r["Function"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort(key=lambda x: x[1])
    api.sort(key=lambda x: x[1])
    # the last 8 blind-rotation launches and what lies around them
    br = [r for r in rows if "k_blind_rotate<3, true, true, true, true>" in r[0] or "k_blind_rotate<3,true,true,true,true>" in r[0]]
    if not br:
        br = [r for r in rows if "k_blind_rotate" in r[0] and "false, true>" not in r[0]]
    for k in br[-3:]:
        lo, hi = k[1] - 600_000, k[2] + 400_000
        print("---- call around blind rotation at", k[1])
        for r in sorted([x for x in rows + api if lo <= x[1] <= hi], key=lambda x: x[1]):
            print(f"{(r[1] - k[1]) / 1e3:10.1f} us  dur {(r[2] - r[1]) / 1e3:9.1f} us  {r[0][:90]}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--report":
        report(sys.argv[2])
    else:
        run()
