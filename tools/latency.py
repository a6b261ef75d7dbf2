"""Gate-bootstrap latency/throughput vs batch size for each blind-rotation form (dev tool)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zig-tfhe_amd"))
import numpy as np
import torch  # noqa: F401
import tfhe_amd
c = tfhe_amd.Context("128", 0)
sk, _ = c.keygen(42, 43)
g = np.random.default_rng(0)
for B in [1, 8, 64, 128, 256, 512, 1024]:
    A = sk.encrypt_bool(g.integers(0, 2, B).astype(np.uint8), seed0=1)
    Bc = sk.encrypt_bool(g.integers(0, 2, B).astype(np.uint8), seed0=9999)
    ops = np.zeros(B, np.uint8)
    row = [f"B={B:5d}"]
    for form in ["whole", "octo", "wide"]:
        c.set_option("br_form", form)
        c.gate_batch(ops, A, Bc)
        t0 = time.perf_counter()
        for _ in range(3):
            out = c.gate_batch(ops, A, Bc)
        ms = (time.perf_counter() - t0) / 3 * 1e3
        ok = np.array_equal(sk.decrypt_bool(out), ~(sk.decrypt_bool(A) & sk.decrypt_bool(Bc)))
        row.append(f"{form} {ms:8.2f} ms ({B / ms * 1e3:9.0f}/s){'' if ok else ' WRONG'}")
    print("  ".join(row), flush=True)
