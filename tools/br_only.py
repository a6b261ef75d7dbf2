"""Runs the blind-rotation+KS path on a B=1024 NAND batch a few times (for rocprofv3 passes)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zig-tfhe_amd"))
import numpy as np
import tfhe_amd
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
c = tfhe_amd.Context("128", 0)
if len(sys.argv) > 3:  # blind-rotation form (tfhe_amd.BR_FORMS), e.g. pair
    c.set_option("br_form", sys.argv[3])
sk, _ = c.keygen(42, 43)
g = np.random.default_rng(0)
A = sk.encrypt_bool(g.integers(0, 2, B).astype(np.uint8), seed0=1)
Bc = sk.encrypt_bool(g.integers(0, 2, B).astype(np.uint8), seed0=9999)
for _ in range(reps):
    out = c.gate_batch(np.zeros(B, np.uint8), A, Bc)
print("done", B)
