"""Margin-guard recompute rate and cost on honest batches.
Runs STEPS batches of 1,024 NAND gates over fresh encryptions (a new set every batch), device-
resident, under the library TFHE_GPU_LIB points at (the product's 1/4 guard, or an A/B build with
-DTFHE_GUARD_EIGHTH), and prints one JSON line: items recomputed by the guard, batches that had
any, ms per batch, and whether every output decrypts.

    [TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=...] python tools/guard_rate.py STEPS [params]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zig-tfhe_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (HIP runtime first)

import tfhe_amd  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    pname = sys.argv[2] if len(sys.argv) > 2 else "128"
    B = 1024
    c = tfhe_amd.Context(pname, 0)
    sk, _ = c.keygen(42, 43)
    dev = torch.device("cuda", 0)
    g = np.random.default_rng(77)
    t_ops = torch.zeros(B, dtype=torch.uint8, device=dev)
    t_o = torch.zeros((B, c.params.n + 1), dtype=torch.int32, device=dev)
    c.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    hit_batches, ok, el = 0, True, 0.0
    c.sync()
    base = c.near_tie_items()
    for s in range(steps):
        a, b = g.integers(0, 2, B).astype(np.uint8), g.integers(0, 2, B).astype(np.uint8)
        t_a = torch.from_numpy(sk.encrypt_bool(a, seed0=10_000_000 + 2 * s * B).view(np.int32)).to(dev)
        t_b = torch.from_numpy(sk.encrypt_bool(b, seed0=10_000_000 + (2 * s + 1) * B).view(np.int32)).to(dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        c.gate_batch_dev(t_ops.data_ptr(), t_a.data_ptr(), t_b.data_ptr(), t_o.data_ptr(), B)
        torch.cuda.synchronize()
        el += time.perf_counter() - t0
        c.sync()
        now = c.near_tie_items()
        hit_batches += now != base
        base = now
        out = t_o.cpu().numpy().view(np.uint32)
        ok &= bool(np.array_equal(sk.decrypt_bool(out), ~(a.astype(bool) & b.astype(bool))))
    c.sync()
    print(json.dumps({"lib": tfhe_amd.build_id(), "params": pname, "batches": steps, "items": steps * B,
                      "recomputed_items": int(c.near_tie_items()), "batches_with_recompute": int(hit_batches),
                      "ms_per_batch": round(el / steps * 1e3, 3), "decrypt_check": ok,
                      "kernels": c.last_kernels()}), flush=True)
    c.set_stream(None)
    c.close()


if __name__ == "__main__":
    main()
