"""Tail of |v - rint(v)| over the values the fused blind rotation rounds on honest data
(DESIGN.md §6.1, round 6): the seeded 128-bit cloud key, uniformly random TLWELv0 inputs, the
oracle's fused mode (the GPU default's arithmetic, bit for bit), every pre-rounding value of
every inverse transform captured.  Prints the value count, the maximum and a histogram of the
tail above 1/16: how often a guard at 1/8 instead of 1/4 would flag an honest item.

    python tools/honest_error_tail.py [rotations per worker] [workers]   (CPU; test infrastructure)
"""
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("oracle", "tests", "zig-tfhe_amd"):
    sys.path.insert(0, os.path.join(ROOT, sub))


def work(args):
    seed, rotations = args
    from oracle import Oracle
    from conftest import get_keys
    o = Oracle(fast=True)
    k = get_keys(o, "128")
    g = np.random.default_rng(seed)
    o.set_fused(1)
    hist, mx, n = np.zeros(64, np.int64), 0.0, 0
    for _ in range(rotations):
        ct = g.integers(0, 1 << 32, k.p.n + 1, dtype=np.uint64).astype(np.uint32)
        v = o.rounded_values(lambda: o.blind_rotate(k.p, ct, k.ck.testvec, k.ck.bk, k.ck.offset), cap=1 << 21)
        e = np.abs(v - np.rint(v))
        n += e.size
        mx = max(mx, float(e.max()))
        hist += np.histogram(e, bins=64, range=(0, 0.25))[0]
    return hist, mx, n


def main():
    per = int(sys.argv[1]) if len(sys.argv) > 1 else 90
    workers = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    t0 = time.time()
    with Pool(workers) as p:
        res = p.map(work, [(100 + w, per) for w in range(workers)])
    hist, mx, n = sum(r[0] for r in res), max(r[1] for r in res), sum(r[2] for r in res)
    print(f"values {n} ({workers * per} rotations of 700 steps x 2,048 coefficients), max |v - rint v| {mx}, "
          f"{time.time() - t0:.1f} s")
    edges = np.linspace(0, 0.25, 65)
    for i in range(16, 64):
        if hist[i]:
            print(f"[{edges[i]:.4f}, {edges[i + 1]:.4f})  {hist[i]}")
    print(f">= 1/8: {int(hist[32:].sum())} values")


if __name__ == "__main__":
    main()
