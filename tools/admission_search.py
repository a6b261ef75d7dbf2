"""Search for the worst cloud key the fused arithmetic's key admission still
admits: hill-climb the six TRGSW rows of one
CMUX (integers in [-(2^31 - 1), 2^31 - 1], the range of a BK row's torus
words) to maximise the gap between the reference's and the fused pre-rounding
values of externalProductWithFft, under the admission rule (largest BK
spectrum component <= 2^39, tfhe_gpu.cpp key_admission), against the digits
the adversary picks with the public key in hand: every level's digits
sign-aligned with its row at one output coefficient (the largest |ExtProd| the
rows admit).

The fused kernels' margin guard gives the reference's words only while that
gap stays below 1/4; DESIGN.md §6.1 records the maximum found here.

Objective of a key: max over the 2,048 outputs of |v_ref - v| for v in the
fused trees (mode 1: the whole and octo forms) and the latency form's summed
row terms (mode 4), and the pair/duo forms' regrouped sums (mode 3, A/B forms).
Moves: flip the signs of a random run of coefficients of one row, set a run to
+-(2^31 - 1), or blend the row toward a low-frequency pattern; a move is kept
when the key stays admitted and the objective does not fall.

    python tools/admission_search.py [--restarts 16] [--iters 600] [--workers 8] [--out profiles/r05_admission_search.json]

Test infrastructure (oracle/ only); writes the worst key found as a fixture
(tests/golden/admission_worst.npz) for tests/test_oracle.py.
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

R = (1 << 31) - 1
CAP = 2.0 ** 39
RMS_CAP = 0.0  # --rms-cap: largest row RMS / 2^31 admitted (0 = no energy rule); set per worker
MODES = (1, 4, 3)
PRODUCT_MODES = (1, 4)  # the product's fused forms; mode 3 (regrouped sums) is the A/B-only duo form


PARAMS = "128"  # --params: the set whose decomposition (offset, L, Bg) the external product uses


def _setup(pname=None):
    from oracle import Oracle, params
    return Oracle(), params(pname or PARAMS)


def spectrum_max(o, rows):
    return max(float(np.abs(o.ifft((r % (1 << 32)).astype(np.uint32))).max()) for rr in rows for r in rr)


def row_rms_max(rows):
    """Largest row RMS / 2^31 (the admission computes it from the spectrum by
    Parseval: spectrum energy = 2048 x row energy)."""
    return float(np.sqrt((rows.astype(np.float64) ** 2).mean(axis=-1)).max() / 2 ** 31)


def admitted(o, rows, rms_cap):
    return (rms_cap <= 0 or row_rms_max(rows) <= rms_cap) and spectrum_max(o, rows) <= CAP


def aligned_x(o, p, rows, k, part):
    """TRLWE words whose digits (decomposition offset included) are +31 / -32
    aligned in sign with row i at output k of polynomial `part`."""
    off = o.decomposition_offset(p)
    j = np.arange(1024)
    m, w = (k - j) % 1024, np.where(j <= k, 1, -1)
    F = [np.where(w * np.sign(rows[i][part][m]) >= 0, 63, 0).astype(np.uint64) for i in range(6)]

    def tmp3(f0, f1, f2):
        v = (f0 << 26) | (f1 << 20) | (f2 << 14)
        return ((v - off) % (1 << 32)).astype(np.uint32)
    return np.concatenate([tmp3(F[0], F[1], F[2]), tmp3(F[3], F[4], F[5])])


def ext_values(o, p, rows, x, mode):
    off = o.decomposition_offset(p)
    trgsw = np.array([[o.ifft((r[0] % (1 << 32)).astype(np.uint32)), o.ifft((r[1] % (1 << 32)).astype(np.uint32))]
                      for r in rows])
    try:
        o.set_fused(1 if mode in (3, 4) else mode)
        o.set_regroup({3: 1, 4: 2}.get(mode, 0))
        out = {}
        v = o.rounded_values(lambda: out.setdefault("w", o.external_product(p, trgsw, x, off)))
    finally:
        o.set_fused(0)
        o.set_regroup(False)
    return v, out["w"]


def evaluate(o, p, rows, k, part, target=None):
    """(objective, per-mode gaps, every parting word flagged by the guard); the
    objective is the max gap over the `target` modes (default: all)."""
    x = aligned_x(o, p, rows, k, part)
    v0, w0 = ext_values(o, p, rows, x, 0)
    gaps, flagged = {}, True
    for mode in MODES:
        v, wv = ext_values(o, p, rows, x, mode)
        gaps[mode] = float(np.abs(v0 - v).max())
        near = ((v + 3377699720527872.5).view(np.uint64) & np.uint64(1)) == 0
        flagged &= not bool(((w0 != wv) & ~near).any())
    return max(gaps[m] for m in (target or MODES)), gaps, flagged


def start_rows(kind, g):
    if kind == "keygen_like":
        return g.integers(-R, R + 1, (6, 2, 1024))
    if kind == "max_magnitude":
        return np.where(g.random((6, 2, 1024)) < 0.5, R, -R)
    if kind == "sparse_max":  # +-(2^31 - 1) on ~half the coefficients: the most L1 an energy cap allows
        return np.where(g.random((6, 2, 1024)) < 0.45, np.where(g.random((6, 2, 1024)) < 0.5, R, -R), 0)
    if kind == "low_frequency_scaled":  # a concentrated spectrum scaled to sit just under the cap
        f = g.integers(1, 6, (6, 2, 1))
        ph = g.random((6, 2, 1)) * 6.283
        base = np.cos(2 * np.pi * np.arange(1024) * f / 2048 + ph)
        return np.round(base * R * 0.55).astype(np.int64)
    raise ValueError(kind)


def worker(args):
    kind, seed, iters, rms_cap, target, pname = args
    o, p = _setup(pname)
    g = np.random.default_rng(seed)
    rows = start_rows(kind, g)
    while not admitted(o, rows, rms_cap):  # scale a start point in under the caps
        rows = (rows * 0.95).astype(np.int64)
    k, part = int(g.integers(0, 1024)), int(g.integers(0, 2))
    best, gaps, flagged = evaluate(o, p, rows, k, part, target)
    all_flagged = flagged
    seen = dict(gaps)  # largest gap per mode over every admitted key evaluated
    hist = [best]
    for it in range(iters):
        cand = rows.copy()
        i, h = int(g.integers(0, 6)), int(g.integers(0, 2))
        a = int(g.integers(0, 1024))
        ln = int(g.integers(1, 65))
        idx = (a + np.arange(ln)) % 1024
        mv = g.integers(0, 3)
        if mv == 0:
            cand[i, h, idx] = -cand[i, h, idx]
        elif mv == 1:
            cand[i, h, idx] = np.where(g.random(ln) < 0.5, R, -R)
        else:
            f = int(g.integers(1, 8))
            patt = np.round(R * np.cos(2 * np.pi * np.arange(1024) * f / 2048 + g.random() * 6.283)).astype(np.int64)
            t = g.random() * 0.3
            cand[i, h] = np.clip(np.round((1 - t) * cand[i, h] + t * patt), -R, R).astype(np.int64)
        if not admitted(o, cand, rms_cap):
            continue
        val, cg, fl = evaluate(o, p, cand, k, part, target)
        all_flagged &= fl
        for mode in MODES:
            seen[mode] = max(seen[mode], cg[mode])
        if val >= best:
            rows, best, gaps = cand, val, cg
        hist.append(best)
    return {"kind": kind, "seed": seed, "k": k, "part": part, "best": best, "gaps": gaps,
            "max_gap_per_mode": {str(m): v for m, v in seen.items()},
            "spectrum_max_log2": float(np.log2(spectrum_max(o, rows))), "row_rms_max": row_rms_max(rows),
            "all_flagged": bool(all_flagged), "start": hist[0], "rows": rows.astype(np.int32)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--restarts", type=int, default=16)
    ap.add_argument("--iters", type=int, default=600)
    ap.add_argument("--workers", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--rms-cap", type=float, default=0.70,
                    help="largest admitted row RMS / 2^31 (0: the spectrum cap alone, round 4's rule)")
    ap.add_argument("--target", default="", help="comma-separated modes the hill climb maximises (default: all)")
    ap.add_argument("--params", default="128", choices=["128", "80"],
                    help="parameter set (80-bit: the same L = 3, Bg = 2^6, N = 1024 external product, params.zig:70-95)")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05_admission_search.json"))
    ap.add_argument("--fixture", default=os.path.join(ROOT, "tests", "golden", "admission_worst.npz"))
    a = ap.parse_args()
    kinds = ("max_magnitude", "keygen_like", "low_frequency_scaled", "sparse_max")
    target = tuple(int(m) for m in a.target.split(",")) if a.target else None
    jobs = [(kinds[r % len(kinds)], 5000 + r, a.iters, a.rms_cap, target, a.params) for r in range(a.restarts)]
    t0 = time.time()
    with mp.get_context("spawn").Pool(a.workers) as pool:
        res = pool.map(worker, jobs)
    worst = max(res, key=lambda r: max(r["max_gap_per_mode"][str(m)] for m in PRODUCT_MODES))
    per_mode = {str(m): max(r["max_gap_per_mode"][str(m)] for r in res) for m in MODES}
    rec = {"method": __doc__.split("\n\n")[0].replace("\n", " "),
           "params": a.params, "restarts": a.restarts, "iters_per_restart": a.iters, "cap_log2": 39, "row_rms_cap": a.rms_cap,
           "objective_modes": list(target or MODES),
           "modes": {"1": "fused trees (whole, octo, latency forms' forward/MAC order)", "4": "latency form's summed row terms",
                     "3": "regrouped sums (duo form, A/B libraries only)"},
           "max_gap_per_mode": per_mode,
           "max_gap_product": max(per_mode[str(m)] for m in PRODUCT_MODES),
           "seconds": round(time.time() - t0, 1),
           "worst": {k: worst[k] for k in ("kind", "seed", "k", "part", "gaps", "max_gap_per_mode",
                                           "spectrum_max_log2", "row_rms_max", "start")},
           "every_parting_word_flagged": all(r["all_flagged"] for r in res),
           "runs": [{k: r[k] for k in ("kind", "seed", "start", "best", "max_gap_per_mode", "spectrum_max_log2",
                                       "row_rms_max", "all_flagged")} for r in res]}
    json.dump(rec, open(a.out, "w"), indent=1)
    if a.fixture:  # --fixture '': no fixture written
        np.savez_compressed(a.fixture, rows=worst["rows"], k=worst["k"], part=worst["part"], gap=worst["best"])
    print(json.dumps({k: rec[k] for k in ("max_gap_per_mode", "max_gap_product", "worst", "every_parting_word_flagged",
                                          "seconds")}, indent=1))


if __name__ == "__main__":
    main()
