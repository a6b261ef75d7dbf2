"""Generates the committed fixtures in tests/golden/ (run from the repo root).

The reference (Zig) cannot be built or run in this image and ships no golden
vectors for this path, so the fixtures are of two kinds:

* independent exact values, computed here WITHOUT the oracle:
  - twiddles.npz: the reference's twist factors cos/sin(i*pi/1024) (fft.zig:98-106)
    evaluated by the platform libm (glibc, via Python's math module) and
    correctly rounded by mpmath (200 bits); the stage-twiddle recurrence of
    radix2FFT (fft.zig:590-616) restated in Python floats (IEEE doubles); and
    the same tables from the fdlibm/musl cos/sin that Zig's compiler_rt ports
    (fdlibm_trig.py, the `*_fdlibm` arrays), the other libm a Zig build can bind.
  - polymul_bigint.npz: exact negacyclic products mod 2^32 by Python big ints.
* oracle regression vectors (oracle_vectors.npz): seeded inputs and the
  oracle's outputs for the FFT pair and a small gate batch, so the GPU tests
  have fixed expected bits even before the oracle is rebuilt on a box.
"""
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def stage_recurrence(cos, sin, N=1024):
    """radix2FFT's stage twiddles (fft.zig:590-616): w <- w*wlen per block, restated in Python floats."""
    fr, fi = [0.0] * (N // 2 - 1), [0.0] * (N // 2 - 1)
    ln = 2
    while ln <= N // 2:
        ang = -2.0 * math.pi / ln
        wr, wi = cos(ang), sin(ang)
        w_re, w_im = 1.0, 0.0
        for j in range(ln // 2):
            fr[ln // 2 - 1 + j], fi[ln // 2 - 1 + j] = w_re, w_im
            t = w_re * wr - w_im * wi
            w_im = w_re * wi + w_im * wr
            w_re = t
        ln *= 2
    return fr, fi


def twiddles():
    import mpmath
    sys.path.insert(0, HERE)
    import fdlibm_trig as fd
    mpmath.mp.prec = 200
    N = 1024
    unit = math.pi / N
    re_g, im_g, re_c, im_c, re_f, im_f = [], [], [], [], [], []
    for i in range(N // 2):
        ang = float(i) * unit  # one f64 rounding, like the reference
        re_g.append(math.cos(ang))
        im_g.append(math.sin(ang))
        re_f.append(fd.cos(ang))
        im_f.append(fd.sin(ang))
        a = mpmath.mpf(ang)
        re_c.append(float(mpmath.cos(a)))
        im_c.append(float(mpmath.sin(a)))
    fr, fi = stage_recurrence(math.cos, math.sin, N)
    fr_f, fi_f = stage_recurrence(fd.cos, fd.sin, N)
    np.savez(os.path.join(HERE, "twiddles.npz"),
             twist_re_glibc=np.array(re_g), twist_im_glibc=np.array(im_g),
             twist_re_cr=np.array(re_c), twist_im_cr=np.array(im_c),
             stage_fwd_re=np.array(fr), stage_fwd_im=np.array(fi),
             twist_re_fdlibm=np.array(re_f), twist_im_fdlibm=np.array(im_f),
             stage_fwd_re_fdlibm=np.array(fr_f), stage_fwd_im_fdlibm=np.array(fi_f))
    for name, (r, m) in {"glibc": (re_g, im_g), "fdlibm": (re_f, im_f)}.items():
        diff = [(i, "cos") for i in range(N // 2) if r[i] != re_c[i]] + \
               [(i, "sin") for i in range(N // 2) if m[i] != im_c[i]]
        print(f"twist entries where {name} != correctly rounded:", sorted(diff))
    print("twist entries glibc != fdlibm:", sorted([(i, "cos") for i in range(N // 2) if re_g[i] != re_f[i]] +
                                                   [(i, "sin") for i in range(N // 2) if im_g[i] != im_f[i]]))
    print("stage entries glibc != fdlibm:", [i for i in range(N // 2 - 1) if fr[i] != fr_f[i] or fi[i] != fi_f[i]])


def polymul_bigint(count=3):
    g = np.random.default_rng(2024)
    A, B, E = [], [], []
    for _ in range(count):
        a = g.integers(0, 1 << 32, 1024, dtype=np.uint64).astype(np.uint32)
        b = (g.integers(0, 1 << 32, 1024, dtype=np.uint64) % 64).astype(np.uint32)
        ai, bi = [int(x) for x in a], [int(x) for x in b]
        res = [0] * 1024
        for i in range(1024):
            x = ai[i]
            for j in range(1024):
                k = i + j
                if k < 1024:
                    res[k] += x * bi[j]
                else:
                    res[k - 1024] -= x * bi[j]
        A.append(a)
        B.append(b)
        E.append(np.array([v % (1 << 32) for v in res], np.uint32))
    np.savez(os.path.join(HERE, "polymul_bigint.npz"), a=np.array(A), b=np.array(B), exact=np.array(E))


def oracle_vectors():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle, params
    o = Oracle()
    g = np.random.default_rng(77)
    polys = g.integers(0, 1 << 32, (6, 1024), dtype=np.uint64).astype(np.uint32)
    polys[0] = 0
    polys[1] = 0xFFFFFFFF
    polys[2] = 0
    polys[2][0] = 1 << 31
    polys[3] = 0x7FFFFFFF
    fwd = np.array([o.ifft(x) for x in polys])
    inv = np.array([o.fft(f) for f in fwd])
    p = params("80")
    k0, k1 = o.secret_key(p, 42)
    ck = o.cloud_key(p, 43, k0, k1)
    ops = np.arange(10, dtype=np.uint8)
    bits_a = g.integers(0, 2, 10)
    bits_b = g.integers(0, 2, 10)
    A = np.array([o.tlwe_encrypt_bool(p.n, a, p.alpha_lv0, k0, 7000 + i) for i, a in enumerate(bits_a)])
    B = np.array([o.tlwe_encrypt_bool(p.n, b, p.alpha_lv0, k0, 8000 + i) for i, b in enumerate(bits_b)])
    out = o.gate_batch(p, ops, A, B, ck, threads=8)
    np.savez(os.path.join(HERE, "oracle_vectors.npz"), fft_in=polys, fft_fwd=fwd, fft_inv=inv,
             gate_ops=ops, gate_a=A, gate_b=B, gate_out=out, gate_params="80", sk_seed=42, ck_seed=43)




def gates128_vectors():
    """The headline configuration's bits: the 128-bit cloud key from
    seeds (sk 42, ck 43), one gate of each op plus NANDs, 700-step blind rotations and the
    key switch, stored as inputs + outputs + sha256 of the outputs (the 172 MB key is
    regenerated from the seeds)."""
    import hashlib
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle, params
    o = Oracle()
    p = params("128")
    k0, k1 = o.secret_key(p, 42)
    ck = o.cloud_key(p, 43, k0, k1)
    g = np.random.default_rng(128)
    ops = np.concatenate([np.arange(10), np.zeros(6)]).astype(np.uint8)
    bits_a = g.integers(0, 2, ops.size)
    bits_b = g.integers(0, 2, ops.size)
    A = np.array([o.tlwe_encrypt_bool(p.n, a, p.alpha_lv0, k0, 17000 + i) for i, a in enumerate(bits_a)])
    B = np.array([o.tlwe_encrypt_bool(p.n, b, p.alpha_lv0, k0, 18000 + i) for i, b in enumerate(bits_b)])
    out = o.gate_batch(p, ops, A, B, ck, threads=8)
    digest = hashlib.sha256(np.ascontiguousarray(out, np.uint32).tobytes()).hexdigest()
    np.savez(os.path.join(HERE, "gates128.npz"), ops=ops, a=A, b=B, bits_a=bits_a, bits_b=bits_b, out=out,
             out_sha256=digest, params="128", sk_seed=42, ck_seed=43)
    print("gates128 sha256", digest)


def gates128_fdlibm_vectors():
    """gates128_vectors with the FFT twiddles from the fdlibm/musl cos/sin (the
    other libm a Zig build can bind): the key is regenerated from
    the same seeds (its BK transforms use those twiddles too), same inputs."""
    import hashlib
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle, params
    o = Oracle()
    o.set_trig_source(1)
    p = params("128")
    k0, k1 = o.secret_key(p, 42)
    ck = o.cloud_key(p, 43, k0, k1)
    g = np.load(os.path.join(HERE, "gates128.npz"))
    out = o.gate_batch(p, g["ops"], g["a"], g["b"], ck, threads=8)
    o.set_trig_source(0)
    digest = hashlib.sha256(np.ascontiguousarray(out, np.uint32).tobytes()).hexdigest()
    np.savez(os.path.join(HERE, "gates128_fdlibm.npz"), ops=g["ops"], a=g["a"], b=g["b"], out=out,
             out_sha256=digest, params="128", sk_seed=42, ck_seed=43, twiddles="fdlibm")
    print("gates128_fdlibm sha256", digest, "words differing from the glibc fixture:",
          int((out != g["out"]).sum()), "of", out.size)


def lut_uint4_vectors():
    """BASELINE config 5's bits: UINT4 keys from seeds (sk 42, ck 43), the LUT of
    f(x) = (x + 1) mod 16 (lut/generator.zig:85-135), every message 0..15 encrypted
    (tlwe.zig:74-88), 820-step blind rotations with the LUT test vector + sample
    extract + key switch (trgsw.zig:336-400, :471-502): inputs, test vector, outputs and
    the outputs' sha256 (the 350 MB key is regenerated from the seeds)."""
    import hashlib
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle, params
    o = Oracle()
    p = params("uint4")
    k0, k1 = o.secret_key(p, 42)
    ck = o.cloud_key(p, 43, k0, k1)
    msgs = np.arange(16, dtype=np.uint32)
    tv = o.lut_generate(p.N, 16, (msgs + 1) % 16)
    cts = np.array([o.encrypt_lwe_message(p.n, int(m), 16, p.alpha_lv0, k0, 27000 + i) for i, m in enumerate(msgs)])
    out = o.gate_batch(p, np.full(16, 255, np.uint8), cts, cts, ck, testvec=tv, threads=8)
    digest = hashlib.sha256(np.ascontiguousarray(out, np.uint32).tobytes()).hexdigest()
    np.savez(os.path.join(HERE, "lut_uint4.npz"), msgs=msgs, cts=cts, testvec=tv, out=out, out_sha256=digest,
             params="uint4", sk_seed=42, ck_seed=43)
    print("lut_uint4 sha256", digest)


if __name__ == "__main__":
    what = sys.argv[1:] or ["twiddles", "polymul_bigint", "oracle_vectors", "gates128_vectors",
                            "gates128_fdlibm_vectors", "lut_uint4_vectors"]
    for name in what:
        globals()[name]()
