"""Python restatement of the fdlibm/musl double-precision cos/sin (test
infrastructure: generates the `*_fdlibm` twiddle fixtures).

Why: the reference computes its FFT twiddles with Zig's @cos/@sin
(fft.zig:98-106 twists, :591-593 stage angles).  A Zig 0.15 build binds them
either to the platform libm (glibc on Linux, which tests/golden/twiddles.npz's
`*_glibc` arrays record) or to Zig's compiler_rt, whose cos/sin are ports of
musl's src/math/{cos,sin,__cos,__sin,__rem_pio2}.c (the fdlibm algorithm).
This module restates that algorithm op for op in Python floats (IEEE binary64,
round to nearest, no fused multiply-add), so the fixtures pin the second
candidate table independently of the C++ restatement in
zig-tfhe_amd/csrc/host_math.hpp (fdlibm::) and of the oracle's.

Only the argument range the tables use is restated: |x| <= 5*pi/4 (plus the
medium reduction musl takes for |x| ~ pi/2 and ~ pi).
"""
import struct

C1, C2, C3 = 4.16666666666666019037e-02, -1.38888888888741095749e-03, 2.48015872894767294178e-05
C4, C5, C6 = -2.75573143513906633035e-07, 2.08757232129817482790e-09, -1.13596475577881948265e-11
S1, S2, S3 = -1.66666666666666324348e-01, 8.33333333332248946124e-03, -1.98412698298579493134e-04
S4, S5, S6 = 2.75573137070700676789e-06, -2.50507602534068634195e-08, 1.58969099521155010221e-10
TOINT = 1.5 / 2.220446049250313080847e-16
PIO4 = float.fromhex("0x1.921fb54442d18p-1")
INVPIO2 = 6.36619772367581382433e-01
PIO2_1, PIO2_1T = 1.57079632673412561417e+00, 6.07710050650619224932e-11
PIO2_2, PIO2_2T = 6.07710050630396597660e-11, 2.02226624879595063154e-21
PIO2_3, PIO2_3T = 2.02226624871116645580e-21, 8.47842766036889956997e-32


def _bits(x: float) -> int:
    return struct.unpack("<Q", struct.pack("<d", x))[0]


def k_cos(x, y):  # musl __cos.c
    z = x * x
    w = z * z
    r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6))
    hz = 0.5 * z
    w = 1.0 - hz
    return w + (((1.0 - w) - hz) + (z * r - x * y))


def k_sin(x, y, iy):  # musl __sin.c
    z = x * x
    w = z * z
    r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6)
    v = z * x
    if iy == 0:
        return x + v * (S1 + z * r)
    return x - ((z * (0.5 * y - v * r) - y) - v * S1)


def rem_pio2(x):  # musl __rem_pio2.c, |x| <= 5pi/4 and the medium case
    u = _bits(x)
    sign = u >> 63
    ix = (u >> 32) & 0x7FFFFFFF
    if ix <= 0x400F6A7A and (ix & 0xFFFFF) != 0x921FB:
        k = 1 if ix <= 0x4002D97C else 2
        if not sign:
            z = x - k * PIO2_1
            y0 = z - k * PIO2_1T
            return k, y0, (z - y0) - k * PIO2_1T
        z = x + k * PIO2_1
        y0 = z + k * PIO2_1T
        return -k, y0, (z - y0) + k * PIO2_1T
    fn = x * INVPIO2 + TOINT - TOINT
    n = int(fn)
    r = x - fn * PIO2_1
    w = fn * PIO2_1T
    if r - w < -PIO4:
        n, fn = n - 1, fn - 1
        r, w = x - fn * PIO2_1, fn * PIO2_1T
    elif r - w > PIO4:
        n, fn = n + 1, fn + 1
        r, w = x - fn * PIO2_1, fn * PIO2_1T
    y0 = r - w
    ex = ix >> 20
    ey = (_bits(y0) >> 52) & 0x7FF
    if ex - ey > 16:
        t = r
        w = fn * PIO2_2
        r = t - w
        w = fn * PIO2_2T - ((t - r) - w)
        y0 = r - w
        ey = (_bits(y0) >> 52) & 0x7FF
        if ex - ey > 49:
            t = r
            w = fn * PIO2_3
            r = t - w
            w = fn * PIO2_3T - ((t - r) - w)
            y0 = r - w
    return n, y0, (r - y0) - w


def cos(x: float) -> float:
    ix = (_bits(x) >> 32) & 0x7FFFFFFF
    if ix <= 0x3FE921FB:
        return 1.0 if ix < 0x3E46A09E else k_cos(x, 0.0)
    n, y0, y1 = rem_pio2(x)
    return (k_cos(y0, y1), -k_sin(y0, y1, 1), -k_cos(y0, y1), k_sin(y0, y1, 1))[n & 3]


def sin(x: float) -> float:
    ix = (_bits(x) >> 32) & 0x7FFFFFFF
    if ix <= 0x3FE921FB:
        return x if ix < 0x3E500000 else k_sin(x, 0.0, 0)
    n, y0, y1 = rem_pio2(x)
    return (k_sin(y0, y1, 1), k_cos(y0, y1), -k_sin(y0, y1, 1), -k_cos(y0, y1))[n & 3]
