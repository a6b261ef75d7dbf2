/*
 * tfhe_oracle.c — CPU restatement of zig-tfhe's gate-bootstrap path.
 *
 * TEST INFRASTRUCTURE ONLY (see tfhe_oracle.h): the parity checker and the
 * CPU baseline.  Never linked into, or called by, the product library.
 *
 * Every function restates the cited reference lines literally: same
 * expression trees, same loop order, same rounding.  Build with
 * -ffp-contract=off (no FMA contraction): Zig's default float mode is strict
 * and the reference never uses @mulAdd.  Twiddles come from the
 * host libm (glibc) exactly as the reference's @cos/@sin calls,
 * or from the fdlibm/musl restatement below (oracle_set_trig_source(1)).
 *
 * Paths are relative to the reference root (thedonutfactory/zig-tfhe).
 */
#include "tfhe_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#if defined(__FP_FAST_FMA) && !defined(TFHE_ORACLE_ALLOW_FMA)
/* not an error by itself: -ffp-contract=off is what matters; checked in Makefile */
#endif

#define PI_F64 3.14159265358979323846264338327950288

typedef struct { double re, im; } cplx;

/* ======================================================================== */
/* RNG: Zig std.Random.DefaultPrng (Xoshiro256) seeded through SplitMix64.  */
/* Restated from the Zig 0.15 std library (not verifiable here: no Zig).    */
/* Used only by key generation / encryption, which is off the hot path.     */
/* ======================================================================== */
static uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

void oracle_rng_init(oracle_rng *r, uint64_t seed) {
    uint64_t s = seed;
    for (int i = 0; i < 4; i++) {          /* SplitMix64.next() */
        s += 0x9e3779b97f4a7c15ULL;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
        r->s[i] = z ^ (z >> 31);
    }
}

uint64_t oracle_rng_next(oracle_rng *r) {   /* Xoshiro256++ next() */
    uint64_t *s = r->s;
    uint64_t res = rotl64(s[0] + s[3], 23) + s[0];
    uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl64(s[3], 45);
    return res;
}

/* Random.int(u32): fill(4 bytes) takes the low bytes of one next() */
uint32_t oracle_rng_u32(oracle_rng *r) { return (uint32_t)oracle_rng_next(r); }
/* Random.boolean() = int(u1) != 0: one byte from one next(), low bit */
int oracle_rng_bool(oracle_rng *r) { return (int)(oracle_rng_next(r) & 1u); }
/* Random.float(f64): 52 mantissa bits + exponent from leading zeros */
double oracle_rng_f64(oracle_rng *r) {
    uint64_t rnd = oracle_rng_next(r);
    uint64_t lz = rnd ? (uint64_t)__builtin_clzll(rnd) : 64;
    if (lz >= 12) {
        lz = 12;
        for (;;) {
            uint64_t x = oracle_rng_next(r);
            uint64_t add = x ? (uint64_t)__builtin_clzll(x) : 64;
            lz += add;
            if (add != 64) break;
            if (lz >= 1022) { lz = 1022; break; }
        }
    }
    uint64_t mant = rnd & 0xFFFFFFFFFFFFFULL;
    uint64_t bits = ((1022 - lz) << 52) | mant;
    double d;
    memcpy(&d, &bits, 8);
    return d;
}

/* ======================================================================== */
/* Torus utils — utils.zig:28-38                                             */
/* ======================================================================== */
/* Zig @mod(f64) lowers to: a = fmod(x,y); select(x < 0, fmod(a + y, y), a) */
static double zig_mod1(double d) {
    double a = fmod(d, 1.0);
    if (d < 0.0) return fmod(a + 1.0, 1.0);
    return a;
}

uint32_t oracle_f64_to_torus(double d) {           /* utils.zig:28-33 */
    double normalized = zig_mod1(d);
    double torus = normalized * 4294967296.0;
    double hi = 4294967295.0;
    double clamped = torus < hi ? torus : hi;      /* @min(torus, maxInt) */
    clamped = 0.0 > clamped ? 0.0 : clamped;       /* @max(0.0, ...)      */
    return (uint32_t)clamped;                      /* @intFromFloat truncates */
}

double oracle_torus_to_f64(uint32_t t) { return (double)t / 4294967296.0; } /* utils.zig:36-38 */

/* NormalDist (Box-Muller) — utils.zig:50-82.  Note the reference multiplies
 * the spare sample by stddev a second time (:64-66); restated as is. */
typedef struct { double mean, stddev; int has_spare; double spare; } normal_dist;

static double normal_next(normal_dist *nd, oracle_rng *r) {
    if (nd->has_spare) {
        nd->has_spare = 0;
        return nd->spare * nd->stddev + nd->mean;
    }
    double u1 = oracle_rng_f64(r);
    double u2 = oracle_rng_f64(r);
    double mag = nd->stddev * sqrt(-2.0 * log(u1));
    double two_pi = 2.0 * PI_F64;
    double z0 = mag * cos(two_pi * u2);
    double z1 = mag * sin(two_pi * u2);
    nd->has_spare = 1;
    nd->spare = z1;
    return z0 + nd->mean;
}

/* gaussianTorus — utils.zig:85-92 */
static uint32_t gaussian_torus(uint32_t mu, normal_dist *nd, oracle_rng *r) {
    double s = normal_next(nd, r);
    return oracle_f64_to_torus(s) + mu;
}

/* ======================================================================== */
/* cos/sin of the twiddles: the reference's @cos/@sin (fft.zig:98-106,       */
/* :591-593) bind to glibc (source 0, this host's libm) or, in a Zig build   */
/* that keeps compiler_rt's, to its port of the fdlibm/musl kernels (source  */
/* 1, restated here from musl __cos.c / __sin.c / __rem_pio2.c / cos.c /     */
/* sin.c for |x| <= 5pi/4 and the medium reduction at ~pi/2, ~pi).  The      */
/* Box-Muller noise (utils.zig:50-82) keeps glibc in both.                   */
/* ======================================================================== */
static double fd_kcos(double x, double y) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03, C3 = 2.48015872894767294178e-05,
                 C4 = -2.75573143513906633035e-07, C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = x * x, w = z * z;
    double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
    double hz = 0.5 * z;
    w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + (z * r - x * y));
}

static double fd_ksin(double x, double y, int iy) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03, S3 = -1.98412698298579493134e-04,
                 S4 = 2.75573137070700676789e-06, S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    double z = x * x, w = z * z;
    double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
    double v = z * x;
    if (iy == 0) return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

static uint64_t f64_bits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }

static int fd_rem_pio2(double x, double *y) {
    const double toint = 1.5 / 2.220446049250313080847e-16, pio4 = 0x1.921fb54442d18p-1,
                 invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
                 pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
                 pio2_3t = 8.47842766036889956997e-32;
    uint64_t u = f64_bits(x);
    int sign = (int)(u >> 63);
    uint32_t ix = (uint32_t)(u >> 32) & 0x7fffffffu;
    if (ix <= 0x400f6a7a && (ix & 0xfffff) != 0x921fb) {
        double k = ix <= 0x4002d97c ? 1.0 : 2.0, z;
        if (!sign) {
            z = x - k * pio2_1;
            y[0] = z - k * pio2_1t;
            y[1] = (z - y[0]) - k * pio2_1t;
            return (int)k;
        }
        z = x + k * pio2_1;
        y[0] = z + k * pio2_1t;
        y[1] = (z - y[0]) + k * pio2_1t;
        return -(int)k;
    }
    double fn = x * invpio2 + toint - toint;
    int n = (int)fn;
    double r = x - fn * pio2_1, w = fn * pio2_1t;
    if (r - w < -pio4) { n--; fn--; r = x - fn * pio2_1; w = fn * pio2_1t; }
    else if (r - w > pio4) { n++; fn++; r = x - fn * pio2_1; w = fn * pio2_1t; }
    y[0] = r - w;
    int ex = (int)(ix >> 20), ey = (int)((f64_bits(y[0]) >> 52) & 0x7ff);
    if (ex - ey > 16) {
        double t = r;
        w = fn * pio2_2; r = t - w; w = fn * pio2_2t - ((t - r) - w); y[0] = r - w;
        ey = (int)((f64_bits(y[0]) >> 52) & 0x7ff);
        if (ex - ey > 49) { t = r; w = fn * pio2_3; r = t - w; w = fn * pio2_3t - ((t - r) - w); y[0] = r - w; }
    }
    y[1] = (r - y[0]) - w;
    return n;
}

static double fd_cos(double x) {
    uint32_t ix = (uint32_t)(f64_bits(x) >> 32) & 0x7fffffffu;
    if (ix <= 0x3fe921fb) return ix < 0x3e46a09e ? 1.0 : fd_kcos(x, 0.0);
    double y[2];
    switch (fd_rem_pio2(x, y) & 3) {
    case 0: return fd_kcos(y[0], y[1]);
    case 1: return -fd_ksin(y[0], y[1], 1);
    case 2: return -fd_kcos(y[0], y[1]);
    default: return fd_ksin(y[0], y[1], 1);
    }
}

static double fd_sin(double x) {
    uint32_t ix = (uint32_t)(f64_bits(x) >> 32) & 0x7fffffffu;
    if (ix <= 0x3fe921fb) return ix < 0x3e500000 ? x : fd_ksin(x, 0.0, 0);
    double y[2];
    switch (fd_rem_pio2(x, y) & 3) {
    case 0: return fd_ksin(y[0], y[1], 1);
    case 1: return fd_kcos(y[0], y[1]);
    case 2: return -fd_ksin(y[0], y[1], 1);
    default: return -fd_kcos(y[0], y[1]);
    }
}

static int g_trig_source = 0;  /* oracle_set_trig_source; tests switch it around a call */
void oracle_set_trig_source(int source) { g_trig_source = source == 1 ? 1 : 0; }
int oracle_get_trig_source(void) { return g_trig_source; }
static double tw_cos(double x) { return g_trig_source ? fd_cos(x) : cos(x); }
static double tw_sin(double x) { return g_trig_source ? fd_sin(x) : sin(x); }
double oracle_trig_cos(double x, int source) { return source == 1 ? fd_cos(x) : cos(x); }
double oracle_trig_sin(double x, int source) { return source == 1 ? fd_sin(x) : sin(x); }

/* Arithmetic of the transforms and the MAC: 0 = the reference's expression
 * trees (default, fft.zig / trgsw.zig as written); 1 = "fused": every
 * complex multiply-add as fused multiply-adds (a = u + x*w by two fma, the
 * butterfly's b = 2u - a by one), the form the MI355X kernels use at the
 * L=3 / Bg=2^6 sets (there the exact external product is an
 * integer polynomial and both forms round to it).  Twiddle values and the
 * operation order are unchanged.  Test infrastructure, like the rest. */
/* 2 = "guarded": fused, plus the kernels' margin guard (torus_from_f64_guarded,
 * tfhe_kernels.hip): a blind rotation that rounds a value with
 * rint(2v + 1) even (|v - rint(v)| >= 1/4, via the same f64 add as the
 * kernel) is redone in the reference's trees — the MI355X default.  FUSED is
 * the arithmetic in force on this thread (a guarded recompute forces 0). */
static int g_fused = 0, g_guard = 0;
/* Regrouped row sums (the MI355X pair and duo forms):
 * in fused mode each output's MAC is two fma chains from 0.0, one over the
 * rows of a (0..L-1) and one over the rows of b (L..2L-1), added once at the
 * end, instead of one chain over rows 0..2L-1. */
/* 2 = "terms" (the latency forms): each row's product is its
 * own fma chain from 0.0, and the six products are added in row order. */
static int g_regroup = 0;
void oracle_set_regroup(int mode) { g_regroup = mode == 2 ? 2 : mode ? 1 : 0; }
/* Folded twist (evidence only; no kernel uses it):
 * fused mode only.  The forward transform takes the digit pairs
 * untwisted and every stage-len butterfly j multiplies by the folded twiddle
 * exp(i*pi*(1/2 - 2j)/len) = W_len^j * twist[512/len] instead of the
 * recurrence W_len^j: the twist of each sub-transform's second half, relative
 * to its first half's, rides on the butterfly, and the whole transform's root
 * (index 0) carries twist 1.  Exact in real arithmetic, 108 f64 instructions
 * fewer per CMUX, but its rounding errors are independent of the reference's:
 * on adversarial digits the values part by more than the margin guard's 1/4
 * (tests/test_oracle.py::test_folded_twist_decorrelates_from_the_reference). */
static int g_fold = 0;
void oracle_set_fold(int fold) { g_fold = fold ? 1 : 0; }
/* the folded twiddle of stage len, j */
void oracle_folded_twiddles(uint32_t N, double *re, double *im) {
    size_t n = N / 2;
    for (size_t len = 2; len <= n; len *= 2)
        for (size_t j = 0; j < len / 2; j++) {
            double a = (0.5 - 2.0 * (double)j) * (PI_F64 / (double)len);
            re[len / 2 - 1 + j] = tw_cos(a);
            im[len / 2 - 1 + j] = tw_sin(a);
        }
}
static __thread int tl_force_ref = 0, tl_near = 0;
#define FUSED (g_fused && !tl_force_ref)
void oracle_set_fused(int fused) {
    g_fused = fused ? 1 : 0;
    g_guard = fused == 2;
}
int oracle_get_fused(void) { return g_fused ? (g_guard ? 2 : 1) : 0; }

/* ======================================================================== */
/* FFT — fft.zig KlemsaProcessor                                             */
/* ======================================================================== */
/* twisties: KlemsaProcessor.new, fft.zig:92-106 */
void oracle_twist_table(uint32_t N, double *re, double *im) {
    double twist_unit = PI_F64 / (double)N;
    for (uint32_t i = 0; i < N / 2; i++) {
        double angle = (double)i * twist_unit;
        re[i] = tw_cos(angle);
        im[i] = tw_sin(angle);
    }
}

/* The reference keeps the twist table in its (threadlocal) processor
 * (fft.zig:79-90, :983-992); cache it per N (and trig source) the same way. */
static pthread_once_t twist_once[2] = {PTHREAD_ONCE_INIT, PTHREAD_ONCE_INIT};
static double twist1024_re[2][512], twist1024_im[2][512];
static void twist_fill(int src) {
    double twist_unit = PI_F64 / 1024.0;
    for (uint32_t i = 0; i < 512; i++) {
        double angle = (double)i * twist_unit;
        twist1024_re[src][i] = oracle_trig_cos(angle, src);
        twist1024_im[src][i] = oracle_trig_sin(angle, src);
    }
}
static void twist1024_init0(void) { twist_fill(0); }
static void twist1024_init1(void) { twist_fill(1); }

static void get_twist(uint32_t N, double *re, double *im) {
    if (N == 1024) {
        int src = g_trig_source;
        pthread_once(&twist_once[src], src ? twist1024_init1 : twist1024_init0);
        memcpy(re, twist1024_re[src], sizeof twist1024_re[src]);
        memcpy(im, twist1024_im[src], sizeof twist1024_im[src]);
    } else {
        oracle_twist_table(N, re, im);
    }
}

/* bitReverseRadix2 — fft.zig:647-669 */
static void bit_reverse_radix2(cplx *data, size_t n) {
    size_t i = 0, j = 0;
    while (i < n) {
        if (j > i) { cplx t = data[i]; data[i] = data[j]; data[j] = t; }
        size_t mask = n >> 1;
        while (mask > 0 && (j & mask) != 0) { j ^= mask; mask >>= 1; }
        j ^= mask;
        i += 1;
    }
}

/* radix2FFT — fft.zig:582-619 (reached through fftInPlace, :515-521).
 * fold (fused forward only): the folded twiddles instead of the recurrence. */
static void radix2_fft_ex(cplx *data, size_t n, int inverse, const double *fre, const double *fim) {
    bit_reverse_radix2(data, n);
    for (size_t len = 2; len <= n; len *= 2) {
        double angle = inverse ? 2.0 * PI_F64 / (double)len : -2.0 * PI_F64 / (double)len;
        double wlen_re = tw_cos(angle);
        double wlen_im = tw_sin(angle);
        for (size_t i = 0; i < n; i += len) {
            double w_re = 1.0, w_im = 0.0;
            for (size_t j = 0; j < len / 2; j++) {
                if (fre) {
                    w_re = fre[len / 2 - 1 + j];
                    w_im = fim[len / 2 - 1 + j];
                }
                cplx u = data[i + j];
                cplx x = data[i + j + len / 2];
                if (FUSED) {                               /* a = u + x*w, b = 2u - a */
                    double a_re = fma(x.re, w_re, fma(-x.im, w_im, u.re));
                    double a_im = fma(x.re, w_im, fma(x.im, w_re, u.im));
                    data[i + j].re = a_re;
                    data[i + j].im = a_im;
                    data[i + j + len / 2].re = fma(2.0, u.re, -a_re);
                    data[i + j + len / 2].im = fma(2.0, u.im, -a_im);
                } else {
                cplx v;                                    /* Complex.mul :50-55 */
                v.re = x.re * w_re - x.im * w_im;
                v.im = x.re * w_im + x.im * w_re;
                data[i + j].re = u.re + v.re;
                data[i + j].im = u.im + v.im;
                data[i + j + len / 2].re = u.re - v.re;
                data[i + j + len / 2].im = u.im - v.im;
                }
                double temp = w_re * wlen_re - w_im * wlen_im;
                w_im = w_re * wlen_im + w_im * wlen_re;
                w_re = temp;
            }
        }
    }
}
static void radix2_fft(cplx *data, size_t n, int inverse) { radix2_fft_ex(data, n, inverse, NULL, NULL); }

/* The per-stage recurrence values w_j used by radix2FFT (same for every block
 * i of a stage), exported so tests can pin the GPU twiddle tables to them.
 * Layout: stage len = 2^s (s = 1..log2(N/2)), offset len/2 - 1, j < len/2. */
void oracle_stage_twiddles(uint32_t N, int inverse, double *re, double *im) {
    size_t n = N / 2;
    for (size_t len = 2; len <= n; len *= 2) {
        double angle = inverse ? 2.0 * PI_F64 / (double)len : -2.0 * PI_F64 / (double)len;
        double wlen_re = tw_cos(angle), wlen_im = tw_sin(angle);
        double w_re = 1.0, w_im = 0.0;
        for (size_t j = 0; j < len / 2; j++) {
            re[len / 2 - 1 + j] = w_re;
            im[len / 2 - 1 + j] = w_im;
            double temp = w_re * wlen_re - w_im * wlen_im;
            w_im = w_re * wlen_im + w_im * wlen_re;
            w_re = temp;
        }
    }
}

/* ifft (torus -> frequency, the FORWARD transform) — fft.zig:142-170;
 * the N=1024 twin ifft1024 (:293-366) evaluates the identical expressions. */
void oracle_ifft(uint32_t N, const uint32_t *in, double *out) {
    size_t n2 = N / 2;
    cplx *buf = (cplx *)malloc(sizeof(cplx) * n2);
    double *tre = (double *)malloc(sizeof(double) * n2), *tim = (double *)malloc(sizeof(double) * n2);
    get_twist(N, tre, tim);
    if (FUSED && g_fold) {  /* untwisted input, folded stage twiddles */
        double *fre = (double *)malloc(sizeof(double) * n2), *fim = (double *)malloc(sizeof(double) * n2);
        oracle_folded_twiddles(N, fre, fim);
        for (size_t i = 0; i < n2; i++) {
            buf[i].re = (double)(int32_t)in[i];
            buf[i].im = (double)(int32_t)in[i + n2];
        }
        radix2_fft_ex(buf, n2, 0, fre, fim);
        for (size_t i = 0; i < n2; i++) {
            out[i] = buf[i].re * 2.0;
            out[i + n2] = buf[i].im * 2.0;
        }
        free(fre); free(fim); free(buf); free(tre); free(tim);
        return;
    }
    for (size_t i = 0; i < n2; i++) {
        double in_re = (double)(int32_t)in[i];
        double in_im = (double)(int32_t)in[i + n2];
        double w_re = tre[i], w_im = tim[i];
        if (FUSED) {
            buf[i].re = fma(in_re, w_re, -(in_im * w_im));
            buf[i].im = fma(in_re, w_im, in_im * w_re);
        } else {
            buf[i].re = in_re * w_re - in_im * w_im;
            buf[i].im = in_re * w_im + in_im * w_re;
        }
    }
    radix2_fft(buf, n2, 0);
    for (size_t i = 0; i < n2; i++) {
        out[i] = buf[i].re * 2.0;
        out[i + n2] = buf[i].im * 2.0;
    }
    free(buf); free(tre); free(tim);
}

/* fft (frequency -> torus, the INVERSE transform) — fft.zig:207-246;
 * twin fft1024 :370-443. */
/* Largest |value - nearest integer| the inverse transform has rounded on
 * this thread since the last oracle_take_round_error() (test evidence for
 * at the L=3 / Bg=2^6 sets the exact external product is an
 * integer polynomial and the float error stays far below 1/2). */
static __thread double tl_round_err = 0.0;
double oracle_take_round_error(void) {
    double e = tl_round_err;
    tl_round_err = 0.0;
    return e;
}

/* Optional capture of the values the inverse transform rounds (test evidence
 * for DESIGN.md §6.1: the distance between the reference's and the fused
 * arithmetic's pre-rounding values).  oracle_capture_rounded(buf, cap) starts
 * appending to buf (NULL stops); returns the count captured so far. */
static __thread double *tl_cap = NULL;
static __thread size_t tl_cap_n = 0, tl_cap_max = 0;
size_t oracle_capture_rounded(double *buf, size_t cap) {
    size_t n = tl_cap_n;
    tl_cap = buf;
    tl_cap_max = cap;
    tl_cap_n = 0;
    return n;
}

void oracle_fft(uint32_t N, const double *in, uint32_t *out) {
    size_t n2 = N / 2;
    cplx *buf = (cplx *)malloc(sizeof(cplx) * n2);
    double *tre = (double *)malloc(sizeof(double) * n2), *tim = (double *)malloc(sizeof(double) * n2);
    get_twist(N, tre, tim);
    for (size_t i = 0; i < n2; i++) {
        buf[i].re = in[i] * 0.5;
        buf[i].im = in[i + n2] * 0.5;
    }
    radix2_fft(buf, n2, 1);
    double normalization = 1.0 / (double)n2;
    for (size_t i = 0; i < n2; i++) {
        double w_re = tre[i], w_im = tim[i];
        double f_re = buf[i].re, f_im = buf[i].im;
        double tmp_re = (FUSED ? fma(f_re, w_re, f_im * w_im) : f_re * w_re + f_im * w_im) * normalization;
        double tmp_im = (FUSED ? fma(f_im, w_re, -(f_re * w_im)) : f_im * w_re - f_re * w_im) * normalization;
        /* reference: @round, half away from zero.  Fused mode restates the fused
         * kernels' conversion (to_torus<SMALL, true>, tfhe_kernels.hip): round to
         * nearest even (there, v + 1.5*2^52).  Inside the exact-integer regime the
         * two agree: v is within ~0.1 of an integer, so no tie occurs. */
        int64_t rr = (int64_t)(FUSED ? nearbyint(tmp_re) : round(tmp_re));
        int64_t ri = (int64_t)(FUSED ? nearbyint(tmp_im) : round(tmp_im));
        if (FUSED && g_guard) {
            double s_re = tmp_re + 3377699720527872.5, s_im = tmp_im + 3377699720527872.5;  /* 1.5*2^51 + 0.5 */
            uint64_t b_re, b_im;
            memcpy(&b_re, &s_re, 8);
            memcpy(&b_im, &s_im, 8);
            if ((b_re & 1u) == 0 || (b_im & 1u) == 0) tl_near = 1;  /* rint(2v + 1) even: |v - rint(v)| >= 1/4 */
        }
        double e_re = fabs(tmp_re - round(tmp_re)), e_im = fabs(tmp_im - round(tmp_im));
        if (e_re > tl_round_err) tl_round_err = e_re;
        if (e_im > tl_round_err) tl_round_err = e_im;
        if (tl_cap && tl_cap_n + 2 <= tl_cap_max) {  /* output order: i, then i + n2 */
            tl_cap[tl_cap_n + 0] = tmp_re;
            tl_cap[tl_cap_n + 1] = tmp_im;
            tl_cap_n += 2;
        }
        out[i] = (uint32_t)(int32_t)rr;
        out[i + n2] = (uint32_t)(int32_t)ri;
    }
    free(buf); free(tre); free(tim);
}

/* poly_mul — fft.zig:458-492 */
void oracle_poly_mul(uint32_t N, const uint32_t *a, const uint32_t *b, uint32_t *out) {
    size_t n2 = N / 2;
    double *af = (double *)malloc(sizeof(double) * N);
    double *bf = (double *)malloc(sizeof(double) * N);
    double *rf = (double *)malloc(sizeof(double) * N);
    oracle_ifft(N, a, af);
    oracle_ifft(N, b, bf);
    for (size_t i = 0; i < n2; i++) {
        double ar = af[i], ai = af[i + n2], br = bf[i], bi = bf[i + n2];
        rf[i] = (ar * br - ai * bi) * 0.5;
        rf[i + n2] = (ar * bi + ai * br) * 0.5;
    }
    oracle_fft(N, rf, out);
    free(af); free(bf); free(rf);
}

/* naive negacyclic product — fft.zig:695-714 (the reference's in-test oracle) */
void oracle_poly_mul_naive(uint32_t N, const uint32_t *a, const uint32_t *b, uint32_t *out) {
    for (uint32_t i = 0; i < N; i++) out[i] = 0;
    for (uint32_t i = 0; i < N; i++)
        for (uint32_t j = 0; j < N; j++) {
            if (i + j < N) out[i + j] += a[i] * b[j];
            else out[i + j - N] -= a[i] * b[j];
        }
}

/* ======================================================================== */
/* TRGSW / TRLWE — trgsw.zig, trlwe.zig                                     */
/* ======================================================================== */
/* genDecompositionOffset — key.zig:121-131 */
uint32_t oracle_decomposition_offset(const oracle_params *p) {
    uint32_t offset = 0, bg = 1u << p->bgbit;
    for (uint32_t i = 0; i < p->L; i++) {
        uint32_t shift = 32 - (i + 1) * p->bgbit;
        offset += (bg / 2) * (1u << shift);
    }
    return offset;
}

/* decompositionIntoStorage — trgsw.zig:193-219 (rows 0..L-1 from a, L..2L-1 from b) */
void oracle_decomposition(const oracle_params *p, const uint32_t *trlwe, uint32_t offset,
                          uint32_t *dec) {
    uint32_t N = p->N, L = p->L;
    uint32_t mask = (1u << p->bgbit) - 1, half_bg = 1u << (p->bgbit - 1);
    for (uint32_t j = 0; j < N; j++) {
        uint32_t tmp0 = trlwe[j] + offset;
        uint32_t tmp1 = trlwe[N + j] + offset;
        for (uint32_t i = 0; i < L; i++)
            dec[i * N + j] = ((tmp0 >> (32 - (i + 1) * p->bgbit)) & mask) - half_bg;
        for (uint32_t i = 0; i < L; i++)
            dec[(i + L) * N + j] = ((tmp1 >> (32 - (i + 1) * p->bgbit)) & mask) - half_bg;
    }
}

/* polyMulWithXK — trgsw.zig:442-466; k in [0, 2N] */
void oracle_poly_mul_with_xk(uint32_t N, const uint32_t *a, uint32_t k, uint32_t *res) {
    if (k < N) {
        for (uint32_t i = 0; i < N - k; i++) res[k + i] = a[i];
        for (uint32_t i = N - k; i < N; i++) res[i + k - N] = 0u - a[i];
    } else {
        for (uint32_t i = 0; i < 2 * N - k; i++) res[i + k - N] = 0u - a[i];
        for (uint32_t i = 0; i < N - (2 * N - k); i++) res[i] = a[2 * N - k + i];
    }
}

/* fmaInFd1024 — trgsw.zig:157-189 */
static void fma_in_fd(size_t n2, double *res, const double *a, const double *b) {
    for (size_t i = 0; i < n2; i++) {
        double a_re = a[i], a_im = a[i + n2], b_re = b[i], b_im = b[i + n2];
        if (FUSED) {  /* res += a*b*0.5 by fma; b*0.5 is exact */
            res[i] = fma(a_re, b_re * 0.5, fma(-a_im, b_im * 0.5, res[i]));
            res[i + n2] = fma(a_re, b_im * 0.5, fma(a_im, b_re * 0.5, res[i + n2]));
            continue;
        }
        double real_part = (a_re * b_re - a_im * b_im) * 0.5;
        res[i] = res[i] + real_part;
        double imag_part = (a_re * b_im + a_im * b_re) * 0.5;
        res[i + n2] = res[i + n2] + imag_part;
    }
}

/* externalProductWithFft — trgsw.zig:111-154.  trgsw_fft layout (A14):
 * [2L rows][a | b][N f64: re0..re_{N/2-1}, im0..im_{N/2-1}] */
void oracle_external_product(const oracle_params *p, const double *trgsw_fft,
                             const uint32_t *trlwe, uint32_t offset, uint32_t *out) {
    uint32_t N = p->N, R = 2 * p->L;
    uint32_t *dec = (uint32_t *)malloc(sizeof(uint32_t) * R * N);
    double *dec_fft = (double *)malloc(sizeof(double) * R * N);
    double *out_a = (double *)calloc(N, sizeof(double));
    double *out_b = (double *)calloc(N, sizeof(double));
    oracle_decomposition(p, trlwe, offset, dec);
    for (uint32_t r = 0; r < R; r++) oracle_ifft(N, dec + (size_t)r * N, dec_fft + (size_t)r * N);
    if (FUSED && g_regroup == 2) {  /* ((t0 + t1) + t2) + ..., each term from 0.0 */
        double *ta = (double *)malloc(sizeof(double) * N), *tb = (double *)malloc(sizeof(double) * N);
        for (uint32_t r = 0; r < R; r++) {
            const double *row = trgsw_fft + (size_t)r * 2 * N;
            memset(ta, 0, sizeof(double) * N);
            memset(tb, 0, sizeof(double) * N);
            fma_in_fd(N / 2, ta, dec_fft + (size_t)r * N, row);
            fma_in_fd(N / 2, tb, dec_fft + (size_t)r * N, row + N);
            for (uint32_t i = 0; i < N; i++) {
                out_a[i] = r ? out_a[i] + ta[i] : ta[i];
                out_b[i] = r ? out_b[i] + tb[i] : tb[i];
            }
        }
        free(ta); free(tb);
    } else if (FUSED && g_regroup) {  /* (rows 0..L-1) + (rows L..2L-1), each chain from 0.0 */
        double *hi_a = (double *)calloc(N, sizeof(double)), *hi_b = (double *)calloc(N, sizeof(double));
        for (uint32_t r = 0; r < R; r++) {
            const double *row = trgsw_fft + (size_t)r * 2 * N;
            fma_in_fd(N / 2, r < p->L ? out_a : hi_a, dec_fft + (size_t)r * N, row);
            fma_in_fd(N / 2, r < p->L ? out_b : hi_b, dec_fft + (size_t)r * N, row + N);
        }
        for (uint32_t i = 0; i < N; i++) {
            out_a[i] = out_a[i] + hi_a[i];
            out_b[i] = out_b[i] + hi_b[i];
        }
        free(hi_a); free(hi_b);
    } else {
    for (uint32_t r = 0; r < R; r++) {
        const double *row = trgsw_fft + (size_t)r * 2 * N;
        fma_in_fd(N / 2, out_a, dec_fft + (size_t)r * N, row);
        fma_in_fd(N / 2, out_b, dec_fft + (size_t)r * N, row + N);
    }
    }
    oracle_fft(N, out_a, out);
    oracle_fft(N, out_b, out + N);
    free(dec); free(dec_fft); free(out_a); free(out_b);
}

/* cmux — trgsw.zig:260-284: tmp = in2 - in1; out = ExtProd(cond, tmp) + in1 */
void oracle_cmux(const oracle_params *p, const uint32_t *in1, const uint32_t *in2,
                 const double *trgsw_fft, uint32_t offset, uint32_t *out) {
    uint32_t N = p->N;
    uint32_t *tmp = (uint32_t *)calloc(2 * N, sizeof(uint32_t));
    uint32_t *tmp2 = (uint32_t *)malloc(sizeof(uint32_t) * 2 * N);
    for (uint32_t i = 0; i < 2 * N; i++) tmp[i] = in2[i] - in1[i]; /* rot - acc */
    oracle_external_product(p, trgsw_fft, tmp, offset, tmp2);
    for (uint32_t i = 0; i < 2 * N; i++) out[i] = tmp2[i] + in1[i];
    free(tmp); free(tmp2);
}

/* blindRotate — trgsw.zig:290-333 (cloud testvec) and blindRotateWithTestvec
 * :336-400 (custom testvec).  b~ uses a 64-bit add (:297); the testvec
 * variant's 32-bit wrapping add (:345) yields the same rotation because
 * X^0 = X^{2N} = 1 (both give the identity at the wrap point). */
void oracle_blind_rotate(const oracle_params *p, const uint32_t *src, const uint32_t *testvec,
                         const double *bk, uint32_t offset, uint32_t *acc) {
    uint32_t N = p->N, nbit = p->nbit;
    uint64_t round_half = 1ull << (32 - 1 - nbit - 1);
    uint32_t shift = 32 - nbit - 1;
    uint32_t b_tilda = 2 * N - (uint32_t)(((uint64_t)src[p->n] + round_half) >> shift);
    uint32_t *res2 = (uint32_t *)malloc(sizeof(uint32_t) * 2 * N);
    uint32_t *nxt = (uint32_t *)malloc(sizeof(uint32_t) * 2 * N);
    size_t row = (size_t)2 * p->L * 2 * N;
    tl_near = 0;
    for (int pass = 0; pass < 2; pass++) {  /* guarded mode: a second pass in the reference's trees */
        oracle_poly_mul_with_xk(N, testvec, b_tilda, acc);
        oracle_poly_mul_with_xk(N, testvec + N, b_tilda, acc + N);
        for (uint32_t i = 0; i < p->n; i++) {
            uint32_t a_tilda = (uint32_t)(((uint64_t)src[i] + round_half) >> shift);
            oracle_poly_mul_with_xk(N, acc, a_tilda, res2);
            oracle_poly_mul_with_xk(N, acc + N, a_tilda, res2 + N);
            oracle_cmux(p, acc, res2, bk + i * row, offset, nxt);
            memcpy(acc, nxt, sizeof(uint32_t) * 2 * N);
        }
        if (!(FUSED && g_guard && tl_near)) break;
        tl_force_ref = 1;
    }
    tl_force_ref = 0;
    tl_near = 0;
    free(res2); free(nxt);
}

/* sampleExtractIndex — trlwe.zig:146-162 */
void oracle_sample_extract_index(uint32_t N, const uint32_t *trlwe, uint32_t k, uint32_t *out) {
    for (uint32_t i = 0; i < N; i++) {
        if (i <= k) out[i] = trlwe[k - i];
        else out[i] = 0u - trlwe[N + k - i];
    }
    out[N] = trlwe[N + k];
}

/* sampleExtractIndex2 — trlwe.zig:165-180.  The reference bounds the loop
 * by tlwe_lv0.N (= n), not the ring size: p[i] = a[k-i] (i<=k),
 * -a[n+k-i] (k<i<n), p[n] = b[k] (b at offset N in the TRLWE). */
void oracle_sample_extract_index2(uint32_t n, uint32_t N, const uint32_t *trlwe, uint32_t k, uint32_t *out) {
    for (uint32_t i = 0; i < n; i++) {
        if (i <= k) out[i] = trlwe[k - i];
        else out[i] = 0u - trlwe[n + k - i];
    }
    out[n] = trlwe[N + k];
}

/* identityKeySwitching — trgsw.zig:471-502; ksk layout [(BASE*T*i)+(BASE*j)+k][n+1] */
void oracle_identity_key_switch(const oracle_params *p, const uint32_t *src, const uint32_t *ksk,
                                uint32_t *res) {
    uint32_t N = p->N, n = p->n, basebit = p->basebit, T = p->iks_t;
    uint32_t base = 1u << basebit;
    for (uint32_t x = 0; x <= n; x++) res[x] = 0;
    res[n] = src[N];
    uint32_t prec_offset = 1u << (32 - (1 + basebit * T));
    for (uint32_t i = 0; i < N; i++) {
        uint32_t a_bar = src[i] + prec_offset;
        for (uint32_t j = 0; j < T; j++) {
            uint32_t k = (a_bar >> (32 - (j + 1) * basebit)) & (base - 1);
            if (k != 0) {
                size_t idx = (size_t)base * T * i + (size_t)base * j + k;
                const uint32_t *row = ksk + idx * (n + 1);
                for (uint32_t x = 0; x <= n; x++) res[x] -= row[x];
            }
        }
    }
}

/* VanillaBootstrap.bootstrap — bootstrap/vanilla.zig:38-52 */
void oracle_bootstrap(const oracle_params *p, const uint32_t *in, const uint32_t *testvec,
                      const double *bk, const uint32_t *ksk, uint32_t offset, uint32_t *out) {
    uint32_t N = p->N;
    uint32_t *acc = (uint32_t *)malloc(sizeof(uint32_t) * 2 * N);
    uint32_t *lv1 = (uint32_t *)malloc(sizeof(uint32_t) * (N + 1));
    oracle_blind_rotate(p, in, testvec, bk, offset, acc);
    oracle_sample_extract_index(N, acc, 0, lv1);
    oracle_identity_key_switch(p, lv1, ksk, out);
    free(acc); free(lv1);
}

/* VanillaBootstrap.bootstrapWithoutKeySwitch — vanilla.zig:58-69 */
void oracle_bootstrap_without_key_switch(const oracle_params *p, const uint32_t *in, const uint32_t *testvec,
                                         const double *bk, uint32_t offset, uint32_t *out) {
    uint32_t *acc = (uint32_t *)malloc(sizeof(uint32_t) * 2 * p->N);
    oracle_blind_rotate(p, in, testvec, bk, offset, acc);
    oracle_sample_extract_index2(p->n, p->N, acc, 0, out);
    free(acc);
}

/* Gate linear pre-combination — gates.zig:48-121 (tlwe.zig:120-239 ops),
 * constants via f64ToTorus.  Op numbering = include/tfhe_gpu.h TFHE_GATE_*. */
void oracle_gate_combine(const oracle_params *p, int op, const uint32_t *a, const uint32_t *b,
                         uint32_t *out) {
    uint32_t n1 = p->n + 1;
    double c = 0.0;
    for (uint32_t i = 0; i < n1; i++) {
        uint32_t x = a[i], y = b[i], r = 0;
        switch (op) {
        case 0: r = (0u - x) + (0u - y); break;  /* NAND  :48-54  */
        case 1: r = x + y; break;                /* OR    :57-61  */
        case 2: r = x + y; break;                /* AND   :64-68  */
        case 3: r = x + y * 2u; break;           /* XOR   :71-75 addMul */
        case 4: r = x - y * 2u; break;           /* XNOR  :78-82 subMul */
        case 5: r = (0u - x) + (0u - y); break;  /* NOR   :85-91  */
        case 6: r = (0u - x) + y; break;         /* ANDNY :94-99  */
        case 7: r = x - y; break;                /* ANDYN :102-106 */
        case 8: r = (0u - x) + y; break;         /* ORNY  :109-114 */
        case 9: r = x - y; break;                /* ORYN  :117-121 */
        default: r = x; break;
        }
        out[i] = r;
    }
    switch (op) {
    case 0: case 1: case 8: case 9: c = 0.125; break;
    case 2: case 5: case 6: case 7: c = -0.125; break;
    case 3: c = 0.25; break;
    case 4: c = -0.25; break;
    default: return;
    }
    out[p->n] = out[p->n] + oracle_f64_to_torus(c);
}

void oracle_gate(const oracle_params *p, int op, const uint32_t *a, const uint32_t *b,
                 const uint32_t *testvec, const double *bk, const uint32_t *ksk, uint32_t offset,
                 uint32_t *out) {
    uint32_t *t = (uint32_t *)malloc(sizeof(uint32_t) * (p->n + 1));
    oracle_gate_combine(p, op, a, b, t);
    oracle_bootstrap(p, t, testvec, bk, ksk, offset, out);
    free(t);
}

typedef struct {
    const oracle_params *p; size_t lo, hi; const uint8_t *ops; const uint32_t *a, *b, *tv;
    const double *bk; const uint32_t *ksk; uint32_t offset; uint32_t *out;
} gate_job;

static void *gate_worker(void *arg) {
    gate_job *j = (gate_job *)arg;
    size_t n1 = j->p->n + 1;
    for (size_t g = j->lo; g < j->hi; g++)
        oracle_gate(j->p, j->ops[g], j->a + g * n1, j->b + g * n1, j->tv, j->bk, j->ksk, j->offset,
                    j->out + g * n1);
    return NULL;
}

void oracle_gate_batch(const oracle_params *p, int threads, size_t B, const uint8_t *ops,
                       const uint32_t *a, const uint32_t *b, const uint32_t *testvec,
                       const double *bk, const uint32_t *ksk, uint32_t offset, uint32_t *out) {
    if (threads < 1) threads = 1;
    if ((size_t)threads > B) threads = (int)(B ? B : 1);
    pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    gate_job *jobs = (gate_job *)malloc(sizeof(gate_job) * threads);
    for (int t = 0; t < threads; t++) {
        gate_job j = {p, B * t / threads, B * (t + 1) / threads, ops, a, b, testvec, bk, ksk, offset, out};
        jobs[t] = j;
        pthread_create(&tid[t], NULL, gate_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    free(tid); free(jobs);
}

/* ======================================================================== */
/* Keys and encryption                                                       */
/* ======================================================================== */
/* SecretKey.new — key.zig:41-57; `seed` replaces getUniqueSeed() */
void oracle_secret_key_new(const oracle_params *p, uint64_t seed, uint32_t *k0, uint32_t *k1) {
    oracle_rng r;
    oracle_rng_init(&r, seed);
    for (uint32_t i = 0; i < p->n; i++) k0[i] = oracle_rng_bool(&r) ? 1u : 0u;
    for (uint32_t i = 0; i < p->N; i++) k1[i] = oracle_rng_bool(&r) ? 1u : 0u;
}

/* genTestvec — key.zig:134-145 */
void oracle_testvec(const oracle_params *p, uint32_t *tv) {
    uint32_t bt = oracle_f64_to_torus(0.125);
    for (uint32_t i = 0; i < p->N; i++) { tv[i] = 0; tv[p->N + i] = bt; }
}

/* TLWELv0.encryptF64 — tlwe.zig:34-49 (also TLWELv1.encryptF64 :270-285) */
void oracle_tlwe_encrypt_f64(uint32_t n, double mu, double alpha, const uint32_t *key, uint64_t seed,
                             uint32_t *out) {
    oracle_rng r;
    oracle_rng_init(&r, seed);
    uint32_t inner = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t rt = oracle_rng_u32(&r);
        inner += key[i] * rt;
        out[i] = rt;
    }
    normal_dist nd = {0.0, alpha, 0, 0.0};
    uint32_t mu_t = oracle_f64_to_torus(mu);               /* gaussianF64 :95-102 */
    uint32_t noise = gaussian_torus(mu_t, &nd, &r);
    out[n] = inner + noise;
}

/* decryptBool — tlwe.zig:58-68 */
uint32_t oracle_tlwe_phase(uint32_t n, const uint32_t *ct, const uint32_t *key) {
    uint32_t inner = 0;
    for (uint32_t i = 0; i < n; i++) inner += ct[i] * key[i];
    return ct[n] - inner;
}
int oracle_tlwe_decrypt_bool(uint32_t n, const uint32_t *ct, const uint32_t *key) {
    return (int32_t)oracle_tlwe_phase(n, ct, key) >= 0;
}

/* TRLWELv1.encryptF64 — trlwe.zig:30-64 */
void oracle_trlwe_encrypt_f64(const oracle_params *p, const double *mu, double alpha,
                              const uint32_t *key_lv1, uint64_t seed, uint32_t *out) {
    uint32_t N = p->N;
    oracle_rng r;
    oracle_rng_init(&r, seed);
    for (uint32_t i = 0; i < N; i++) out[i] = oracle_rng_u32(&r);
    normal_dist nd = {0.0, alpha, 0, 0.0};
    for (uint32_t i = 0; i < N; i++) out[N + i] = gaussian_torus(oracle_f64_to_torus(mu[i]), &nd, &r);
    uint32_t *pr = (uint32_t *)malloc(sizeof(uint32_t) * N);
    oracle_poly_mul(N, out, key_lv1, pr);
    for (uint32_t i = 0; i < N; i++) out[N + i] = out[N + i] + pr[i];
    free(pr);
}

/* TRLWELv1.decryptBool — trlwe.zig:82-98 */
void oracle_trlwe_decrypt_bool(const oracle_params *p, const uint32_t *ct, const uint32_t *key_lv1,
                               uint8_t *out) {
    uint32_t N = p->N;
    uint32_t *pr = (uint32_t *)malloc(sizeof(uint32_t) * N);
    oracle_poly_mul(N, ct, key_lv1, pr);
    for (uint32_t i = 0; i < N; i++) out[i] = (int32_t)(ct[N + i] - pr[i]) >= 0;
    free(pr);
}

/* TRGSWLv1.encryptTorus — trgsw.zig:35-71, then TRGSWLv1FFT.new :81-91 */
void oracle_trgsw_encrypt_torus_fft(const oracle_params *p, uint32_t mu, double alpha,
                                    const uint32_t *key_lv1, oracle_rng *master, double *out) {
    uint32_t N = p->N, L = p->L;
    uint32_t *rows = (uint32_t *)malloc(sizeof(uint32_t) * 2 * L * 2 * N);
    double *zero = (double *)calloc(N, sizeof(double));
    for (uint32_t i = 0; i < 2 * L; i++)
        oracle_trlwe_encrypt_f64(p, zero, alpha, key_lv1, oracle_rng_next(master), rows + (size_t)i * 2 * N);
    for (uint32_t i = 0; i < L; i++) {
        /* std.math.pow(f64, BG, -(i+1)) is an exact power of two */
        uint32_t h = oracle_f64_to_torus(ldexp(1.0, -(int)((i + 1) * p->bgbit)));
        rows[(size_t)i * 2 * N] += mu * h;                       /* trlwe[i].a[0]   */
        rows[(size_t)(i + L) * 2 * N + N] += mu * h;             /* trlwe[i+L].b[0] */
    }
    for (uint32_t i = 0; i < 2 * L; i++) {                       /* TRLWELv1FFT.new trlwe.zig:112-132 */
        oracle_ifft(N, rows + (size_t)i * 2 * N, out + (size_t)i * 2 * N);
        oracle_ifft(N, rows + (size_t)i * 2 * N + N, out + (size_t)i * 2 * N + N);
    }
    free(rows); free(zero);
}

/* CloudKey.new — key.zig:70-77: KSK (genKeySwitchingKey :148-172) then BK
 * (genBootstrappingKey :175-212).  Every getUniqueSeed() draws the master
 * stream.  KSK k=0 slots are left undefined by the reference (`resize`,
 * :156) and never read (trgsw.zig:490); here they are zeroed. */
void oracle_cloud_key_new(const oracle_params *p, uint64_t seed, const uint32_t *key_lv0,
                          const uint32_t *key_lv1, uint32_t *ksk, double *bk) {
    uint32_t N = p->N, n = p->n, T = p->iks_t, basebit = p->basebit, base = 1u << basebit;
    oracle_rng master;
    oracle_rng_init(&master, seed);
    for (uint32_t i = 0; i < N; i++)
        for (uint32_t j = 0; j < T; j++)
            for (uint32_t k = 0; k < base; k++) {
                size_t idx = (size_t)base * T * i + (size_t)base * j + k;
                uint32_t *row = ksk + idx * (n + 1);
                if (k == 0) { memset(row, 0, sizeof(uint32_t) * (n + 1)); continue; }
                uint32_t shift = (j + 1) * basebit;
                double pv = ((double)k * (double)key_lv1[i]) / (double)(1u << shift);
                oracle_tlwe_encrypt_f64(n, pv, p->alpha_ksk, key_lv0, oracle_rng_next(&master), row);
            }
    size_t row = (size_t)2 * p->L * 2 * N;
    for (uint32_t i = 0; i < n; i++)
        oracle_trgsw_encrypt_torus_fft(p, key_lv0[i], p->alpha_bsk, key_lv1, &master, bk + i * row);
}

/* ======================================================================== */
/* Programmable bootstrap (LUT) — lut/generator.zig:85-135, encoder.zig     */
/* ======================================================================== */
size_t oracle_div_round(size_t a, size_t b) { return (a + b / 2) / b; }  /* divRound, generator.zig:253-255 */

/* generateLookupTableFullAssign (generator.zig:155-191): raw[divRound(xN, m) ..
 * divRound((x+1)N, m)) = values[x]; rotate by divRound(N, 2m); negate the tail */
void oracle_lut_generate_full(uint32_t N, uint32_t m, const uint32_t *values, uint32_t *tv) {
    uint32_t *raw = (uint32_t *)calloc(N, sizeof(uint32_t));
    for (uint32_t x = 0; x < m; x++) {
        size_t start = oracle_div_round((size_t)x * N, m), end = oracle_div_round((size_t)(x + 1) * N, m);
        for (size_t xx = start; xx < end; xx++) raw[xx] = values[x];
    }
    size_t offset = oracle_div_round(N, 2 * (size_t)m);
    for (size_t i = 0; i < N; i++) tv[N + i] = raw[(i + offset) % N];
    for (size_t i = N - offset; i < N; i++) tv[N + i] = ~tv[N + i] + 1u;
    for (size_t i = 0; i < N; i++) tv[i] = 0;
    free(raw);
}

/* generateLookupTableAssign (generator.zig:85-135) with Encoder.withScale(m,
 * scale) (encoder.zig:49-74): values[x] = f64ToTorus((f(x) mod m) * scale) */
void oracle_lut_generate_scaled(uint32_t N, uint32_t m, double scale, const uint32_t *f_table, uint32_t *tv) {
    uint32_t *enc = (uint32_t *)calloc(m, sizeof(uint32_t));
    for (uint32_t x = 0; x < m; x++) enc[x] = oracle_f64_to_torus((double)(f_table[x] % m) * scale);
    oracle_lut_generate_full(N, m, enc, tv);
    free(enc);
}

/* Generator.new(m) (generator.zig:29-41): Encoder.new(m), scale 1/(2m) (encoder.zig:29-42) */
void oracle_lut_generate(uint32_t N, uint32_t m, const uint32_t *f_table, uint32_t *tv) {
    oracle_lut_generate_scaled(N, m, 1.0 / (2.0 * (double)m), f_table, tv);
}

/* Generator.modSwitch (generator.zig:223-227): (x / maxInt(u32)) * size, + 0.5, truncated, mod size */
size_t oracle_lut_mod_switch(uint32_t x, size_t size) {
    double scaled = ((double)x / (double)4294967295u) * (double)size;
    return (size_t)(scaled + 0.5) % size;
}

/* encryptLweMessage / decryptLweMessage — tlwe.zig:74-117 */
void oracle_tlwe_encrypt_lwe_message(uint32_t n, uint32_t msg, uint32_t m, double alpha,
                                     const uint32_t *key, uint64_t seed, uint32_t *out) {
    uint32_t norm = msg % m;
    double scale = 1.0 / (2.0 * (double)m);
    oracle_tlwe_encrypt_f64(n, (double)norm * scale, alpha, key, seed, out);
}

uint32_t oracle_tlwe_decrypt_lwe_message(uint32_t n, const uint32_t *ct, uint32_t m, const uint32_t *key) {
    uint32_t res = oracle_tlwe_phase(n, ct, key);
    double f = oracle_torus_to_f64(res);
    double scale = 1.0 / (2.0 * (double)m);
    uint64_t msg = (uint64_t)(f / scale + 0.5);
    return (uint32_t)(msg % m);
}

/* ---- proxy re-encryption — proxy_reenc.zig -------------------------------- */

/* reencryptTLWELv0 — proxy_reenc.zig:267-306: the identity key switch with an
 * n-coefficient input and the re-encryption key in place of the KSK. */
void oracle_reencrypt(uint32_t n, uint32_t basebit, uint32_t t, const uint32_t *ct, const uint32_t *key,
                      uint32_t *out) {
    uint32_t base = 1u << basebit;
    for (uint32_t x = 0; x < n; x++) out[x] = 0;
    out[n] = ct[n];
    uint32_t prec_offset = 1u << (32 - (1 + basebit * t));
    for (uint32_t i = 0; i < n; i++) {
        uint32_t a_bar = ct[i] + prec_offset;
        for (uint32_t j = 0; j < t; j++) {
            uint32_t k = (a_bar >> (32 - (j + 1) * basebit)) & (base - 1);
            if (k == 0) continue;
            const uint32_t *row = key + ((size_t)base * t * i + (size_t)base * j + k) * (n + 1);
            for (uint32_t x = 0; x <= n; x++) out[x] -= row[x];
        }
    }
}

/* PublicKeyLv0.newWithParams — proxy_reenc.zig:57-76 */
void oracle_public_key_gen(uint32_t n, const uint32_t *key, size_t size, double alpha, uint64_t seed0,
                           uint32_t *pk) {
    for (size_t e = 0; e < size; e++) oracle_tlwe_encrypt_f64(n, 0.0, alpha, key, seed0 + e, pk + e * (n + 1));
}

/* PublicKeyLv0.encryptF64 — proxy_reenc.zig:83-113 */
void oracle_public_key_encrypt_f64(uint32_t n, const uint32_t *pk, size_t size, double plaintext, double alpha,
                                   uint64_t seed, uint32_t *out) {
    oracle_rng r;
    oracle_rng_init(&r, seed);
    for (uint32_t x = 0; x <= n; x++) out[x] = 0;
    out[n] = oracle_f64_to_torus(plaintext);
    for (size_t e = 0; e < size; e++) {
        if (!oracle_rng_bool(&r)) continue;           /* keep this encryption of zero? */
        const uint32_t *enc = pk + e * (n + 1);
        if (oracle_rng_bool(&r)) { for (uint32_t x = 0; x <= n; x++) out[x] += enc[x]; }
        else                     { for (uint32_t x = 0; x <= n; x++) out[x] -= enc[x]; }
    }
    normal_dist nd = {0.0, alpha, 0, 0.0};
    out[n] += gaussian_torus(0u, &nd, &r);            /* gaussianF64(0.0, ...) */
}

/* ProxyReencryptionKey.newAsymmetricWithParams :150-196 / newSymmetricWithParams :214-256 */
void oracle_reenc_key_gen(uint32_t n, const uint32_t *key_from, const uint32_t *key_to, const uint32_t *pk,
                          size_t pk_size, double alpha, uint32_t basebit, uint32_t t, uint64_t seed0,
                          uint32_t *out) {
    uint32_t base = 1u << basebit;
    memset(out, 0, sizeof(uint32_t) * (size_t)n * t * base * (n + 1));
    uint64_t c = 0;
    for (uint32_t i = 0; i < n; i++)
        for (uint32_t j = 0; j < t; j++)
            for (uint32_t k = 1; k < base; k++) {
                double pv = ((double)k * (double)key_from[i]) / (double)(1u << ((j + 1) * basebit));
                uint32_t *row = out + ((size_t)base * t * i + (size_t)base * j + k) * (n + 1);
                if (pk) oracle_public_key_encrypt_f64(n, pk, pk_size, pv, alpha, seed0 + c++, row);
                else    oracle_tlwe_encrypt_f64(n, pv, alpha, key_to, seed0 + c++, row);
            }
}
