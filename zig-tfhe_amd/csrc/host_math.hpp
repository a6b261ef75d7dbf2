// host_math.hpp — host-side scalar helpers of the product library: the Zig
// DefaultPrng stream, torus conversion, Box-Muller noise and FFT twiddle
// tables.  These restate reference host code (utils.zig, fft.zig setup,
// Zig std.Random) that runs once per key / encryption, never per bootstrap.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace tfhe {
namespace host {

constexpr double kPi = 3.14159265358979323846264338327950288;

// std.Random.DefaultPrng = Xoshiro256 (++), seeded through SplitMix64.
struct Rng {
    uint64_t s[4];
    explicit Rng(uint64_t seed) {
        uint64_t x = seed;
        for (int i = 0; i < 4; i++) {
            x += 0x9e3779b97f4a7c15ULL;
            uint64_t z = x;
            z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
            z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
            s[i] = z ^ (z >> 31);
        }
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        uint64_t r = rotl(s[0] + s[3], 23) + s[0];
        uint64_t t = s[1] << 17;
        s[2] ^= s[0];
        s[3] ^= s[1];
        s[1] ^= s[2];
        s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return r;
    }
    uint32_t u32() { return (uint32_t)next(); }          // Random.int(u32)
    bool boolean() { return (next() & 1u) != 0; }        // Random.boolean()
    double f64() {                                       // Random.float(f64)
        uint64_t r = next();
        uint64_t lz = r ? (uint64_t)__builtin_clzll(r) : 64;
        if (lz >= 12) {
            lz = 12;
            for (;;) {
                uint64_t x = next();
                uint64_t add = x ? (uint64_t)__builtin_clzll(x) : 64;
                lz += add;
                if (add != 64) break;
                if (lz >= 1022) {
                    lz = 1022;
                    break;
                }
            }
        }
        uint64_t bits = ((1022 - lz) << 52) | (r & 0xFFFFFFFFFFFFFULL);
        double d;
        std::memcpy(&d, &bits, 8);
        return d;
    }
};

// utils.f64ToTorus (utils.zig:28-33); Zig's float @mod(x, 1.0).
inline uint32_t f64_to_torus(double d) {
    double a = std::fmod(d, 1.0);
    double normalized = d < 0.0 ? std::fmod(a + 1.0, 1.0) : a;
    double torus = normalized * 4294967296.0;
    double c = torus < 4294967295.0 ? torus : 4294967295.0;
    c = 0.0 > c ? 0.0 : c;
    return (uint32_t)c;
}

// utils.NormalDist (utils.zig:50-82), spare sample scaled by stddev again as
// in the reference (:64-66).
struct NormalDist {
    double mean, stddev;
    bool has_spare = false;
    double spare = 0.0;
    NormalDist(double m, double s) : mean(m), stddev(s) {}
    double next(Rng &r) {
        if (has_spare) {
            has_spare = false;
            return spare * stddev + mean;
        }
        double u1 = r.f64(), u2 = r.f64();
        double mag = stddev * std::sqrt(-2.0 * std::log(u1));
        double two_pi = 2.0 * kPi;
        double z0 = mag * std::cos(two_pi * u2);
        double z1 = mag * std::sin(two_pi * u2);
        has_spare = true;
        spare = z1;
        return z0 + mean;
    }
};

// gaussianTorus (utils.zig:85-92)
inline uint32_t gaussian_torus(uint32_t mu, NormalDist &nd, Rng &r) { return f64_to_torus(nd.next(r)) + mu; }

// ---- cos / sin of the twiddle tables ---------------------------------------
// The reference computes its twiddles with Zig's @cos/@sin (fft.zig:98-106,
// :591-593).  Which libm that binds depends on the Zig build: a linkLibC build
// on Linux can resolve them to glibc (correctly rounded here but for two
// entries), a build that keeps Zig's compiler_rt gets its port of the
// fdlibm/musl kernels.  Both are restated: source 0 = glibc (this host's
// libm), source 1 = the fdlibm/musl algorithm below (musl src/math/__cos.c,
// __sin.c, __rem_pio2.c, cos.c, sin.c; Zig lib/compiler_rt/{cos,sin,trig,
// rem_pio2}.zig port them op for op).  Only the |x| <= 5pi/4 paths of
// __rem_pio2 exist (plus its medium case for x ~ pi/2, pi): the tables'
// angles are within [-pi, pi].
namespace fdlibm {

inline double k_cos(double x, double y) {  // __cos
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03, C3 = 2.48015872894767294178e-05,
                 C4 = -2.75573143513906633035e-07, C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = x * x, w = z * z;
    double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
    double hz = 0.5 * z;
    w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + (z * r - x * y));
}

inline double k_sin(double x, double y, int iy) {  // __sin
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03, S3 = -1.98412698298579493134e-04,
                 S4 = 2.75573137070700676789e-06, S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    double z = x * x, w = z * z;
    double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
    double v = z * x;
    if (iy == 0) return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

inline uint64_t bits(double x) {
    uint64_t u;
    std::memcpy(&u, &x, 8);
    return u;
}

// __rem_pio2 for |x| < 2^20*pi/2: x = n*pi/2 + y[0] + y[1]
inline int rem_pio2(double x, double *y) {
    const double toint = 1.5 / 2.220446049250313080847e-16, pio4 = 0x1.921fb54442d18p-1,
                 invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
                 pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
                 pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
                 pio2_3t = 8.47842766036889956997e-32;
    const uint64_t u = bits(x);
    const int sign = (int)(u >> 63);
    const uint32_t ix = (uint32_t)(u >> 32) & 0x7fffffffu;
    if (ix <= 0x400f6a7a && (ix & 0xfffff) != 0x921fb) {  // |x| ~<= 5pi/4, not ~pi/2 or ~pi
        if (ix <= 0x4002d97c) {                            // |x| ~<= 3pi/4
            double z;
            if (!sign) {
                z = x - pio2_1;
                y[0] = z - pio2_1t;
                y[1] = (z - y[0]) - pio2_1t;
                return 1;
            }
            z = x + pio2_1;
            y[0] = z + pio2_1t;
            y[1] = (z - y[0]) + pio2_1t;
            return -1;
        }
        double z;
        if (!sign) {
            z = x - 2 * pio2_1;
            y[0] = z - 2 * pio2_1t;
            y[1] = (z - y[0]) - 2 * pio2_1t;
            return 2;
        }
        z = x + 2 * pio2_1;
        y[0] = z + 2 * pio2_1t;
        y[1] = (z - y[0]) + 2 * pio2_1t;
        return -2;
    }
    // medium case (the ~pi/2 / ~pi cancellation cases come here too)
    double fn = x * invpio2 + toint - toint;
    int n = (int)fn;
    double r = x - fn * pio2_1, w = fn * pio2_1t;
    if (r - w < -pio4) {
        n--, fn--;
        r = x - fn * pio2_1;
        w = fn * pio2_1t;
    } else if (r - w > pio4) {
        n++, fn++;
        r = x - fn * pio2_1;
        w = fn * pio2_1t;
    }
    y[0] = r - w;
    const int ex = (int)(ix >> 20);
    int ey = (int)((bits(y[0]) >> 52) & 0x7ff);
    if (ex - ey > 16) {
        double t = r;
        w = fn * pio2_2;
        r = t - w;
        w = fn * pio2_2t - ((t - r) - w);
        y[0] = r - w;
        ey = (int)((bits(y[0]) >> 52) & 0x7ff);
        if (ex - ey > 49) {
            t = r;
            w = fn * pio2_3;
            r = t - w;
            w = fn * pio2_3t - ((t - r) - w);
            y[0] = r - w;
        }
    }
    y[1] = (r - y[0]) - w;
    return n;
}

inline double cos(double x) {
    const uint32_t ix = (uint32_t)(bits(x) >> 32) & 0x7fffffffu;
    if (ix <= 0x3fe921fb) return ix < 0x3e46a09e ? 1.0 : k_cos(x, 0.0);
    double y[2];
    switch (rem_pio2(x, y) & 3) {
    case 0: return k_cos(y[0], y[1]);
    case 1: return -k_sin(y[0], y[1], 1);
    case 2: return -k_cos(y[0], y[1]);
    default: return k_sin(y[0], y[1], 1);
    }
}

inline double sin(double x) {
    const uint32_t ix = (uint32_t)(bits(x) >> 32) & 0x7fffffffu;
    if (ix <= 0x3fe921fb) return ix < 0x3e500000 ? x : k_sin(x, 0.0, 0);
    double y[2];
    switch (rem_pio2(x, y) & 3) {
    case 0: return k_sin(y[0], y[1], 1);
    case 1: return k_cos(y[0], y[1]);
    case 2: return -k_sin(y[0], y[1], 1);
    default: return -k_cos(y[0], y[1]);
    }
}

}  // namespace fdlibm

inline double trig_cos(double x, int source) { return source == 1 ? fdlibm::cos(x) : std::cos(x); }
inline double trig_sin(double x, int source) { return source == 1 ? fdlibm::sin(x) : std::sin(x); }

// KlemsaProcessor.new twisting factors (fft.zig:92-106).
inline void twist_table(uint32_t N, std::vector<double> &re, std::vector<double> &im, int source = 0) {
    re.resize(N / 2);
    im.resize(N / 2);
    double unit = kPi / (double)N;
    for (uint32_t i = 0; i < N / 2; i++) {
        double a = (double)i * unit;
        re[i] = trig_cos(a, source);
        im[i] = trig_sin(a, source);
    }
}

// radix2FFT recurrence twiddles w_j per stage (fft.zig:590-616); entry
// len/2 - 1 + j for stage len = 2..N/2.
inline void stage_twiddles(uint32_t N, bool inverse, std::vector<double> &re, std::vector<double> &im,
                           int source = 0) {
    size_t n = N / 2;
    re.assign(n - 1, 0.0);
    im.assign(n - 1, 0.0);
    for (size_t len = 2; len <= n; len *= 2) {
        double angle = inverse ? 2.0 * kPi / (double)len : -2.0 * kPi / (double)len;
        double wr = trig_cos(angle, source), wi = trig_sin(angle, source);
        double w_re = 1.0, w_im = 0.0;
        for (size_t j = 0; j < len / 2; j++) {
            re[len / 2 - 1 + j] = w_re;
            im[len / 2 - 1 + j] = w_im;
            double temp = w_re * wr - w_im * wi;
            w_im = w_re * wi + w_im * wr;
            w_re = temp;
        }
    }
}

}  // namespace host
}  // namespace tfhe
