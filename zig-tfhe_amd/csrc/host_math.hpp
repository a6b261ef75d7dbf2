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

// KlemsaProcessor.new twisting factors (fft.zig:92-106), glibc cos/sin.
inline void twist_table(uint32_t N, std::vector<double> &re, std::vector<double> &im) {
    re.resize(N / 2);
    im.resize(N / 2);
    double unit = kPi / (double)N;
    for (uint32_t i = 0; i < N / 2; i++) {
        double a = (double)i * unit;
        re[i] = std::cos(a);
        im[i] = std::sin(a);
    }
}

// radix2FFT recurrence twiddles w_j per stage (fft.zig:590-616); entry
// len/2 - 1 + j for stage len = 2..N/2.
inline void stage_twiddles(uint32_t N, bool inverse, std::vector<double> &re, std::vector<double> &im) {
    size_t n = N / 2;
    re.assign(n - 1, 0.0);
    im.assign(n - 1, 0.0);
    for (size_t len = 2; len <= n; len *= 2) {
        double angle = inverse ? 2.0 * kPi / (double)len : -2.0 * kPi / (double)len;
        double wr = std::cos(angle), wi = std::sin(angle);
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
