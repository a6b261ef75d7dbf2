// tfhe_device.hpp — device building blocks of the TFHE gate-bootstrap path,
// shared by the product kernel units (tfhe_kernels.hip, tfhe_kernels_whole.hip)
// and the A/B unit under tools/ab/.  Not installed.
//
// Hot path: trgsw.blindRotate (trgsw.zig:290-333) -> cmux (:260-284) ->
// externalProductWithFft (:111-154) over the negacyclic f64 FFT
// (fft.zig:293-443), then sampleExtractIndex (trlwe.zig:146-162) and
// identityKeySwitching (trgsw.zig:471-502).
//
// Bit-exactness contract.  Two arithmetics, selected per
// instantiation (template parameter FU):
//  - reference trees (FU = false; UINT4 always, every set under
//    TFHE_ARITH_REFERENCE, the near-tie recompute): every f64 operation of the
//    reference with the same operands, the same expression tree and
//    round-to-nearest; the compiler never contracts (file-wide
//    `fp contract(off)` plus -ffp-contract=off);
//  - fused (FU = true; the default at the L=3 / Bg=2^6 sets): explicit fused
//    multiply-adds (fmad below, __builtin_fma) in the reference's operation
//    order, with a margin guard on every rounding: an item that rounds a fused
//    value 1/4 or more off its integer is recomputed in the reference trees
//    (torus_from_f64_guarded, launch_br_recompute), so both give the
//    reference's integers.
// The key switch (k_key_switch_gemm, the default form) is integer-exact: a
// one-hot int8 GEMM on the matrix cores.
// Twiddles are uploaded from the host (never sin/cos on the device).  Exact
// power-of-two rescalings (×2 in ifft1024, ×0.5 in fmaInFd1024 and fft1024)
// are folded, which leaves every result bit-identical.
//
// FFT mapping: one wavefront owns one 512-point complex transform (N=1024
// negacyclic), 8 complex values per lane, three radix-2^3 register passes
// (each pass = three radix-2 DIT stages with the reference's butterflies and
// recurrence twiddles) and two conflict-free LDS exchanges.
// Lane t always owns coefficients / frequencies {t + 64q}, so the forward
// output feeds the MAC and the inverse input with no data movement, and the
// accumulator update is lane-local.
#pragma once

#include <hip/hip_runtime.h>

#include "tfhe_internal.hpp"

#pragma clang fp contract(off)

namespace tfhe {

#define DEV __device__ __forceinline__

// Development-only phase timing of the blind-rotation kernels (tools/phase_prof.hip
// defines TFHE_PHASE_PROF, which makes the library an A/B build that
// tfhe_gpu_create refuses by default): s_memtime deltas per phase, summed per
// wave and added to g_phase_cycles at the end.  Compiles to nothing otherwise.
// TFHE_PHASE_PROF=2 is the clock probe: no per-phase marks (they drain the LDS
// queue and slow the kernel), only the wave's s_memtime (core clock) and
// s_memrealtime (100 MHz) deltas from start() to flush(), so the kernel runs as
// unprofiled and the ratio is the clock it held (tools/phase_prof.hip clock).
struct PhaseProf {
#ifdef TFHE_PHASE_PROF
    uint64_t last;
    int cur;
    uint64_t acc[16];
#if TFHE_PHASE_PROF == 2
    uint64_t real0;
    DEV void start() {
        real0 = __builtin_amdgcn_s_memrealtime();
        last = __builtin_amdgcn_s_memtime();
    }
    DEV void mark(int) {}
    // dst[0] += core-clock ticks, dst[1] += 1 wave, dst[2] += 100 MHz ticks
    DEV void flush(unsigned long long *dst, int) {
        const uint64_t now = __builtin_amdgcn_s_memtime(), real = __builtin_amdgcn_s_memrealtime();
        atomicAdd(dst, (unsigned long long)(now - last));
        atomicAdd(dst + 1, 1ull);
        atomicAdd(dst + 2, (unsigned long long)(real - real0));
    }
#else
    DEV void start() {
        cur = 0;
        for (int k = 0; k < 16; k++) acc[k] = 0;
        last = __builtin_amdgcn_s_memtime();
    }
    DEV void mark(int k) {
        const uint64_t now = __builtin_amdgcn_s_memtime();
        acc[cur] += now - last;
        last = now;
        cur = k;
    }
    DEV void flush(unsigned long long *dst, int nq) {
        for (int q = 0; q < nq; q++) atomicAdd(dst + q, (unsigned long long)acc[q]);
    }
#endif
#else
    DEV void start() {}
    DEV void mark(int) {}
#endif
};
#ifdef TFHE_PHASE_PROF
__device__ unsigned long long g_phase_cycles[128];  // [wave][phase < 16] for the wide form
#endif

DEV C2 c2(double x, double y) {
    C2 r;
    r.x = x;
    r.y = y;
    return r;
}

// Complex.mul (fft.zig:50-55) by a forward twiddle; INV: by the inverse
// table, which is the exact conjugate of the forward one (checked on the host
// at table upload), written as the identical IEEE expression tree.
template <bool INV>
DEV C2 twmul(C2 a, C2 w) {
    if (!INV) return c2(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x);
    return c2(a.x * w.x + a.y * w.y, a.y * w.x - a.x * w.y);
}

// Fused arithmetic (FU = true).  At the L=3 / Bg=2^6 sets the
// exact external product is an integer polynomial and the reference's f64
// evaluation stays within ~0.09 of it (oracle_take_round_error), so any
// evaluation with an error below 1/2 rounds to the same integers.  FU kernels
// evaluate every complex multiply-add with fused multiply-adds, in the
// reference's operation order with the reference's twiddles: a butterfly is
// a = u + x*w (two fma) and b = 2u - a (one fma), 6 ops instead of 10; a MAC
// term is two fma per component.  The oracle's fused mode (oracle_set_fused)
// restates exactly these expressions.  Never used where products exceed 2^53
// (UINT4: SMALL = false), where the reference's rounding is the result.
DEV double fmad(double a, double b, double c) { return __builtin_fma(a, b, c); }

// radix2FFT inner butterfly (fft.zig:600-606)
template <bool INV, bool FU = false>
DEV void bf(C2 &u, C2 &x, C2 w) {
    if (FU) {  // x*w for the forward twiddle, x*conj(w) for INV
        const double ax = INV ? fmad(x.x, w.x, fmad(x.y, w.y, u.x)) : fmad(x.x, w.x, fmad(-x.y, w.y, u.x));
        const double ay = INV ? fmad(-x.x, w.y, fmad(x.y, w.x, u.y)) : fmad(x.x, w.y, fmad(x.y, w.x, u.y));
        x = c2(fmad(2.0, u.x, -ax), fmad(2.0, u.y, -ay));
        u = c2(ax, ay);
        return;
    }
    C2 v = twmul<INV>(x, w);
    C2 a = c2(u.x + v.x, u.y + v.y);
    C2 b = c2(u.x - v.x, u.y - v.y);
    u = a;
    x = b;
}
// j == 0 butterfly: the recurrence twiddle is exactly (1, 0); x*(1,0) == x up
// to the sign of zero, which never reaches an output integer.  FU: a = u + x
// is the fused form's a exactly, b = 2u - a as in every fused butterfly.
template <bool FU = false>
DEV void bf1(C2 &u, C2 &x) {
    if (FU) {
        const C2 a = c2(u.x + x.x, u.y + x.y);
        x = c2(fmad(2.0, u.x, -a.x), fmad(2.0, u.y, -a.y));
        u = a;
        return;
    }
    C2 a = c2(u.x + x.x, u.y + x.y);
    C2 b = c2(u.x - x.x, u.y - x.y);
    u = a;
    x = b;
}

// Butterfly with a twiddle whose imaginary part is exactly -1.0 in the
// forward table (W4[1] and W8[2] of the recurrence; checked on the host when
// the tables are built, tfhe_gpu.cpp): x.y * -1.0 == -x.y exactly, so the
// reference's products by w.y are sign flips folded into the adds.  Same
// results as bf<INV>(u, x, (wx, -1.0)) bit for bit, two multiplies fewer.
template <bool INV, bool FU = false>
DEV void bf_m1(C2 &u, C2 &x, double wx) {
    if (FU) {  // the fused butterfly with w.y = -1: x.y * -1 and x.x * -1 are exact
        const double ax = INV ? fmad(x.x, wx, u.x - x.y) : fmad(x.x, wx, u.x + x.y);
        const double ay = INV ? fmad(x.y, wx, u.y) + x.x : fmad(x.y, wx, u.y) - x.x;
        x = c2(fmad(2.0, u.x, -ax), fmad(2.0, u.y, -ay));
        u = c2(ax, ay);
        return;
    }
    const C2 v = INV ? c2(x.x * wx - x.y, x.y * wx + x.x) : c2(x.x * wx + x.y, x.y * wx - x.x);
    C2 a = c2(u.x + v.x, u.y + v.y);
    C2 b = c2(u.x - v.x, u.y - v.y);
    u = a;
    x = b;
}

DEV int br3(int q) { return ((q & 1) << 2) | (q & 2) | ((q >> 2) & 1); }
DEV int br6(int t) { return (int)(__builtin_bitreverse32((uint32_t)t) >> 26); }

// Stage twiddles.  Table index of stage len, j: len/2 - 1 + j.
//   pass A (len 4, 8):     W4[1], W8[1..3]                   lane-uniform
//   pass B (len 16..64):   W16[r], W32[r + 8k], W64[r + 8k]  r = t & 7
//   pass C (len 128..512): W128[t], W256[t+64k], W512[t+64k]
// Two providers: RegTw keeps all of them in registers (single-wave stage
// kernels), LdsTw reads passes B/C from a block-shared LDS copy of the table
// when a pass starts (blind rotation: frees ~60 VGPRs per lane).
DEV void tw_pass_b(C2 *w, const C2 *tw, int t) {
    const int r = t & 7;
    w[0] = tw[7 + r];
    w[1] = tw[15 + r];
    w[2] = tw[15 + r + 8];
#pragma unroll
    for (int k = 0; k < 4; k++) w[3 + k] = tw[31 + r + 8 * k];
}
DEV void tw_pass_c(C2 *w, const C2 *tw, int t) {
    w[0] = tw[63 + t];
    w[1] = tw[127 + t];
    w[2] = tw[127 + t + 64];
#pragma unroll
    for (int k = 0; k < 4; k++) w[3 + k] = tw[255 + t + 64 * k];
}

struct RegTw {
    C2 a[4], b[7], c[7];
    DEV void init(const C2 *__restrict__ tw, int t) {
        a[0] = tw[2];
        a[1] = tw[4];
        a[2] = tw[5];
        a[3] = tw[6];
        tw_pass_b(b, tw, t);
        tw_pass_c(c, tw, t);
    }
    DEV void pass_b(C2 *w, int) const {
#pragma unroll
        for (int k = 0; k < 7; k++) w[k] = b[k];
    }
    DEV void pass_c(C2 *w, int) const {
#pragma unroll
        for (int k = 0; k < 7; k++) w[k] = c[k];
    }
};

struct LdsTw {
    C2 a[4];
    const C2 *tw;  // LDS copy of the stage table
    DEV void init(const C2 *lds_tw) {
        tw = lds_tw;
        a[0] = tw[2];
        a[1] = tw[4];
        a[2] = tw[5];
        a[3] = tw[6];
    }
    // pass-A twiddles are lane-uniform: kernel-argument copies keep them in
    // SGPRs (VALU f64 ops take one SGPR-pair operand), not 16 VGPRs
    DEV void init(const C2 *lds_tw, const DevTables &TT) {
        tw = lds_tw;
        for (int k = 0; k < 4; k++) a[k] = TT.twa[k];
    }
    DEV void pass_b(C2 *w, int t) const { tw_pass_b(w, tw, t); }
    DEV void pass_c(C2 *w, int t) const { tw_pass_c(w, tw, t); }
};

// LdsTw whose table reads stay at their pass (an opaque pointer per read): with
// many transforms per step hipcc otherwise hoists the loop-invariant twiddles of
// passes B and C out of the step loop, 56 VGPRs held for the whole launch (the
// octo form spilled).
struct LdsTwAtPass : LdsTw {
    DEV void pass_b(C2 *w, int t) const {
        const C2 *p = tw;
        asm volatile("" : "+v"(p));
        tw_pass_b(w, p, t);
    }
    DEV void pass_c(C2 *w, int t) const {
        const C2 *p = tw;
        asm volatile("" : "+v"(p));
        tw_pass_c(w, p, t);
    }
};

// Pass A: stages len = 2, 4, 8 (bits 0-2 of the bit-reversed position are the
// register index q).
template <bool INV, bool FU = false>
DEV void passA(C2 *d, const C2 *a) {
    bf1<FU>(d[0], d[1]); bf1<FU>(d[2], d[3]); bf1<FU>(d[4], d[5]); bf1<FU>(d[6], d[7]);
    bf1<FU>(d[0], d[2]); bf_m1<INV, FU>(d[1], d[3], a[0].x); bf1<FU>(d[4], d[6]); bf_m1<INV, FU>(d[5], d[7], a[0].x);
    bf1<FU>(d[0], d[4]); bf<INV, FU>(d[1], d[5], a[1]); bf_m1<INV, FU>(d[2], d[6], a[2].x); bf<INV, FU>(d[3], d[7], a[3]);
}
// Pass B: stages 16, 32, 64 (position bits 3-5 in q; j = (t&7) + 8*(...)).
// Pass C: stages 128, 256, 512 (position bits 6-8 in q; j = t + 64*(...)).
// w = {W_s1, W_s2[0..1], W_s3[0..3]} of the pass's three stages.
template <bool INV, bool FU = false>
DEV void passBC(C2 *d, const C2 *w) {
    bf<INV, FU>(d[0], d[1], w[0]); bf<INV, FU>(d[2], d[3], w[0]); bf<INV, FU>(d[4], d[5], w[0]); bf<INV, FU>(d[6], d[7], w[0]);
    bf<INV, FU>(d[0], d[2], w[1]); bf<INV, FU>(d[1], d[3], w[2]); bf<INV, FU>(d[4], d[6], w[1]); bf<INV, FU>(d[5], d[7], w[2]);
    bf<INV, FU>(d[0], d[4], w[3]); bf<INV, FU>(d[1], d[5], w[4]); bf<INV, FU>(d[2], d[6], w[5]); bf<INV, FU>(d[3], d[7], w[6]);
}

// Exchange 1 (after pass A): lane t wrote positions 8*br6(t)+q, reads
// (t&7) + 8q + 64(t>>3).  XOR swizzle of the 16-B slot makes both the
// ds_write_b128 and the ds_read_b128 bank-conflict-free.
DEV int swz1(int p) {
    return p ^ ((((p >> 6) & 1) * 1) ^ (((p >> 7) & 1) * 10) ^ (((p >> 8) & 1) * 4));
}

// Exchanges go through a wave-private LDS region: the LDS executes one
// wave's DS instructions in issue order, so a wavefront-scope fence (which
// only stops the compiler from reordering; no s_waitcnt, no s_barrier) is
// the whole synchronisation.
DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int NF>
DEV void exchange1(C2 (*d)[8], C2 *xb, int t) {
    int wb = 8 * br6(t);
#pragma unroll
    for (int f = 0; f < NF; f++)
#pragma unroll
        for (int q = 0; q < 8; q++) xb[f * 512 + swz1(wb + q)] = d[f][q];
    wave_sync();
    int rb = (t & 7) + 64 * (t >> 3);
#pragma unroll
    for (int f = 0; f < NF; f++)
#pragma unroll
        for (int q = 0; q < 8; q++) d[f][q] = xb[f * 512 + swz1(rb + 8 * q)];
    wave_sync();
}

// Exchange 2 in registers, for the single-transform fft512 (latency form, stage
// kernels):
// the latency form's 16-bit adder 114.5 -> 111.9 ms, the pair form 8.31 -> 7.99
// ms.  The pipelined pair of the whole form (fft512_x2) keeps the LDS exchange,
// which its other transform's butterflies hide: 7.52 vs 7.75 ms with registers
// (profiles/r02_ab_exchange2.txt).
// Lane t = 8a + b holds positions b + 8q + 64a (q < 8) after pass B; pass C
// needs lane 8q + b to hold it in register a: an 8 x 8 transpose of (lane bits
// 3-5, register bits 0-2) among the 8 lanes sharing b, done as three swap
// rounds, one per bit pair: lane bit 5 <-> register bit 2 by
// v_permlane32_swap, lane bit 4 <-> bit 1 by v_permlane16_swap, lane bit 3 <->
// bit 0 by two bank-masked DPP row_ror:8 moves.  Pure data movement: the same
// values as the LDS exchange, 80 VALU moves instead of 8 ds_write_b128 + 8
// ds_read_b128 (a ds_write_b128 holds the CU's LDS write path ~13 cycles).
DEV void c2_words(const C2 &v, uint32_t *w) {
    w[0] = (uint32_t)__double2loint(v.x);
    w[1] = (uint32_t)__double2hiint(v.x);
    w[2] = (uint32_t)__double2loint(v.y);
    w[3] = (uint32_t)__double2hiint(v.y);
}
DEV C2 c2_from_words(const uint32_t *w) {
    return c2(__hiloint2double((int)w[1], (int)w[0]), __hiloint2double((int)w[3], (int)w[2]));
}
template <int ROUND>
DEV void swap_lane_reg(C2 &x, C2 &y) {  // x: register bit clear, y: set
    uint32_t a[4], b[4];
    c2_words(x, a);
    c2_words(y, b);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (ROUND == 2) {  // x's lanes 32-63 <-> y's lanes 0-31
            const auto r = __builtin_amdgcn_permlane32_swap(a[k], b[k], false, false);
            a[k] = r[0];
            b[k] = r[1];
        } else if (ROUND == 1) {  // x's odd 16-lane rows <-> y's even rows
            const auto r = __builtin_amdgcn_permlane16_swap(a[k], b[k], false, false);
            a[k] = r[0];
            b[k] = r[1];
        } else {  // lane bit 3: y's lanes with bit 3 clear <- x's (lane ^ 8); x's with bit 3 set <- old y's
            const uint32_t old_b = b[k];
            b[k] = (uint32_t)__builtin_amdgcn_update_dpp((int)b[k], (int)a[k], 0x128, 0xf, 0x3, false);
            a[k] = (uint32_t)__builtin_amdgcn_update_dpp((int)a[k], (int)old_b, 0x128, 0xf, 0xc, false);
        }
    }
    x = c2_from_words(a);
    y = c2_from_words(b);
}
DEV void ex2_regs(C2 *d) {
    swap_lane_reg<2>(d[0], d[4]); swap_lane_reg<2>(d[1], d[5]); swap_lane_reg<2>(d[2], d[6]); swap_lane_reg<2>(d[3], d[7]);
    swap_lane_reg<1>(d[0], d[2]); swap_lane_reg<1>(d[1], d[3]); swap_lane_reg<1>(d[4], d[6]); swap_lane_reg<1>(d[5], d[7]);
    swap_lane_reg<0>(d[0], d[1]); swap_lane_reg<0>(d[2], d[3]); swap_lane_reg<0>(d[4], d[5]); swap_lane_reg<0>(d[6], d[7]);
}

template <int NF, bool LDS = false>
DEV void exchange2(C2 (*d)[8], C2 *xb, int t) {
    if (!LDS) {
#pragma unroll
        for (int f = 0; f < NF; f++) ex2_regs(d[f]);
        return;
    }
    int wb = (t & 7) + 64 * (t >> 3);
#pragma unroll
    for (int f = 0; f < NF; f++)
#pragma unroll
        for (int q = 0; q < 8; q++) xb[f * 512 + wb + 8 * q] = d[f][q];
    wave_sync();
#pragma unroll
    for (int f = 0; f < NF; f++)
#pragma unroll
        for (int q = 0; q < 8; q++) d[f][q] = xb[f * 512 + t + 64 * q];
    wave_sync();
}

// 512-point radix-2 DIT (bitReverseRadix2 + radix2FFT, fft.zig:582-669) on NF
// transforms at once.  In: d[f][q] = z[t + 64*br3(q)] (the bit reversal is
// absorbed into the load order).  Out: d[f][q] = Z[t + 64q].
// Exchange halves for one transform: write its registers to its region
// (xb already offset to it), or read the next layout back.
DEV void ex1_write(const C2 *d, C2 *xb, int t) {
    const int wb = 8 * br6(t);
#pragma unroll
    for (int q = 0; q < 8; q++) xb[swz1(wb + q)] = d[q];
}
DEV void ex1_read(C2 *d, const C2 *xb, int t) {
    const int rb = (t & 7) + 64 * (t >> 3);
#pragma unroll
    for (int q = 0; q < 8; q++) d[q] = xb[swz1(rb + 8 * q)];
}
DEV void ex2_write(const C2 *d, C2 *xb, int t) {
    const int wb = (t & 7) + 64 * (t >> 3);
#pragma unroll
    for (int q = 0; q < 8; q++) xb[wb + 8 * q] = d[q];
}
DEV void ex2_read(C2 *d, const C2 *xb, int t) {
#pragma unroll
    for (int q = 0; q < 8; q++) d[q] = xb[t + 64 * q];
}

// Two independent transforms, software-pipelined so that each transform's
// LDS exchange (write burst, in-order read-back) overlaps the other one's
// butterfly pass: the wave always has VALU work while its DS queue drains.
// Same arithmetic as fft512<2, INV>.
// ONEBUF: both transforms exchange through one 8 KB buffer.  Every write
// into it follows, in this wave's program order, the reads of the data it
// overwrites, and one wave's LDS operations execute in order.
// hipcc's one s_waitcnt per consumed LDS read lets each butterfly start as soon
// as its own operand lands; one explicit wait per read group measured slower
// (6.10-6.11 vs 6.07 ms, profiles/r04_ab_x2_waits.txt).  Exchange 2 in
// registers here measured slower too (7.75 vs 7.52 ms, profiles/r02_ab_exchange2.txt).
template <bool INV, bool ONEBUF = false, bool FU = false, class TW>
DEV void fft512_x2(C2 (*d)[8], C2 *xb, const TW &T, int t) {
    C2 *x0 = xb, *x1 = ONEBUF ? xb : xb + 512;
    C2 wb_[7], wc_[7];
    passA<INV, FU>(d[0], T.a);
    ex1_write(d[0], x0, t);
    wave_sync();
    passA<INV, FU>(d[1], T.a);
    ex1_read(d[0], x0, t);
    ex1_write(d[1], x1, t);
    wave_sync();
    T.pass_b(wb_, t);
    passBC<INV, FU>(d[0], wb_);
    ex1_read(d[1], x1, t);
    ex2_write(d[0], x0, t);
    wave_sync();
    passBC<INV, FU>(d[1], wb_);
    T.pass_c(wc_, t);
    ex2_read(d[0], x0, t);
    ex2_write(d[1], x1, t);
    wave_sync();
    passBC<INV, FU>(d[0], wc_);
    ex2_read(d[1], x1, t);
    wave_sync();
    passBC<INV, FU>(d[1], wc_);
}

template <int NF, bool INV, bool FU = false, class TW, bool EX2LDS = false>
DEV void fft512(C2 (*d)[8], C2 *xb, const TW &T, int t) {
#pragma unroll
    for (int f = 0; f < NF; f++) passA<INV, FU>(d[f], T.a);
    exchange1<NF>(d, xb, t);
    {
        C2 w[7];
        T.pass_b(w, t);
#pragma unroll
        for (int f = 0; f < NF; f++) passBC<INV, FU>(d[f], w);
    }
    exchange2<NF, EX2LDS>(d, xb, t);
    {
        C2 w[7];
        T.pass_c(w, t);
#pragma unroll
        for (int f = 0; f < NF; f++) passBC<INV, FU>(d[f], w);
    }
}

// Fold + twist of ifft1024 (fft.zig:301-323): z = (x_re, x_im) * twist.
template <bool FU = false>
DEV C2 twist_in(double xr, double xi, C2 w) {
    if (FU) return c2(fmad(xr, w.x, -(xi * w.y)), fmad(xr, w.y, xi * w.x));
    return c2(xr * w.x - xi * w.y, xr * w.y + xi * w.x);
}

// Untwist + normalisation of fft1024 (fft.zig:412-429).  `f` is 2x the
// reference's value (the ×0.5 input scaling is folded), hence 1/(2*512).
// NORM = false: the 2^-10 is already in `f` because the device BK is stored
// scaled by 2^-10 (k_bk_permute); a power-of-two factor commutes with every
// rounded add and multiply of the MAC, the inverse FFT and the untwist (no
// overflow or subnormal at these magnitudes), so the results are identical.
template <bool NORM = true, bool FU = false>
DEV void untwist_out(C2 f, C2 w, double &tr, double &ti) {
    const double norm = 1.0 / 1024.0;
    if (FU) {
        tr = fmad(f.x, w.x, f.y * w.y);
        ti = fmad(f.y, w.x, -(f.x * w.y));
    } else {
        tr = f.x * w.x + f.y * w.y;
        ti = f.y * w.x - f.x * w.y;
    }
    if (NORM) {
        tr = tr * norm;
        ti = ti * norm;
    }
}

// @round (half away from zero) -> i64 -> @truncate i32 -> u32 == r mod 2^32,
// computed exactly in f64 for any finite r.  |r| >= 2^63 (or NaN) is
// undefined in the reference (@intFromFloat out of range); on the x86-64
// platform the oracle defines parity on, cvttsd2si yields
// 0x8000000000000000, whose low word is 0 — reproduced here.  Never reached
// by bootstrap inputs (|r| < 2^53 there).
DEV uint32_t torus_from_f64(double v) {
    double r = round(v);
    double hi = floor(r * (1.0 / 4294967296.0));
    double lo = r - hi * 4294967296.0;
    return fabs(r) < 9223372036854775808.0 ? (uint32_t)lo : 0u;
}

// Same result in 8 VALU ops when |v| < 2^51 is guaranteed by the parameter
// set (|ExtProd| <= 2L * N * Bg/2 * 2^31; 2^47.6 at L=3, Bg=2^6): trunc,
// then t + 1.5*2^52 is exact and its low mantissa word is t mod 2^32.
DEV uint32_t torus_from_f64_small(double v) {
    const double t = trunc(v);
    const double frac = v - t;                // exact, |frac| < 1, sign of v
    const double adj = trunc(frac + frac);    // exact: +-1 iff |frac| >= 0.5 (half away from zero), else 0
    const double s = (t + adj) + 6755399441055744.0;  // exact integers < 2^51, then 1.5*2^52
    return (uint32_t)__double_as_longlong(s);
}

// Fused kernels (FU, the exact-integer regime of DESIGN.md §6.1), with the
// margin guard.  The fused value v and the reference's value differ by less
// than 1/4 (measured max 0.094 at the largest magnitude a keygen'd key admits,
// DESIGN.md §6.1), so wherever v is within 1/4 of an integer both round to
// that integer.  One add rounds v + 0.5 to a multiple of 1/2:
// s = v + (1.5*2^51 + 0.5) (|v| < 2^49), whose mantissa is 2^51 + Q with
// Q = rint(2v + 1).  Q odd <=> |v - rint(v)| < 1/4, and then Q >> 1 (mantissa
// bits 32..1, one v_alignbit) is rint(v).  `near` ANDs the low words over the
// launch (one v_bitop3 per two values); bit 0 clear sends the item to the
// reference-tree recompute (near_tie_flag, k_blind_rotate FALLBACK), which
// replaces every word of the item.
// A/B build only (TFHE_GUARD_EIGHTH, round 6): the guard at 1/8.
// s = v + (1.5*2^50 + 3/4) (|v| < 2^49) has mantissa 2^51 + Q, Q = rint(4v + 3):
// Q mod 4 == 3 <=> |v - rint(v)| < 1/8, and then Q >> 2 (bits 33..2) is rint(v).  Same
// instruction count; the margin to the reference becomes 3/8.  Not the product's: honest
// rotations reach 1/8 about once per 10^10 values, i.e. a recompute
// launch in a sizeable fraction of 1,024-gate batches.
#ifdef TFHE_GUARD_EIGHTH
#ifndef TFHE_AB_BUILD
#error "TFHE_GUARD_EIGHTH is an A/B-build switch (Makefile EXTRA, tools/ab_forms.sh)"
#endif
constexpr uint32_t NEAR_MASK = 3u;
DEV uint32_t torus_from_f64_guarded(double v, uint32_t &near) {
    const uint64_t b = (uint64_t)__double_as_longlong(v + 1688849860263936.75);
    const uint32_t lo = (uint32_t)b, hi = (uint32_t)(b >> 32);
    near &= lo;
    return __builtin_amdgcn_alignbit(hi, lo, 2);
}
#else
constexpr uint32_t NEAR_MASK = 1u;
DEV uint32_t torus_from_f64_guarded(double v, uint32_t &near) {
    const uint64_t b = (uint64_t)__double_as_longlong(v + 3377699720527872.5);
    const uint32_t lo = (uint32_t)b, hi = (uint32_t)(b >> 32);
    near &= lo;
    return __builtin_amdgcn_alignbit(hi, lo, 1);
}
#endif

template <bool SMALL, bool FU = false>
DEV uint32_t to_torus(double v, uint32_t &near) {
    if (FU) return torus_from_f64_guarded(v, near);
    return SMALL ? torus_from_f64_small(v) : torus_from_f64(v);
}
// Initial value of a `near` accumulator: no value off its integer by 1/4 or more.
constexpr uint32_t NEAR_NONE = ~0u;
// End of a fused item: if any lane of this wave rounded near a tie, flag item g
// (one byte, a vector store; the flag is rare, the ballot is one SALU compare).
DEV void near_tie_flag(const KParams &P, uint32_t near, size_t g, bool valid) {
    if (__builtin_amdgcn_ballot_w64((near & NEAR_MASK) != NEAR_MASK) != 0 && valid && P.tie_flags && (threadIdx.x & 63) == 0)
        P.tie_flags[g] = 1;
}

// decompositionIntoStorage digit (trgsw.zig:207-217); `x` already has the
// decomposition offset added.
DEV double digit_f64(uint32_t x, int level, int bgbit) {
    uint32_t d = ((x >> (32 - (level + 1) * bgbit)) & ((1u << bgbit) - 1u)) - (1u << (bgbit - 1));
    return (double)(int32_t)d;
}

// The whole and octo forms keep tmp words with the top bit of every
// decomposition field flipped (x ^ digit_msbs): the signed bgbit-bit field of
// x ^ (Bg/2 << s) is ((x >> s) & (Bg - 1)) - Bg/2, digit_f64's digit, in one
// v_bfe_i32 instead of a shift, a mask and a subtract (flipping a field's top
// bit adds Bg/2 modulo Bg; the signed read maps [Bg/2, Bg) to [-Bg/2, 0)).
DEV uint32_t digit_msbs(int L, int bgbit) {
    uint32_t m = 0;
    for (int l = 0; l < L; l++) m |= 1u << (31 - l * bgbit);
    return m;
}
DEV double digit_f64_flipped(uint32_t xf, int level, int bgbit) {
    return (double)(int32_t)__builtin_amdgcn_sbfe(xf, 32 - (level + 1) * bgbit, bgbit);
}

// tmp word of the rotation gather, flipped: ((neg ? -v : v) - acc + offset) ^ msbs
// with s = neg ? ~0 : 0 and off_s = offset - s, since (v ^ s) - s = (neg ? -v : v).
DEV uint32_t tmp_word(uint32_t v, uint32_t s, uint32_t off_s, uint32_t acc, uint32_t msbs) {
    return ((v ^ s) + (off_s - acc)) ^ msbs;
}

// Rotation gather (polyMulWithXK, trgsw.zig:442-466) from an accumulator copy in
// LDS at a 4 KB-aligned byte address `base` (a at words [0, 1024), b at
// [1024, 2048)): lane word m is coefficient t + 64m, at byte index
// xb[m] = 4 ((t - a~) mod 2N) + 256 m; its word is at (xb & 0xFFC) | base (one
// v_and_or) and its negacyclic sign is bit 12 of xb (gather_sign).
typedef __attribute__((address_space(3))) const uint32_t lds_cu32_t;
DEV uint32_t lds_read_u32(uint32_t byte_addr) { return *(lds_cu32_t *)(size_t)byte_addr; }
DEV void gather_rot(uint32_t base, int t, int at, uint32_t *xb, uint32_t *tA, uint32_t *tB) {
    const uint32_t rbb = (uint32_t)((t - at) & 2047) << 2;
    // hipcc splits (x & 0xFFC) | base into v_and + v_or; v_and_or_b32 with the
    // mask in a VGPR (VOP3 takes no literal here, and base is the one SGPR)
    const uint32_t mask = __builtin_amdgcn_readfirstlane(0xFFCu);
    uint32_t vmask;
    asm volatile("v_mov_b32 %0, %1" : "=v"(vmask) : "s"(mask));
#pragma unroll
    for (int m = 0; m < 16; m++) {
        xb[m] = rbb + 256u * m;
        uint32_t a;
        asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(a) : "v"(xb[m]), "v"(vmask), "s"(base));
        tA[m] = lds_read_u32(a);
        tB[m] = lds_read_u32(a + 4096u);
    }
}
DEV uint32_t gather_sign(uint32_t xb) { return (uint32_t)__builtin_amdgcn_sbfe(xb, 12, 1); }

// X^k rotation read (polyMulWithXK, trgsw.zig:442-466) of coefficient k from
// the accumulator polynomial `p` (N=1024) held in LDS, k in [0, 2N].
DEV uint32_t rot_read(const uint32_t *p, int k, int at) {
    int idx = (k - at) & 2047;
    uint32_t v = p[idx & 1023];
    return (idx & 1024) ? 0u - v : v;
}

// Gate pre-combination, gates.zig:48-121 (constants utils.f64ToTorus).
DEV uint32_t gate_combine(int op, uint32_t x, uint32_t y, bool is_b) {
    uint32_t r;
    switch (op) {
    case 0: r = (0u - x) + (0u - y); break;              // NAND
    case 1: case 2: r = x + y; break;                    // OR, AND
    case 3: r = x + y * 2u; break;                       // XOR  (addMul)
    case 4: r = x - y * 2u; break;                       // XNOR (subMul)
    case 5: r = (0u - x) + (0u - y); break;              // NOR
    case 6: case 8: r = (0u - x) + y; break;             // ANDNY, ORNY
    case 7: case 9: r = x - y; break;                    // ANDYN, ORYN
    default: return x;                                   // COPY
    }
    if (is_b) {
        switch (op) {
        case 0: case 1: case 8: case 9: r += 0x20000000u; break;  // +f64ToTorus(0.125)
        case 2: case 5: case 6: case 7: r += 0xE0000000u; break;  // +f64ToTorus(-0.125)
        case 3: r += 0x40000000u; break;                          // +f64ToTorus(0.25)
        case 4: r += 0xC0000000u; break;                          // +f64ToTorus(-0.25)
        default: break;
        }
    }
    return r;
}

// Load an fft512 input (one decomposition row, compile-time) from the
// accumulator difference: src[m] = (rot - acc + offset) at coefficient
// t + 64m, m < 16.  Twist factor of coefficient t + 64m at tws[m * TS].
template <int L, int ROW, int TS>
DEV void load_digits(C2 *d, const uint32_t *srcA, const uint32_t *srcB, int bgbit, const C2 *tws) {
    const uint32_t *src = ROW < L ? srcA : srcB;
    constexpr int level = ROW < L ? ROW : ROW - L;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const int m = br3(q);
        d[q] = twist_in(digit_f64(src[m], level, bgbit), digit_f64(src[m + 8], level, bgbit), tws[m * TS]);
    }
}

// One frequency-domain multiply-accumulate row (fmaInFd1024, trgsw.zig:157-189)
// for both output polynomials.  Device BK row layout: [q][a|b][lane] double2,
// a = (a_re, a_im), b = (b_re, b_im) at frequency t + 64q (16-B lanes: the
// LDS reads are conflict-free ds_read_b128).  FIRST: the reference starts
// from 0.0, and 0.0 + x == x.
template <bool FIRST>
DEV void mac_row(C2 *fa, C2 *fb, const C2 *d, const double2 *bk, int t) {
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const double2 ka = bk[(2 * q) * 64 + t];
        const double2 kb = bk[(2 * q + 1) * 64 + t];
        const C2 ta = c2(d[q].x * ka.x - d[q].y * ka.y, d[q].x * ka.y + d[q].y * ka.x);
        const C2 tb = c2(d[q].x * kb.x - d[q].y * kb.y, d[q].x * kb.y + d[q].y * kb.x);
        if (FIRST) {
            fa[q] = ta;
            fb[q] = tb;
        } else {
            fa[q] = c2(fa[q].x + ta.x, fa[q].y + ta.y);
            fb[q] = c2(fb[q].x + tb.x, fb[q].y + tb.y);
        }
    }
}

// MAC of a row pair from LDS, software-pipelined one frequency group ahead:
// the 4 BK words of group q+1 are read while group q's 32 flops issue, and a
// scheduling fence per group keeps hipcc from hoisting all 32 reads (128
// VGPRs) ahead of the arithmetic, which pushes the kernel into AGPR copies.
template <bool FU = false>
DEV void mac_pair_lds(C2 *fa, C2 *fb, const C2 *d0, const C2 *d1, const double2 *bk, int t,
                      const double2 *k0 = nullptr) {
    double2 k[2][4];
    if (k0) {  // group 0 already read (TFHE_OPT_PUB: with the slot counter)
#pragma unroll
        for (int e = 0; e < 4; e++) k[0][e] = k0[e];
    } else {
        k[0][0] = bk[t];
        k[0][1] = bk[64 + t];
        k[0][2] = bk[1024 + t];
        k[0][3] = bk[1024 + 64 + t];
    }
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const int c = q & 1;
        if (q + 1 < 8) {
            k[c ^ 1][0] = bk[(2 * q + 2) * 64 + t];
            k[c ^ 1][1] = bk[(2 * q + 3) * 64 + t];
            k[c ^ 1][2] = bk[1024 + (2 * q + 2) * 64 + t];
            k[c ^ 1][3] = bk[1024 + (2 * q + 3) * 64 + t];
        }
#pragma unroll
        for (int r = 0; r < 2; r++) {
            const C2 x = r ? d1[q] : d0[q];
            const double2 ka = k[c][2 * r], kb = k[c][2 * r + 1];
            if (FU) {  // acc += x*k: two fma per component (oracle fused fma_in_fd)
                fa[q] = c2(fmad(x.x, ka.x, fmad(-x.y, ka.y, fa[q].x)), fmad(x.x, ka.y, fmad(x.y, ka.x, fa[q].y)));
                fb[q] = c2(fmad(x.x, kb.x, fmad(-x.y, kb.y, fb[q].x)), fmad(x.x, kb.y, fmad(x.y, kb.x, fb[q].y)));
                continue;
            }
            const C2 ta = c2(x.x * ka.x - x.y * ka.y, x.x * ka.y + x.y * ka.x);
            const C2 tb = c2(x.x * kb.x - x.y * kb.y, x.x * kb.y + x.y * kb.x);
            fa[q] = c2(fa[q].x + ta.x, fa[q].y + ta.y);
            fb[q] = c2(fb[q].x + tb.x, fb[q].y + tb.y);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Inverse transforms of the two accumulated spectra (fft1024 x2) and the
// CMUX add acc' = ExtProd + acc (trgsw.zig:277-281), lane-local.
template <bool SMALL, int TS, bool ONEBUF = false, bool FU = false, class TW>
DEV void inverse_and_add(const C2 *fa, const C2 *fb, C2 *xb, const TW &T, const C2 *tws, int t,
                         uint32_t *accA, uint32_t *accB, uint32_t &near) {
    C2 e[2][8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
        e[0][q] = fa[br3(q)];
        e[1][q] = fb[br3(q)];
    }
    // (the untwist factors read before the transforms measured slower: 6.15-6.17
    // vs 6.08-6.10 ms, profiles/r04_ab_early_reads.txt)
    fft512_x2<true, ONEBUF, FU>(e, xb, T, t);
    // four independent near-tie accumulators, joined at the end: one chain
    // would serialise its 32 updates per call (A/B with the round-3 min form,
    // profiles/r03e_guard_chains_lut_octo.txt: guard cost 0.8 % with four chains,
    // 2.2 % with one)
    uint32_t nq[4] = {NEAR_NONE, NEAR_NONE, NEAR_NONE, NEAR_NONE};
#pragma unroll
    for (int q = 0; q < 8; q++) {
        double ra, ia, rb, ib;
        const C2 w = tws[q * TS];
        untwist_out<false, FU>(e[0][q], w, ra, ia);
        untwist_out<false, FU>(e[1][q], w, rb, ib);
        accA[q] += to_torus<SMALL, FU>(ra, nq[0]);
        accA[q + 8] += to_torus<SMALL, FU>(ia, nq[1]);
        accB[q] += to_torus<SMALL, FU>(rb, nq[2]);
        accB[q + 8] += to_torus<SMALL, FU>(ib, nq[3]);
    }
    near &= nq[0] & nq[1] & nq[2] & nq[3];
}

// Forward transforms + MAC of row pair (2RP, 2RP+1) against `bk` (the pair's
// two TRGSW rows in device layout, global or LDS).
template <int L, int RP, int TS, class TW>
DEV void forward_pair(const uint32_t *tA, const uint32_t *tB, int bgbit, const TW &T, const C2 *tws,
                      C2 *xb, int t, C2 (*d)[8]) {
    load_digits<L, 2 * RP, TS>(d[0], tA, tB, bgbit, tws);
    load_digits<L, 2 * RP + 1, TS>(d[1], tA, tB, bgbit, tws);
    fft512_x2<false>(d, xb, T, t);
}

template <int RP>
DEV void mac_pair(C2 *fa, C2 *fb, C2 (*d)[8], const double2 *bk, int t) {
    mac_row<RP == 0>(fa, fb, d[0], bk, t);
    mac_row<false>(fa, fb, d[1], bk + 1024, t);
}

// ExternalProduct(BK row, tmp) for one TRLWE with the BK row read from global
// memory (stage kernel); tmp per lane as (value + offset) at t + 64m.
template <int L, int RP = 0>
DEV void ext_pairs_global(const uint32_t *tA, const uint32_t *tB, const double2 *__restrict__ bkrow, int bgbit,
                          const RegTw &T, const C2 *twl, C2 *xb, int t, C2 *fa, C2 *fb) {
    if constexpr (RP < L) {
        C2 d[2][8];
        forward_pair<L, RP, 1>(tA, tB, bgbit, T, twl, xb, t, d);
        mac_pair<RP>(fa, fb, d, bkrow + (size_t)RP * 2048, t);
        ext_pairs_global<L, RP + 1>(tA, tB, bkrow, bgbit, T, twl, xb, t, fa, fb);
    }
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void global_void_t;

// ---------------------------------------------------------------------------
// Blind rotation, "whole" form (the default): one wavefront per item for all n
// CMUX steps, 4 items per 512-thread workgroup:
//   acc = X^{b~} * testvec;  for i < n: acc = CMUX(BK[i], acc, X^{a~_i} acc)
// then sampleExtractIndex(acc, 0) (TLWELv1) or the TRLWE itself.
// Waves 0-3 are the gate waves; waves 4-7, one beside each gate wave on its
// SIMD, are loader waves that only issue the BK row-pair LDS-DMAs.  The four
// gates consume the same BK rows, so each row pair is brought into LDS once per
// workgroup, two MACs ahead of its use.  FFT twiddles and twist factors are
// read from one workgroup-shared LDS copy.  Accumulator and FFT exchanges live
// in wave-private LDS and need no barrier.
// ---------------------------------------------------------------------------
constexpr int BR_WAVES = 4;
constexpr int BR_LDS_BK = 2 * 2048 * 16;              // two row-pair slots, double2
constexpr int BR_LDS_TW = 512 * 16;                   // stage twiddles (511 used)
constexpr int BR_LDS_TWIST = 512 * 16;                // twist factors
constexpr int BR_LDS_ACC = 2048 * 4;                  // per wave
constexpr int BR_LDS_X = 512 * 16;                    // per wave, one exchange buffer for both FFTs
constexpr int BR_LDS_AT = 1024 * 2;                   // per wave
constexpr int BR_LDS_SYNC = 64;                       // slot counters pub[2], done[2]
constexpr int BR_LDS_TOTAL =
    BR_LDS_BK + BR_LDS_TW + BR_LDS_TWIST + BR_WAVES * (BR_LDS_ACC + BR_LDS_X + BR_LDS_AT) + BR_LDS_SYNC;
constexpr int BR_LDS_ACC_AT = BR_LDS_BK + BR_LDS_TW + BR_LDS_TWIST;  // accumulator copies: 4 KB-aligned (gather_rot)
static_assert(BR_LDS_ACC_AT % 4096 == 0 && BR_LDS_ACC % 4096 == 0, "gather_rot needs 4 KB-aligned copies");

// The kernel's one __shared__ array is the whole static LDS allocation and sits
// at LDS address 0, so the offsets above are absolute; hipcc folds this check
// (a constant address) away, and a layout that broke it fails loudly.
DEV bool lds_layout_bad(const void *smem) { return ((uint32_t)(size_t)(const lds_void_t *)smem & 4095u) != 0; }

// Slot protocol (round 2): monotonic LDS counters per BK slot instead of a
// workgroup barrier per row pair.  A loader wave adds 1 to pub[s] once its
// pieces of a pair landed in slot s; a gate wave reads the pair once pub[s]
// reached 4 x (its use of the slot + 1), and adds 1 to done[s] after its MAC; a
// loader refills slot s once done[s] shows every gate wave through the
// previous use.  Gate waves then wait only for data, not for each other.  Every
// wait is bounded (KParams::spin_cap polls, BR_SPIN_CAP_DEFAULT = 2^22): a
// broken protocol never hangs the GPU.  A wait that gives up sets the wave's
// `fail` flag (an SGPR, inside the asm); the wave ORs it into the context's
// device error word once, at its end (report_wait_failure), and the host fails
// the call (TFHE_ERR_DEVICE) instead of returning the launch's words.
// The loader waves poll `done` at s_sleep LOADER_SLEEP and issue priority 0:
// their polls (an LDS read and a v_readfirstlane each) take issue and LDS slots
// from the gate wave on the same SIMD.  A refill is due two MACs (~9 k cycles)
// before its use, so the coarse poll never makes it late.  Measured settings:
// sleep 12 at priority 0 against sleep 1 at priority 3, 7.39 -> 6.98 ms per
// 1,024 gates (profiles/r02_ab_loader_poll.txt); sleep 96 against 12 under the
// max-memory-clause scheduler, 6.21-6.35 vs 6.39-6.53 ms (48: 6.27-6.32, 64:
// 6.53-6.58, 127: 6.31-6.33; profiles/r03r_ab_loader_sleep.txt), re-checked in
// round 4 (profiles/r04_ab_loader_sleep.txt, r04_ab_loader_prio.txt).
constexpr int LOADER_SLEEP = 96;
constexpr int LOADER_PRIO = 0;
// `cap` >= 1 polls; on a timeout the loop falls through to `s_mov fail, 1`.
template <int SLEEP = 1>
DEV void spin_until_ge(const uint32_t *p, uint32_t target, uint32_t cap, uint32_t &fail) {
    // the poll loop in asm: every lane reads the same word, the loop stays
    // scalar, and hipcc sees one instruction (a compiler-visible loop here made
    // it hoist address arithmetic out of the step loop and spill)
    const uint32_t addr = (uint32_t)(size_t)(const lds_void_t *)p;
    uint32_t v, sv, cnt;
    asm volatile(
        "s_mov_b32 %[cnt], %[cap]\n"
        "1:\n\t"
        "ds_read_b32 %[v], %[addr]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_readfirstlane_b32 %[sv], %[v]\n\t"
        "s_cmp_ge_u32 %[sv], %[tgt]\n\t"
        "s_cbranch_scc1 2f\n\t"
        "s_sleep %[sl]\n\t"
        "s_sub_u32 %[cnt], %[cnt], 1\n\t"
        "s_cmp_eq_u32 %[cnt], 0\n\t"
        "s_cbranch_scc0 1b\n\t"
        "s_mov_b32 %[fail], 1\n"
        "2:"
        : [v] "=&v"(v), [sv] "=&s"(sv), [cnt] "=&s"(cnt), [fail] "+s"(fail)
        : [addr] "v"(addr), [tgt] "s"(target), [cap] "s"(cap), [sl] "i"(SLEEP)
        : "memory", "scc");
}
// One lane of a wave whose wait gave up ORs `bit` into the device error word
// (a vector global atomic).  Called once per wave, after its loop.
DEV void report_wait_failure(const KParams &P, uint32_t fail, uint32_t bit) {
    if (fail && P.err && (threadIdx.x & 63) == 0) __hip_atomic_fetch_or(P.err, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// One add per wave (lane 0's), without a branch: a divergent `if (lane == 0)`
// around an atomic split the live ranges of the MAC and spilled 396 B per lane.
// The LDS unit executes a wave's LDS instructions in order, so the add lands
// after every LDS read the wave issued before it; a loader's DMA is waited for
// (vmcnt) before its add.
DEV void counter_add(uint32_t *p) {
    const uint32_t addr = (uint32_t)(size_t)(lds_void_t *)p;
    uint64_t save;
    asm volatile(
        "s_mov_b64 %[save], exec\n\t"
        "s_mov_b64 exec, 1\n\t"
        "ds_add_u32 %[addr], %[one]\n\t"
        "s_mov_b64 exec, %[save]"
        : [save] "=&s"(save)
        : [addr] "v"(addr), [one] "v"(1u)
        : "memory");
}

// Digits of rows (row, row+1) read back from the wave's LDS copy of the
// flipped tmp words (polynomial a at [0, 1024), b at [1024, 2048)), one read
// of the 8 twist factors for both (L < 3; digit_f64_flipped).
template <bool FU = false>
DEV void load_digits_pair_lds(C2 (*d)[8], const uint32_t *s_tmp, int row, int L, int bgbit, const C2 *twist_t,
                              int t) {
    const uint32_t *src[2];
    int level[2];
#pragma unroll
    for (int f = 0; f < 2; f++) {
        const bool from_a = row + f < L;
        src[f] = s_tmp + (from_a ? 0 : 1024) + t;
        level[f] = from_a ? row + f : row + f - L;
    }
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const int m = br3(q);
        const C2 w = twist_t[64 * m];
#pragma unroll
        for (int f = 0; f < 2; f++)
            d[f][q] = twist_in<FU>(digit_f64_flipped(src[f][64 * m], level[f], bgbit),
                                   digit_f64_flipped(src[f][64 * (m + 8)], level[f], bgbit), w);
    }
}

// Digits of rows (0, 1) from the tmp words still in registers after the
// rotation gather (lane word m = coefficient t + 64m), the same values
// load_digits_pair_lds reads back from LDS: the first pair's transforms then
// do not wait for an LDS round trip at the top of the step (128-bit: 6.64 ->
// 6.60 ms per 1,024 gates; UINT4, where tB must stay live too: 1.4 % slower,
// not used there; profiles/r02_ab_pair0_regs.txt).
// tw0[q] = twist factor of coefficient t + 64 br3(q), read with the gather.
template <bool FU = false>
DEV void load_digits_pair0_regs(C2 (*d)[8], const uint32_t *tA, const uint32_t *tB, int L, int bgbit,
                                const C2 *tw0) {
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const int m = br3(q);
        const C2 w = tw0[q];
#pragma unroll
        for (int f = 0; f < 2; f++) {
            const bool from_a = f < L;
            const uint32_t *src = from_a ? tA : tB;
            const int level = from_a ? f : f - L;
            d[f][q] = twist_in<FU>(digit_f64_flipped(src[m], level, bgbit), digit_f64_flipped(src[m + 8], level, bgbit), w);
        }
    }
}

// Digits of rows (2rp, 2rp+1), rp = 1, 2 at L = 3, from packed tmp words kept in
// registers (round 4): tbx[m] = tmp_b's word m with tmp_a's level-2 field moved
// into its unused low bits (tmp_b's fields sit at bits >= 32 - 3 bgbit > bgbit).
// Row 2 (a, level 2) reads bits [0, bgbit), rows 3-5 (b, levels 0-2) their own
// fields: one v_bfe_i32 per digit as before, and no tmp round trip through LDS
// (32 ds_write_b32 + 48 ds_read_b32 per step fewer; 6.25-6.32 -> 6.12-6.18 ms,
// profiles/r04_ab_tmp_regs.txt).
template <bool FU>
DEV void load_digits_pair_tbx(C2 (*d)[8], const uint32_t *tbx, int rp, int bgbit, const C2 *twist_t) {
    const int off0 = rp == 1 ? 0 : 32 - 2 * bgbit, off1 = rp == 1 ? 32 - bgbit : 32 - 3 * bgbit;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const int m = br3(q);
        const C2 w = twist_t[64 * m];
        d[0][q] = twist_in<FU>((double)(int32_t)__builtin_amdgcn_sbfe(tbx[m], off0, bgbit),
                               (double)(int32_t)__builtin_amdgcn_sbfe(tbx[m + 8], off0, bgbit), w);
        d[1][q] = twist_in<FU>((double)(int32_t)__builtin_amdgcn_sbfe(tbx[m], off1, bgbit),
                               (double)(int32_t)__builtin_amdgcn_sbfe(tbx[m + 8], off1, bgbit), w);
    }
}

// LDS-DMA of one BK row pair (32 KB) into a slot by the 256 loader threads,
// 8 x 16 B per thread, in inline asm (cdna_hip_programming.md §5.7) so that
// hipcc does not guard the MAC's reads of the other slot with vmcnt(0);
// completion is waited for by hand (vmcnt) before the slot is published.
DEV void issue_bk_pair_async(const double2 *__restrict__ src, double2 *slot, int tid) {
    const uint32_t base = (uint32_t)(size_t)(lds_void_t *)slot + (uint32_t)(tid & ~63) * 16;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint32_t dst = __builtin_amdgcn_readfirstlane(base + 256 * 16 * k);
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(src + 256 * k + tid), "s"(dst)
            : "memory");
    }
}

// Wait until pair k is published in its slot, with the MAC's first frequency
// group of BK words read in the same LDS batch as the counter (round 4): a
// wave's LDS operations execute in order, so words read behind a counter value
// that says "published" are the published ones; rarely (0.19 per step,
// profiles/r04_spin_stats.txt) the pair is not in yet: sleep, read both again.
// One asm loop, so hipcc sees four plain 16-B results (6.08-6.09 -> 6.06-6.07 ms,
// profiles/r04_ab_pub_batch.txt).
DEV void wait_pair_first_group(const uint32_t *pub, const double2 *slot_t, uint32_t k, uint32_t spin_cap,
                               uint32_t &fail, double2 *kpre) {
    typedef __attribute__((ext_vector_type(4))) unsigned int u4;
    u4 q0, q1, q2, q3;
    uint32_t v, sv, cnt = fail ? 1u : spin_cap;
    const uint32_t caddr = (uint32_t)(size_t)(lds_void_t *)(pub + (k & 1));
    const uint32_t baddr = (uint32_t)(size_t)(lds_void_t *)slot_t;
    const uint32_t target = 4u * ((k >> 1) + 1u);
    asm volatile(
        "1:\n\t"
        "ds_read_b32 %[v], %[ca]\n\t"
        "ds_read_b128 %[q0], %[ba]\n\t"
        "ds_read_b128 %[q1], %[ba] offset:1024\n\t"
        "ds_read_b128 %[q2], %[ba] offset:16384\n\t"
        "ds_read_b128 %[q3], %[ba] offset:17408\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_readfirstlane_b32 %[sv], %[v]\n\t"
        "s_cmp_ge_u32 %[sv], %[tgt]\n\t"
        "s_cbranch_scc1 2f\n\t"
        "s_sleep 1\n\t"
        "s_sub_u32 %[cnt], %[cnt], 1\n\t"
        "s_cmp_eq_u32 %[cnt], 0\n\t"
        "s_cbranch_scc0 1b\n\t"
        "s_mov_b32 %[fail], 1\n"
        "2:"
        : [v] "=&v"(v), [q0] "=&v"(q0), [q1] "=&v"(q1), [q2] "=&v"(q2), [q3] "=&v"(q3), [sv] "=&s"(sv),
          [cnt] "+s"(cnt), [fail] "+s"(fail)
        : [ca] "v"(caddr), [ba] "v"(baddr), [tgt] "s"(target)
        : "memory", "scc");
    kpre[0] = __builtin_bit_cast(double2, q0);
    kpre[1] = __builtin_bit_cast(double2, q1);
    kpre[2] = __builtin_bit_cast(double2, q2);
    kpre[3] = __builtin_bit_cast(double2, q3);
}

// Row pairs of one CMUX step: digits and forward FFTs of rows (2rp, 2rp+1),
// wait for the pair's BK rows in LDS, MAC, release the slot.  Unrolled: every
// row's source polynomial and level are compile-time constants, so pairs (0,1)
// and (4,5) read their one polynomial's tmp once and the digit shifts are
// immediates (6.78 -> 6.67 ms per 1,024 gates; profiles/r02_ab_pair_unroll.txt).
// Pair k = k0 + rp is use (k >> 1) of slot k & 1.
template <int L, bool FU = false>
DEV void br_pairs(const uint32_t *s_tmp, int bgbit, const LdsTw &T, const C2 *twist_t, C2 *xb, int t, C2 *fa,
                  C2 *fb, double2 *s_bk, PhaseProf &pp, uint32_t &fail, uint32_t spin_cap, uint32_t *sync,
                  uint32_t k0, const uint32_t *tA, const uint32_t *tB, const C2 *tw0, const uint32_t *tbx) {
#pragma unroll
    for (int q = 0; q < 8; q++) {  // fmaInFd1024 accumulates from 0.0 (0.0 + x == x)
        fa[q] = c2(0.0, 0.0);
        fb[q] = c2(0.0, 0.0);
    }
#pragma unroll
    for (int rp = 0; rp < L; rp++) {
        C2 d[2][8];
        double2 kpre[4];
        pp.mark(1);
        if (L > 1 && rp == 0)  // UINT4 (L = 1): 1.4 % slower, LDS kept
            load_digits_pair0_regs<FU>(d, tA, tB, L, bgbit, tw0);
        else if (L == 3)
            load_digits_pair_tbx<FU>(d, tbx, rp, bgbit, twist_t);
        else
            load_digits_pair_lds<FU>(d, s_tmp, 2 * rp, L, bgbit, twist_t, t);
        fft512_x2<false, true, FU>(d, xb, T, t);
        pp.mark(2);
        const uint32_t k = k0 + (uint32_t)rp;
        wait_pair_first_group(sync, s_bk + (k & 1) * 2048 + t, k, spin_cap, fail, kpre);
        __builtin_amdgcn_sched_barrier(0);  // as a barrier would: nothing moves across the wait
        pp.mark(3);
        mac_pair_lds<FU>(fa, fb, d[0], d[1], s_bk + (k & 1) * 2048, t, kpre);
        __builtin_amdgcn_sched_barrier(0);
        counter_add(sync + 2 + (k & 1));  // done with this use of the slot
        pp.mark(4);
    }
}

template <int L, bool SMALL, bool FU>
__global__ __launch_bounds__(512, 1) void k_blind_rotate(
    KParams P, DevTables TT, const uint8_t *__restrict__ ops, const uint32_t *__restrict__ in_a,
    const uint32_t *__restrict__ in_b, const uint32_t *__restrict__ idx, const uint32_t *__restrict__ testvec,
    const double2 *__restrict__ bkd, uint32_t *__restrict__ out, int out_mode, size_t B) {
    // one __shared__ array (a second one can make hipcc drain LDS-DMA early)
    __shared__ __attribute__((aligned(16))) unsigned char smem[BR_LDS_TOTAL];
    const int tid = threadIdx.x;
    const int t = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    double2 *s_bk = reinterpret_cast<double2 *>(smem);
    // pub[2], done[2] (zeroed by the gate waves before the prologue barrier)
    uint32_t *s_sync = reinterpret_cast<uint32_t *>(smem + BR_LDS_TOTAL - BR_LDS_SYNC);
    if (lds_layout_bad(smem)) {
        if (tid == 0) __hip_atomic_fetch_or(P.err, (uint32_t)DEV_ERR_LDS_LAYOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if (!FU && P.fallback) {  // reference-tree recompute: only workgroups with a flagged item
        const size_t g0 = (size_t)blockIdx.x * BR_WAVES;
        uint32_t any = 0;
        for (int k = 0; k < BR_WAVES; k++)
            if (g0 + k < B) any |= P.tie_flags[g0 + k];
        if (!any) return;  // uniform over the workgroup: every wave reads the same flags
    }
    if (w >= BR_WAVES) {  // loader wave (slot protocol above)
        const int ltid = tid - 64 * BR_WAVES;
        __builtin_amdgcn_s_setprio(LOADER_PRIO);
        const size_t stride = (size_t)L * 2048;
        const uint32_t pairs = (uint32_t)P.n * L;
        const uint32_t spin = P.spin_cap ? P.spin_cap : BR_SPIN_CAP_DEFAULT;
        const uint32_t loader_cap = spin / LOADER_SLEEP > 0 ? spin / LOADER_SLEEP : 1u;
        uint32_t fail = 0;
        issue_bk_pair_async(bkd, s_bk, ltid);  // pair 0 into slot 0
        __syncthreads();                       // the gate waves' prologue barrier (counters zeroed)
        PhaseProf lp;  // loader phases (TFHE_PHASE_PROF): 0 DMA landing, 1 waiting for the gates, 2 issue
        lp.start();
        for (uint32_t k = 0; k < pairs; k++) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of pair k landed
            lp.mark(1);
            counter_add(s_sync + (k & 1));
            if (k + 1 < pairs) {
                const uint32_t k1 = k + 1;
                // every gate done with pair k1 - 2
                spin_until_ge<LOADER_SLEEP>(s_sync + 2 + (k1 & 1), 4u * (k1 >> 1), loader_cap, fail);
                lp.mark(2);
                issue_bk_pair_async(bkd + (size_t)(k1 / L) * stride + (size_t)(k1 % L) * 2048, s_bk + (k1 & 1) * 2048,
                                    ltid);
                lp.mark(0);
            }
        }
        lp.mark(3);
        report_wait_failure(P, fail, DEV_ERR_LOADER_WAIT);
#ifdef TFHE_PHASE_PROF
        if (ltid % 64 == 0)
            lp.flush(g_phase_cycles + 8, 4);
#endif
        return;
    }
    C2 *s_tw = reinterpret_cast<C2 *>(smem + BR_LDS_BK);
    C2 *s_twist = reinterpret_cast<C2 *>(smem + BR_LDS_BK + BR_LDS_TW);
    unsigned char *wbase = smem + BR_LDS_BK + BR_LDS_TW + BR_LDS_TWIST;
    uint32_t *s_acc = reinterpret_cast<uint32_t *>(wbase + w * BR_LDS_ACC);
    C2 *s_x = reinterpret_cast<C2 *>(wbase + BR_WAVES * BR_LDS_ACC + w * BR_LDS_X);
    uint16_t *s_at = reinterpret_cast<uint16_t *>(wbase + BR_WAVES * (BR_LDS_ACC + BR_LDS_X) + w * BR_LDS_AT);

    const int n = P.n;
    const size_t g_raw = (size_t)blockIdx.x * BR_WAVES + w;
    const bool valid = g_raw < B;
    const size_t g = valid ? g_raw : B - 1;  // ragged tail: compute a copy, store nothing
    // idx (optional): item g reads ciphertexts idx[2g] of in_a and idx[2g+1] of in_b
    const size_t ia = idx ? idx[2 * g] : g, ib = idx ? idx[2 * g + 1] : g;
    const uint32_t *A = in_a + ia * (size_t)(n + 1);
    const uint32_t *Bv = in_b ? in_b + ib * (size_t)(n + 1) : A;
    const int op = ops ? (int)ops[g] : 255;

    if (tid < 4) s_sync[tid] = 0u;
    for (int x = tid; x < 511; x += 256) s_tw[x] = TT.tw[x];
    for (int x = tid; x < 512; x += 256) s_twist[x] = TT.twist[x];

    // a~_i = (a_i + 2^20) >> 21 and b~ = 2N - ((b + 2^20) >> 21), 64-bit adds
    // (trgsw.zig:297, :312).
    int bt = 0;
    for (int i = t; i <= n; i += 64) {
        uint32_t c = gate_combine(op, A[i], Bv[i], i == n);
        uint32_t tl = (uint32_t)(((uint64_t)c + (1ull << 20)) >> 21);
        if (i < n) s_at[i] = (uint16_t)tl;
        else bt = 2048 - (int)tl;
    }
    bt = __builtin_amdgcn_readlane(bt, n & 63);

    // acc = X^{b~} * testvec (trgsw.zig:300-306), lane owns k = t + 64m.
    uint32_t accA[16], accB[16];
#pragma unroll
    for (int m = 0; m < 16; m++) {
        accA[m] = rot_read(testvec, t + 64 * m, bt);
        accB[m] = rot_read(testvec + 1024, t + 64 * m, bt);
        s_acc[t + 64 * m] = accA[m];
        s_acc[1024 + t + 64 * m] = accB[m];
    }
    __syncthreads();  // tables visible to every wave
    LdsTw T;
    T.init(s_tw, TT);
    const C2 *twist_t = s_twist + t;  // twist of coefficient t + 64m at [64m]
    PhaseProf pp;
    pp.start();
    int at_next = s_at[0];  // a~ of the coming step, read one step ahead
    uint32_t near = NEAR_NONE;  // FU: margin guard (torus_from_f64_guarded)
    uint32_t fail = 0;  // a slot wait gave up (report_wait_failure)
    const uint32_t spin_cap = P.spin_cap ? P.spin_cap : BR_SPIN_CAP_DEFAULT;
    const uint32_t msbs = digit_msbs(L, P.bgbit);
    const uint32_t acc_base = (uint32_t)(size_t)(lds_void_t *)s_acc;  // 4 KB-aligned (BR_LDS_ACC_AT)
    // L = 3: the tmp words stay in registers for every row pair (load_digits_pair_tbx);
    // L < 3 stages them through the accumulator's LDS copy
    constexpr bool tmp_regs = L == 3;

    for (int i = 0; i < n; i++) {
        pp.mark(0);
        // a~ in {0, 2N} gives tmp = 0 and an exactly-zero external product;
        // it is computed anyway so the four waves keep one slot schedule.
        const int at = __builtin_amdgcn_readfirstlane(at_next);
        // tmp = X^{a~} acc - acc (+ decomposition offset); the old acc stays in
        // the accA/accB registers
        uint32_t tA[16], tB[16], tbx[16];
        C2 tw0[8];
        // all 32 gathers first (one wait), then the arithmetic: interleaved,
        // hipcc waits for every gather before issuing the next
        uint32_t xb[16];
        gather_rot(acc_base, t, at, xb, tA, tB);
        // pair 0's twist factors ride with the gather (one wait for both);
        // read after the tmp stores they queued behind them (6.64 -> 6.61 ms,
        // profiles/r02_ab_twist_preload.txt)
        if constexpr (L > 1) {
#pragma unroll
            for (int q = 0; q < 8; q++) tw0[q] = twist_t[64 * br3(q)];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 16; m++) {
            const uint32_t sg = gather_sign(xb[m]), off_s = P.offset - sg;  // X^a~ wraps past N: negacyclic sign
            tA[m] = tmp_word(tA[m], sg, off_s, accA[m], msbs);
            tB[m] = tmp_word(tB[m], sg, off_s, accB[m], msbs);
        }
        if constexpr (tmp_regs) {  // pairs 1, 2 read tbx (load_digits_pair_tbx), not LDS
#pragma unroll
            for (int m = 0; m < 16; m++)
                tbx[m] = __builtin_amdgcn_ubfe(tA[m], 32 - L * P.bgbit, P.bgbit) | (tB[m] & ~((1u << P.bgbit) - 1u));
        } else {  // tmp over the accumulator's LDS copy (its gather reads come first)
            wave_sync();
#pragma unroll
            for (int m = 0; m < 16; m++) {
                s_acc[t + 64 * m] = tA[m];
                s_acc[1024 + t + 64 * m] = tB[m];
            }
            wave_sync();
        }
        C2 fa[8], fb[8];
        at_next = s_at[i + 1 < n ? i + 1 : i];
        br_pairs<L, FU>(s_acc, P.bgbit, T, twist_t, s_x, t, fa, fb, s_bk, pp, fail, spin_cap, s_sync,
                        (uint32_t)(L * i), tA, tB, tw0, tbx);
        pp.mark(5);
        inverse_and_add<SMALL, 64, true, FU>(fa, fb, s_x, T, twist_t, t, accA, accB, near);
        wave_sync();
#pragma unroll
        for (int m = 0; m < 16; m++) {
            s_acc[t + 64 * m] = accA[m];
            s_acc[1024 + t + 64 * m] = accB[m];
        }
        wave_sync();
    }
    pp.mark(6);
#ifdef TFHE_PHASE_PROF
    if (t == 0)
        pp.flush(g_phase_cycles, 8);
#endif
    report_wait_failure(P, fail, DEV_ERR_GATE_WAIT);
    if (FU) near_tie_flag(P, near, g, valid);
    // recompute: every wave of the workgroup read the flags before the prologue
    // barrier, so this item's flag can be cleared now; err[1] counts the items
    // recomputed (tfhe_gpu_near_tie_items)
    if (!FU && P.fallback && valid && t == 0 && P.tie_flags[g]) {
        P.tie_flags[g] = 0;
        __hip_atomic_fetch_add(P.err + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    if (!valid) return;
    if (out_mode == BR_OUT_LV1) {
        // sampleExtractIndex(acc, 0): p[0] = a[0], p[j] = -a[N-j], p[N] = b[0]
        uint32_t *o = out + g * (size_t)1025;
        for (int j = t; j <= 1024; j += 64) {
            uint32_t v;
            if (j == 0) v = s_acc[0];
            else if (j < 1024) v = 0u - s_acc[1024 - j];
            else v = s_acc[1024];
            o[j] = v;
        }
    } else if (out_mode == BR_OUT_LV0_EXTRACT2) {
        // sampleExtractIndex2(acc, 0) over the lv0 length n (trlwe.zig:165-180)
        uint32_t *o = out + g * (size_t)(n + 1);
        for (int j = t; j <= n; j += 64) o[j] = j == 0 ? s_acc[0] : j < n ? 0u - s_acc[n - j] : s_acc[1024];
    } else {
        uint32_t *o = out + g * (size_t)2048;
        for (int j = t; j < 2048; j += 64) o[j] = s_acc[j];
    }
}


// ---- shared by the latency forms (tfhe_kernels.hip, tools/ab/) ------------
// term = D * BK row part (fmaInFd1024's (a_re*b_re - a_im*b_im, a_re*b_im + a_im*b_re));
// FU: one multiply and one fma per component
template <bool FU = false>
DEV C2 cmul_bk(C2 d, double2 k) {
    if (FU) return c2(fmad(d.x, k.x, -(d.y * k.y)), fmad(d.x, k.y, d.y * k.x));
    return c2(d.x * k.x - d.y * k.y, d.x * k.y + d.y * k.x);
}
constexpr int BW_WAVES = 8;  // latency forms: one item per 8-wave workgroup
// Row wave w's BK row of the coming step: parts a|b, every frequency t + 64q.
DEV void wide_prefetch(double2 (*kr)[2], const double2 *__restrict__ nb, int w, int t) {
#pragma unroll
    for (int q = 0; q < 8; q++)
#pragma unroll
        for (int h = 0; h < 2; h++) kr[q][h] = nb[((size_t)w * 8 + q) * 128 + h * 64 + t];
}

}  // namespace tfhe
