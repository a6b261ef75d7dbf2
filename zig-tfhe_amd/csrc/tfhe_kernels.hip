// tfhe_kernels.hip — CDNA4 (gfx950) kernels of the TFHE gate-bootstrap path.
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
#include <hip/hip_runtime.h>

#include <algorithm>

#include "tfhe_internal.hpp"

#pragma clang fp contract(off)

namespace tfhe {

#define DEV __device__ __forceinline__

// Development-only phase timing of the blind-rotation kernels (tools/phase_prof.hip
// defines TFHE_PHASE_PROF): s_memtime deltas per phase, summed per wave and
// added to g_phase_cycles at the end.  Compiles to nothing otherwise.
struct PhaseProf {
#ifdef TFHE_SPIN_STATS
    uint32_t spins = 0;
#endif
#ifdef TFHE_PHASE_PROF
    uint64_t last;
    int cur;
    uint64_t acc[16];
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

// Exchange 2 in registers, for the single-transform fft512 (latency, pair and
// split forms, stage kernels; -DTFHE_EX2_LDS restores the LDS exchange there):
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
#ifndef TFHE_EX2_LDS
    if (!LDS) {
#pragma unroll
        for (int f = 0; f < NF; f++) ex2_regs(d[f]);
        return;
    }
#endif
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
// TFHE_X2_WAITS (A/B): one explicit lgkmcnt wait per read group instead of
// hipcc's one per consumed read (a single wave issues every s_waitcnt too).
// lgkmcnt(n): the LDS unit completes a wave's operations in order, so waiting
// until n remain leaves exactly the n youngest (a group of writes) in flight.
#ifndef TFHE_X2_WAITS
#define TFHE_X2_WAITS 0
#endif
#define X2_LGKM(n_)                                                                 \
    do {                                                                            \
        if (TFHE_X2_WAITS) {                                                        \
            __builtin_amdgcn_sched_barrier(0);                                      \
            __builtin_amdgcn_s_waitcnt(0xC07F | ((n_) << 8));                        \
            __builtin_amdgcn_sched_barrier(0);                                      \
        }                                                                           \
    } while (0)
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
    X2_LGKM(0);
    passBC<INV, FU>(d[0], wb_);
    ex1_read(d[1], x1, t);
#ifdef TFHE_EX2_REGS_X2  // register exchange 2 here too: 7.75 vs 7.52 ms per 1,024 gates (not kept)
    ex2_regs(d[0]);
    wave_sync();  // d[1]'s exchange reads precede any later write into the buffer
    passBC<INV, FU>(d[1], wb_);
    T.pass_c(wc_, t);
    ex2_regs(d[1]);
    passBC<INV, FU>(d[0], wc_);
    passBC<INV, FU>(d[1], wc_);
#else
    ex2_write(d[0], x0, t);
    wave_sync();
    X2_LGKM(8);
    passBC<INV, FU>(d[1], wb_);
    T.pass_c(wc_, t);
    ex2_read(d[0], x0, t);
    ex2_write(d[1], x1, t);
    wave_sync();
    X2_LGKM(8);
    passBC<INV, FU>(d[0], wc_);
    ex2_read(d[1], x1, t);
    wave_sync();
    X2_LGKM(0);
    passBC<INV, FU>(d[1], wc_);
#endif
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
DEV uint32_t torus_from_f64_guarded(double v, uint32_t &near) {
    const uint64_t b = (uint64_t)__double_as_longlong(v + 3377699720527872.5);
    const uint32_t lo = (uint32_t)b, hi = (uint32_t)(b >> 32);
#ifndef TFHE_GUARD_NOFLAG  // A/B timing builds only: the conversion without the flag
    near &= lo;
#endif
    return __builtin_amdgcn_alignbit(hi, lo, 1);
}

// Unguarded fused conversion (TFHE_FU_UNGUARDED A/B builds only): v + 1.5*2^52
// rounds to nearest and leaves rint(v) mod 2^32 in the low mantissa word.
DEV uint32_t torus_from_f64_near_integer(double v) {
    return (uint32_t)__double_as_longlong(v + 6755399441055744.0);
}

template <bool SMALL, bool FU = false>
DEV uint32_t to_torus(double v, uint32_t &near) {
#ifdef TFHE_FU_UNGUARDED
    if (FU) return torus_from_f64_near_integer(v);
#else
    if (FU) return torus_from_f64_guarded(v, near);
#endif
    return SMALL ? torus_from_f64_small(v) : torus_from_f64(v);
}
// Initial value of a `near` accumulator: no value off its integer by 1/4 or more.
constexpr uint32_t NEAR_NONE = ~0u;
// End of a fused item: if any lane of this wave rounded near a tie, flag item g
// (one byte, a vector store; the flag is rare, the ballot is one SALU compare).
DEV void near_tie_flag(const KParams &P, uint32_t near, size_t g, bool valid) {
    if (__builtin_amdgcn_ballot_w64((near & 1u) == 0u) != 0 && valid && P.tie_flags && (threadIdx.x & 63) == 0)
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
#ifndef TFHE_MAC_NO_FENCE
        __builtin_amdgcn_sched_barrier(0);
#endif
    }
}

// Inverse transforms of the two accumulated spectra (fft1024 x2) and the
// CMUX add acc' = ExtProd + acc (trgsw.zig:277-281), lane-local.
#ifndef TFHE_UNTWIST_EARLY
#define TFHE_UNTWIST_EARLY 0
#endif
template <bool SMALL, int TS, bool ONEBUF = false, bool FU = false, class TW>
DEV void inverse_and_add(const C2 *fa, const C2 *fb, C2 *xb, const TW &T, const C2 *tws, int t,
                         uint32_t *accA, uint32_t *accB, uint32_t &near) {
    C2 e[2][8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
        e[0][q] = fa[br3(q)];
        e[1][q] = fb[br3(q)];
    }
#if TFHE_UNTWIST_EARLY  // A/B: the untwist factors read before the transforms (their latency hidden)
    C2 wq[8];
#pragma unroll
    for (int q = 0; q < 8; q++) wq[q] = tws[q * TS];
#endif
#ifndef TFHE_KO_INV
    fft512_x2<true, ONEBUF, FU>(e, xb, T, t);
#endif
    // four independent near-tie accumulators, joined at the end: one chain
    // would serialise its 32 updates per call (A/B with the round-3 min form,
    // profiles/r03e_guard_chains_lut_octo.txt: guard cost 0.8 % with four chains,
    // 2.2 % with one)
    uint32_t nq[4] = {NEAR_NONE, NEAR_NONE, NEAR_NONE, NEAR_NONE};
#pragma unroll
    for (int q = 0; q < 8; q++) {
        double ra, ia, rb, ib;
#if TFHE_UNTWIST_EARLY
        const C2 w = wq[q];
#else
        const C2 w = tws[q * TS];
#endif
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

// Async copy of one BK row pair (2 TRGSW rows = 32 KB, contiguous in the
// device layout) into LDS by the whole 256-thread block: 8 x
// global_load_lds_dwordx4 per thread, LDS destination linear.
DEV void issue_bk_pair(const double2 *__restrict__ src, double2 *lds, int tid) {
    const int wbase = tid & ~63;
#pragma unroll
    for (int k = 0; k < 8; k++)
        __builtin_amdgcn_global_load_lds((global_void_t *)(src + 256 * k + tid),
                                         (lds_void_t *)(lds + 256 * k + wbase), 16, 0, 0);
}

// ---------------------------------------------------------------------------
// Blind rotation, one wavefront per item, 4 items per 256-thread block, all
// n CMUX steps in one launch:
//   acc = X^{b~} * testvec;  for i < n: acc = CMUX(BK[i], acc, X^{a~_i} acc)
// then sampleExtractIndex(acc, 0) (TLWELv1) or the TRLWE itself.
// The four waves consume the same BK rows, so each row pair is brought into
// LDS once per block by LDS-DMA, issued right after the previous pair's MAC
// and landing under the next forward FFTs.  FFT twiddles and twist factors
// are read from one block-shared LDS copy.  Accumulator and FFT exchanges
// live in wave-private LDS and need no block barrier.
// ---------------------------------------------------------------------------
constexpr int BR_WAVES = 4;
constexpr int BR_LDS_BK = 2 * 2048 * 16;              // two row-pair slots, double2
constexpr int BR_LDS_TW = 512 * 16;                   // stage twiddles (511 used)
constexpr int BR_LDS_TWIST = 512 * 16;                // twist factors
constexpr int BR_LDS_ACC = 2048 * 4;                  // per wave
constexpr int BR_LDS_X = 512 * 16;                    // per wave, one exchange buffer for both FFTs
constexpr int BR_LDS_AT = 1024 * 2;                   // per wave
constexpr int BR_LDS_SYNC = 64;                      // slot counters of the flag-synchronised variant
constexpr int BR_LDS_TOTAL =
    BR_LDS_BK + BR_LDS_TW + BR_LDS_TWIST + BR_WAVES * (BR_LDS_ACC + BR_LDS_X + BR_LDS_AT) + BR_LDS_SYNC;
constexpr int BR_LDS_ACC_AT = BR_LDS_BK + BR_LDS_TW + BR_LDS_TWIST;  // accumulator copies: 4 KB-aligned (gather_rot)
static_assert(BR_LDS_ACC_AT % 4096 == 0 && BR_LDS_ACC % 4096 == 0, "gather_rot needs 4 KB-aligned copies");

// The kernel's one __shared__ array is the whole static LDS allocation and sits
// at LDS address 0, so the offsets above are absolute; hipcc folds this check
// (a constant address) away, and a layout that broke it fails loudly.
DEV bool lds_layout_bad(const void *smem) { return ((uint32_t)(size_t)(const lds_void_t *)smem & 4095u) != 0; }

// Flag-synchronised loader variant (FLAGS; TFHE_OPT_BR_SYNC = 1): instead of one
// workgroup barrier per row pair, monotonic LDS counters per BK slot.  A
// loader wave adds 1 to pub[s] once its pieces of a pair landed in slot s; a
// gate wave reads the pair once pub[s] reached 4 x (its use of the slot + 1),
// and adds 1 to done[s] after its MAC; a loader refills slot s once done[s]
// shows every gate wave through the previous use.  Gate waves then wait only
// for data, not for each other.  Every wait is bounded (KParams::spin_cap
// polls, BR_SPIN_CAP_DEFAULT = 2^22): a broken protocol never hangs the GPU.
// A wait that gives up sets the wave's `fail` flag (an SGPR, inside the asm);
// the wave ORs it into the context's device error word once, at its end
// (report_wait_failure), and the host fails the call (TFHE_ERR_DEVICE)
// instead of returning the launch's words.
// The loader waves poll `done` at s_sleep 12 (~770 cycles) and normal issue
// priority: their polls (an LDS read and a v_readfirstlane each) had taken
// issue and LDS slots from the gate wave on the same SIMD.  A refill is due two
// MACs (~9 k cycles) before its use, so the coarse poll never makes it late:
// 7.39 -> 6.98 ms per 1,024 gates (sleep 1 at priority 3 before;
// profiles/r02_ab_loader_poll.txt).
// Round 3, under the max-memory-clause scheduler: s_sleep 96 (~6 k cycles)
// instead of 12, alternating on 6 boxes: 6.21-6.35 vs 6.39-6.53 ms per 1,024
// gates, 80-bit +2.6 %, 4,096 gates 27.3-27.9 vs 28.2-29.4 ms, the 65,536-gate
// circuit 635-639 vs 655-669 ms.  Not monotonic in the sleep (48: 6.27-6.32,
// 64: 6.53-6.58, 127: 6.31-6.33 ms): the poll period interacts with the pair
// period, so this is a measured setting.  s_wakeup from the gate waves and a
// fixed delay after the condition were slower (profiles/r03r_ab_loader_sleep.txt).
#ifndef TFHE_LOADER_SLEEP
#define TFHE_LOADER_SLEEP 96
#endif
#ifndef TFHE_LOADER_PRIO
#define TFHE_LOADER_PRIO 0
#endif
// `cap` >= 1 polls; on a timeout the loop falls through to `s_mov fail, 1`.
#ifdef TFHE_SPIN_STATS  // development: polls that found the counter short, per wave (tools/phase_prof.hip)
__device__ unsigned long long g_spin_stats[4];
#endif
template <int SLEEP = 1>
DEV void spin_until_ge(const uint32_t *p, uint32_t target, uint32_t cap, uint32_t &fail, uint32_t *extra = nullptr) {
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
    if (extra) *extra += cap - cnt;  // spins that slept (cnt counts down per failed poll)
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

// Digits of decomposition row `row` read from the wave's LDS copy of
// (rot - acc + offset): polynomial a at [0, 1024), b at [1024, 2048).  `row`
// is a runtime value (rolled pair loop); only pointer and shift depend on it.
DEV void load_digits_lds(C2 *d, const uint32_t *s_tmp, int row, int L, int bgbit, const C2 *twist_t, int t) {
    const bool from_a = row < L;
    const uint32_t *src = s_tmp + (from_a ? 0 : 1024) + t;
    const int level = from_a ? row : row - L;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const int m = br3(q);
#ifndef TFHE_KO_DIG
        d[q] = twist_in(digit_f64(src[64 * m], level, bgbit), digit_f64(src[64 * (m + 8)], level, bgbit),
                        twist_t[64 * m]);
#else
        d[q] = twist_in(digit_f64((uint32_t)(t * 77 + q), level, bgbit), digit_f64((uint32_t)(t * 5 + m), level, bgbit),
                        twist_t[64 * m]);
#endif
    }
}

// Digits of rows (row, row+1) with one read of the 8 twist factors for both
// (flipped tmp words, digit_f64_flipped).
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
// (32 ds_write_b32 + 48 ds_read_b32 per step fewer).
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
#ifndef TFHE_TMP_LDS  // A/B: 1 = the round-3 tmp words staged through LDS for row pairs 1 and 2
#define TFHE_TMP_LDS 0
#endif

// Row pairs of one CMUX step: forward FFTs of rows (2rp, 2rp+1), wait for the
// pair's BK rows in LDS, MAC, release the buffer and prefetch the next pair.
// LDS-DMA of one BK row pair (32 KB) into a slot, 8 x 16 B per thread, in
// inline asm (cdna_hip_programming.md §5.7) so that hipcc does not guard the
// MAC's reads of the other slot with vmcnt(0); completion is waited for by
// hand before the block barrier that publishes the slot.
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

#ifndef TFHE_OPT_PUB  // A/B: 1 = the slot counter read in one LDS batch with the MAC's first BK words
#define TFHE_OPT_PUB 1
#endif
template <int L, bool LOADER, bool FU = false, bool FLAGS = false>
DEV void br_pairs(const uint32_t *s_tmp, int bgbit, const LdsTw &T, const C2 *twist_t, C2 *xb, int t, int tid,
                  C2 *fa, C2 *fb, double2 *s_bk, int slot0, const double2 *__restrict__ next_pair, bool has_next,
                  PhaseProf &pp, uint32_t &fail, uint32_t spin_cap, uint32_t *sync = nullptr, uint32_t k0 = 0,
                  const uint32_t *tA = nullptr, const uint32_t *tB = nullptr, const C2 *tw0 = nullptr,
                  const uint32_t *tbx = nullptr) {
#pragma unroll
    for (int q = 0; q < 8; q++) {  // fmaInFd1024 accumulates from 0.0 (0.0 + x == x)
        fa[q] = c2(0.0, 0.0);
        fb[q] = c2(0.0, 0.0);
    }
    // unrolled with loader waves: every row's source polynomial and level are
    // compile-time constants, so pairs (0,1) and (4,5) read their one
    // polynomial's tmp once and the digit shifts are immediates (6.78 -> 6.67 ms
    // per 1,024 gates, 228 VGPRs, no spills; profiles/r02_ab_pair_unroll.txt).
    // Without loader waves the gate waves also issue the DMAs and the unrolled
    // loop spills (143-160 VGPRs at L = 3), so that form stays rolled, as does
    // every form under TFHE_PAIR_ROLLED (A/B builds).
#ifdef TFHE_PAIR_ROLLED
    constexpr int PAIR_UNROLL = 1;
#else
    constexpr int PAIR_UNROLL = LOADER ? L : 1;
#endif
#pragma unroll PAIR_UNROLL
    for (int rp = 0; rp < L; rp++) {
        C2 d[2][8];
        double2 kpre[4];
        bool pre = false;
        pp.mark(1);
#ifndef TFHE_PAIR0_LDS
        if (PAIR_UNROLL == L && LOADER && L > 1 && rp == 0)  // UINT4 (L = 1): 1.4 % slower, LDS kept
            load_digits_pair0_regs<FU>(d, tA, tB, L, bgbit, tw0);
        else
#endif
        if (!TFHE_TMP_LDS && PAIR_UNROLL == L && LOADER && L == 3)
            load_digits_pair_tbx<FU>(d, tbx, rp, bgbit, twist_t);
        else
            load_digits_pair_lds<FU>(d, s_tmp, 2 * rp, L, bgbit, twist_t, t);
#ifndef TFHE_KO_FFT  // TFHE_KO_*: development knock-out builds (timing only)
        fft512_x2<false, true, FU>(d, xb, T, t);
#endif
        pp.mark(2);
        const int slot = (slot0 + rp) & 1;
        if (FLAGS) {  // pair k = k0 + rp is use (k >> 1) of slot k & 1: wait until all 4 loaders published it
            const uint32_t k = k0 + (uint32_t)rp;
#if TFHE_OPT_PUB
            // optimistic: the slot counter and the MAC's first BK words in one LDS batch.
            // A wave's LDS operations execute in order, so words read after a counter
            // value that says "published" are the published ones; rarely (0.19 per
            // step, profiles/r04_spin_stats.txt) the pair is not in yet: sleep, read
            // both again.  One asm loop, so hipcc sees four plain 16-B results.
            {
                typedef __attribute__((ext_vector_type(4))) unsigned int u4;
                u4 q0, q1, q2, q3;
                uint32_t v, sv, cnt = fail ? 1u : spin_cap;
                const uint32_t caddr = (uint32_t)(size_t)(lds_void_t *)(sync + (k & 1));
                const uint32_t baddr = (uint32_t)(size_t)(lds_void_t *)(s_bk + slot * 2048 + t);
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
                pre = true;
            }
#elif !defined(TFHE_KO_WAIT)  // knock-out timing build: no wait for the pair's publication (wrong words possible)
#ifdef TFHE_SPIN_STATS
            spin_until_ge(sync + (k & 1), 4u * ((k >> 1) + 1u), spin_cap, fail, &pp.spins);
#else
            spin_until_ge(sync + (k & 1), 4u * ((k >> 1) + 1u), spin_cap, fail);
#endif
#endif
            __builtin_amdgcn_sched_barrier(0);  // as the barrier did: nothing moves across the wait
        } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's part of the pair's DMA landed
#ifndef TFHE_KO_BAR
        // the pair is in slot `slot` for every wave, and every wave is done
        // with the previous pair (the other slot), which the next DMA refills
        __syncthreads();
#endif
        }
        pp.mark(7);
#ifndef TFHE_KO_DMA
        if (!LOADER && (rp + 1 < L || has_next))
            issue_bk_pair_async(next_pair + (size_t)rp * 2048, s_bk + (slot ^ 1) * 2048, tid);
#endif
        pp.mark(3);
#ifndef TFHE_KO_MAC
        mac_pair_lds<FU>(fa, fb, d[0], d[1], s_bk + slot * 2048, t, pre ? kpre : nullptr);
#else
        for (int q = 0; q < 8; q++) fa[q] = c2(fa[q].x + d[0][q].x, fa[q].y + d[1][q].y);
#endif
        if (FLAGS) {  // done with this use of the slot
            __builtin_amdgcn_sched_barrier(0);
            counter_add(sync + 2 + ((k0 + (uint32_t)rp) & 1));
        }
        pp.mark(4);
    }
}

// LOADER: 4 more waves per workgroup, one beside each gate's wave on its SIMD,
// issue the BK row-pair DMAs (the same pieces, slots and barriers), so the
// gate waves only compute.
template <int L, bool SMALL, bool LOADER = false, bool FU = false, bool FLAGS = false>
__global__ __launch_bounds__(LOADER ? 512 : 256, 1) void k_blind_rotate(
    KParams P, DevTables TT, const uint8_t *__restrict__ ops, const uint32_t *__restrict__ in_a,
    const uint32_t *__restrict__ in_b, const uint32_t *__restrict__ idx, const uint32_t *__restrict__ testvec,
    const double2 *__restrict__ bkd, uint32_t *__restrict__ out, int out_mode, size_t B) {
    // one __shared__ array (a second one can make hipcc drain LDS-DMA early)
    __shared__ __attribute__((aligned(16))) unsigned char smem[BR_LDS_TOTAL];
    const int tid = threadIdx.x;
    const int t = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    double2 *s_bk = reinterpret_cast<double2 *>(smem);
    // FLAGS: pub[2], done[2] (zeroed by the gate waves before the prologue barrier)
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
    if constexpr (LOADER && FLAGS) {
        if (w >= BR_WAVES) {  // loader wave, counter protocol (see spin_until_ge)
            const int ltid = tid - 64 * BR_WAVES;
            __builtin_amdgcn_s_setprio(TFHE_LOADER_PRIO);
            const size_t stride = (size_t)L * 2048;
            const uint32_t pairs = (uint32_t)P.n * L;
            const uint32_t spin = P.spin_cap ? P.spin_cap : BR_SPIN_CAP_DEFAULT;
            const uint32_t loader_cap = spin / TFHE_LOADER_SLEEP > 0 ? spin / TFHE_LOADER_SLEEP : 1u;
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
                    spin_until_ge<TFHE_LOADER_SLEEP>(s_sync + 2 + (k1 & 1), 4u * (k1 >> 1), loader_cap, fail);
                    lp.mark(2);
                    issue_bk_pair_async(bkd + (size_t)(k1 / L) * stride + (size_t)(k1 % L) * 2048,
                                        s_bk + (k1 & 1) * 2048, ltid);
                    lp.mark(0);
                }
            }
            lp.mark(3);
            report_wait_failure(P, fail, DEV_ERR_LOADER_WAIT);
#ifdef TFHE_PHASE_PROF
            if (ltid % 64 == 0)
                for (int q = 0; q < 4; q++) atomicAdd(&g_phase_cycles[8 + q], (unsigned long long)lp.acc[q]);
#endif
            return;
        }
    }
    if constexpr (LOADER && !FLAGS) {
        if (w >= BR_WAVES) {  // loader wave: one barrier per row pair, like the gate waves
            const int ltid = tid - 64 * BR_WAVES;
            // top issue priority: a loader wave's DMA issue and barrier arrival
            // never wait behind its gate wave (9.14 vs 9.19 ms; raising the gate
            // waves instead cost 6 %, profiles/r01_ab_loader.txt)
            __builtin_amdgcn_s_setprio(3);
            const size_t stride = (size_t)L * 2048;
            issue_bk_pair_async(bkd, s_bk, ltid);  // pair (0, 0) into slot 0
            __syncthreads();                       // the gate waves' prologue barrier
            for (int i = 0; i < P.n; i++) {
#pragma unroll 1
                for (int rp = 0; rp < L; rp++) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces landed
                    __syncthreads();  // pair published; every gate wave is done with the other slot
                    const int slot = ((L * i) + rp) & 1;
                    if (rp + 1 < L || i + 1 < P.n)
                        issue_bk_pair_async(bkd + (size_t)i * stride + (size_t)(rp + 1) * 2048, s_bk + (slot ^ 1) * 2048,
                                            ltid);
                }
            }
            return;
        }
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
    const size_t step_stride = (size_t)L * 2048;  // double2 per TRGSW (BK[i])

    if (!LOADER) issue_bk_pair(bkd, s_bk, tid);  // pair (0, 0), lands under the prologue
    if (FLAGS && tid < 4) s_sync[tid] = 0u;
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
    uint32_t fail = 0;  // FLAGS: a slot wait gave up (report_wait_failure)
    const uint32_t spin_cap = P.spin_cap ? P.spin_cap : BR_SPIN_CAP_DEFAULT;
    const uint32_t msbs = digit_msbs(L, P.bgbit);
    const uint32_t acc_base = (uint32_t)(size_t)(lds_void_t *)s_acc;  // 4 KB-aligned (BR_LDS_ACC_AT)
    // tmp words stay in registers for every row pair (load_digits_pair_tbx): the loader
    // form at L = 3 (its unrolled pair loop), unless TFHE_TMP_LDS
    constexpr bool tmp_regs = !TFHE_TMP_LDS && LOADER && L == 3;

    for (int i = 0; i < n; i++) {
        pp.mark(0);
        // a~ in {0, 2N} gives tmp = 0 and an exactly-zero external product;
        // it is computed anyway so the four waves keep one barrier schedule.
        const int at = __builtin_amdgcn_readfirstlane(at_next);
        // tmp = X^{a~} acc - acc (+ decomposition offset), written over the
        // accumulator's LDS copy (the old acc stays in accA/accB registers)
        uint32_t tA[16], tB[16], tbx[16];
        C2 tw0[8];
#ifndef TFHE_KO_TMP
        // all 32 gathers first (one wait), then the arithmetic: interleaved,
        // hipcc waits for every gather before issuing the next
        uint32_t xb[16];
        gather_rot(acc_base, t, at, xb, tA, tB);
        // pair 0's twist factors ride with the gather (one wait for both);
        // read after the tmp stores they queued behind them (6.64 -> 6.61 ms,
        // profiles/r02_ab_twist_preload.txt)
        if constexpr (LOADER && L > 1) {
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
        }
#else
#pragma unroll
        for (int m = 0; m < 16; m++) {
            tA[m] = accA[m] * at + P.offset;
            tB[m] = accB[m] * at + P.offset;
        }
#endif
        if constexpr (!tmp_regs) {
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
        br_pairs<L, LOADER, FU, FLAGS>(s_acc, P.bgbit, T, twist_t, s_x, t, tid, fa, fb, s_bk, (L * i) & 1,
                                       bkd + (size_t)i * step_stride + 2048, i + 1 < n, pp, fail, spin_cap, s_sync,
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
        for (int k = 0; k < 8; k++) atomicAdd(&g_phase_cycles[k], (unsigned long long)pp.acc[k]);
#endif
    if (FLAGS) report_wait_failure(P, fail, DEV_ERR_GATE_WAIT);
#ifdef TFHE_SPIN_STATS
    if (t == 0) {
        atomicAdd(&g_spin_stats[0], (unsigned long long)pp.spins);
        atomicAdd(&g_spin_stats[1], 1ull);
    }
#endif
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

#ifdef TFHE_WHOLE_TU
// tfhe_kernels_whole.hip: this file compiled a second time for the default
// whole-form kernels only (loader waves, slot counters, fused arithmetic), with
// hipcc's max-memory-clause machine scheduler (Makefile).  That scheduler
// groups the kernel's LDS operations into clauses: 6.37-6.41 vs 6.48-6.55 ms per
// 1,024 gates, alternating on two boxes, the same words
// (profiles/r03r_ab_sched_strategy.txt).  Applied to the whole file it cost the
// latency form 2 % (16-bit adder 101.5 vs 99.7 ms), hence the separate unit.
hipError_t launch_whole_default(int L, dim3 grid, dim3 block, hipStream_t s, const KParams &P, const DevTables &T,
                                const uint8_t *ops, const uint32_t *in_a, const uint32_t *in_b, const uint32_t *idx,
                                const uint32_t *testvec, const double2 *bk2, uint32_t *out, int out_mode, size_t B) {
    switch (L) {
    case 1: hipLaunchKernelGGL((k_blind_rotate<1, true, true, true, true>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec, bk2, out, out_mode, B); break;
    case 2: hipLaunchKernelGGL((k_blind_rotate<2, true, true, true, true>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec, bk2, out, out_mode, B); break;
    case 3: hipLaunchKernelGGL((k_blind_rotate<3, true, true, true, true>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec, bk2, out, out_mode, B); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
#else  // the rest of the library's kernels and launchers

// ---------------------------------------------------------------------------
// Blind rotation, "octo" form (large batches): EIGHT items per 512-thread
// workgroup, one wave each, so every SIMD runs two gate waves that both issue
// f64 work (the whole form: one gate wave + one loader wave per SIMD).  The 8
// gates share each BK row pair brought into LDS by one DMA (twice the reuse of
// the whole form).  LDS per gate is ONE 8 KB buffer: it holds the accumulator
// between steps (the rotation gather reads it), and once the gather has
// produced tmp = X^a~ acc - acc + offset in registers (kept there for all 2L
// rows' digits) it is the gate's FFT exchange buffer until the accumulator is
// written back.  BK 2 x 32 KB + tables 16 KB + 8 x 8 KB + a~ 8 x 2 KB = 160 KB.
// No loader waves (a third wave per SIMD does not fit the VGPR file): every
// thread issues 4 x 16 B of each pair's DMA, and one workgroup barrier per row
// pair publishes the pair's slot and retires the other (as the whole form's
// non-loader variant).  Same arithmetic and row order as the whole form.
// ---------------------------------------------------------------------------
constexpr int BO_GATES = 8;
constexpr int BO_LDS_BUF = 2048 * 4;  // per gate: accumulator / exchange buffer
constexpr int BO_LDS_AT = 1024 * 2;   // per gate
constexpr int BO_LDS_TOTAL = BR_LDS_BK + BR_LDS_TW + BR_LDS_TWIST + BO_GATES * (BO_LDS_BUF + BO_LDS_AT);
static_assert(BO_LDS_TOTAL <= 160 * 1024, "octo form LDS");
constexpr int BO_LDS_BUF_AT = BR_LDS_BK + BR_LDS_TW + BR_LDS_TWIST;  // gate buffers: 4 KB-aligned (gather_rot)
static_assert(BO_LDS_BUF_AT % 4096 == 0 && BO_LDS_BUF % 4096 == 0, "gather_rot needs 4 KB-aligned buffers");

// LDS-DMA of one BK row pair (32 KB) into a slot by 512 threads: 4 x 16 B each,
// in the scalar-base form (SGPR pair address + the thread's 32-bit byte
// offset): no 64-bit per-lane addresses to keep live across the unrolled rows.
DEV void issue_bk_pair_async512(const double2 *__restrict__ src, double2 *slot, int tid) {
    const uint32_t base = (uint32_t)(size_t)(lds_void_t *)slot + (uint32_t)(tid & ~63) * 16;
    const uint32_t voff = (uint32_t)tid * 16;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t dst = __builtin_amdgcn_readfirstlane(base + 512 * 16 * k);
        const double2 *piece = src + 512 * k;
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(voff), "s"(dst), "s"(piece)
            : "memory");
    }
}

// Digits of row `row` (runtime) from the tmp words in registers (lane word m =
// coefficient t + 64m), twist factors from the LDS table.
template <bool FU>
DEV void load_digits_row_regs(C2 *d, const uint32_t *tA, const uint32_t *tB, int row, int L, int bgbit,
                              const C2 *twist_t) {
    const bool from_a = row < L;
    const int level = from_a ? row : row - L;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const int m = br3(q);
        const uint32_t x0 = from_a ? tA[m] : tB[m], x1 = from_a ? tA[m + 8] : tB[m + 8];
        d[q] = twist_in<FU>(digit_f64_flipped(x0, level, bgbit), digit_f64_flipped(x1, level, bgbit), twist_t[64 * m]);
    }
}

// MAC of one row (fmaInFd1024's row term for both outputs) from LDS, the BK
// words of frequency group q+1 read while group q's flops issue.
template <bool FU>
DEV void mac_row_lds(C2 *fa, C2 *fb, const C2 *d, const double2 *bk, int t) {
    double2 k[2][2];
    k[0][0] = bk[t];
    k[0][1] = bk[64 + t];
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const int c = q & 1;
        if (q + 1 < 8) {
            k[c ^ 1][0] = bk[(2 * q + 2) * 64 + t];
            k[c ^ 1][1] = bk[(2 * q + 3) * 64 + t];
        }
        const C2 x = d[q];
        const double2 ka = k[c][0], kb = k[c][1];
        if (FU) {
            fa[q] = c2(fmad(x.x, ka.x, fmad(-x.y, ka.y, fa[q].x)), fmad(x.x, ka.y, fmad(x.y, ka.x, fa[q].y)));
            fb[q] = c2(fmad(x.x, kb.x, fmad(-x.y, kb.y, fb[q].x)), fmad(x.x, kb.y, fmad(x.y, kb.x, fb[q].y)));
        } else {
            const C2 ta = c2(x.x * ka.x - x.y * ka.y, x.x * ka.y + x.y * ka.x);
            const C2 tb = c2(x.x * kb.x - x.y * kb.y, x.x * kb.y + x.y * kb.x);
            fa[q] = c2(fa[q].x + ta.x, fa[q].y + ta.y);
            fb[q] = c2(fb[q].x + tb.x, fb[q].y + tb.y);
        }
    }
}

// The 2L rows of one CMUX step in the octo form, in the reference's row order
// (rolled: unrolled, hipcc keeps every row's LDS addresses and spills): per row
// the digits, one forward transform (both exchanges through the gate's buffer:
// the partner wave on the SIMD covers their latency), at the first row of a
// pair the pair's barrier (its slot published, the other retired) and the next
// pair's DMA into the other slot, then the row's MAC.  Pair k0 + r/2.
template <int L, bool FU>
DEV void octo_rows(const uint32_t *tA, const uint32_t *tB, int bgbit, const LdsTwAtPass &T, const C2 *twist_t,
                   C2 *xb, int t, int tid, C2 *fa, C2 *fb, double2 *s_bk, uint32_t k0,
                   const double2 *__restrict__ bkd, uint32_t pairs) {
#pragma unroll 1
    for (int r = 0; r < 2 * L; r++) {
        const uint32_t k = k0 + (uint32_t)(r >> 1);
        C2 d[1][8];
        load_digits_row_regs<FU>(d[0], tA, tB, r, L, bgbit, twist_t);
#ifndef TFHE_KO_FFT
        fft512<1, false, FU, LdsTwAtPass, true>(d, xb, T, t);
#endif
        if ((r & 1) == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's pieces of pair k landed
            __syncthreads();  // pair k in slot k & 1 for every wave; every wave done with pair k - 1
            if (k + 1 < pairs)
                issue_bk_pair_async512(bkd + (size_t)((k + 1) / L) * L * 2048 + (size_t)((k + 1) % L) * 2048,
                                       s_bk + ((k + 1) & 1) * 2048, tid);
        }
        mac_row_lds<FU>(fa, fb, d[0], s_bk + (k & 1) * 2048 + (r & 1) * 1024, t);
    }
}

template <int L, bool SMALL, bool FU>
__global__ __launch_bounds__(512, 1) void k_blind_rotate_octo(
    KParams P, DevTables TT, const uint8_t *__restrict__ ops, const uint32_t *__restrict__ in_a,
    const uint32_t *__restrict__ in_b, const uint32_t *__restrict__ idx, const uint32_t *__restrict__ testvec,
    const double2 *__restrict__ bkd, uint32_t *__restrict__ out, int out_mode, size_t B) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[BO_LDS_TOTAL];
    const int tid = threadIdx.x;
    const int t = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    double2 *s_bk = reinterpret_cast<double2 *>(smem);
    C2 *s_tw = reinterpret_cast<C2 *>(smem + BR_LDS_BK);
    C2 *s_twist = reinterpret_cast<C2 *>(smem + BR_LDS_BK + BR_LDS_TW);
    unsigned char *gbase = smem + BR_LDS_BK + BR_LDS_TW + BR_LDS_TWIST;
    uint32_t *s_buf = reinterpret_cast<uint32_t *>(gbase + w * BO_LDS_BUF);
    C2 *s_x = reinterpret_cast<C2 *>(s_buf);
    uint16_t *s_at = reinterpret_cast<uint16_t *>(gbase + BO_GATES * BO_LDS_BUF + w * BO_LDS_AT);

    const int n = P.n;
    const size_t g_raw = (size_t)blockIdx.x * BO_GATES + w;
    const bool valid = g_raw < B;
    const size_t g = valid ? g_raw : B - 1;  // ragged tail: compute a copy, store nothing
    const size_t ia = idx ? idx[2 * g] : g, ib = idx ? idx[2 * g + 1] : g;
    const uint32_t *A = in_a + ia * (size_t)(n + 1);
    const uint32_t *Bv = in_b ? in_b + ib * (size_t)(n + 1) : A;
    const int op = ops ? (int)ops[g] : 255;
    const uint32_t pairs = (uint32_t)n * L;

    if (lds_layout_bad(smem)) {
        if (tid == 0) __hip_atomic_fetch_or(P.err, (uint32_t)DEV_ERR_LDS_LAYOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    issue_bk_pair_async512(bkd, s_bk, tid);  // pair 0 into slot 0, lands under the prologue
    for (int x = tid; x < 511; x += 512) s_tw[x] = TT.tw[x];
    for (int x = tid; x < 512; x += 512) s_twist[x] = TT.twist[x];
    int bt = 0;  // a~_i, b~ (trgsw.zig:297, :312), 64-bit adds
    for (int i = t; i <= n; i += 64) {
        const uint32_t c = gate_combine(op, A[i], Bv[i], i == n);
        const uint32_t tl = (uint32_t)(((uint64_t)c + (1ull << 20)) >> 21);
        if (i < n) s_at[i] = (uint16_t)tl;
        else bt = 2048 - (int)tl;
    }
    bt = __builtin_amdgcn_readlane(bt, n & 63);
    uint32_t accA[16], accB[16];  // acc = X^{b~} * testvec (trgsw.zig:300-306)
#pragma unroll
    for (int m = 0; m < 16; m++) {
        accA[m] = rot_read(testvec, t + 64 * m, bt);
        accB[m] = rot_read(testvec + 1024, t + 64 * m, bt);
        s_buf[t + 64 * m] = accA[m];
        s_buf[1024 + t + 64 * m] = accB[m];
    }
    __syncthreads();  // tables visible to every wave
    LdsTwAtPass T;
    T.init(s_tw, TT);
    const C2 *twist_t = s_twist + t;
    int at_next = s_at[0];
    uint32_t near = NEAR_NONE;
    const uint32_t msbs = digit_msbs(L, P.bgbit);
    const uint32_t buf_base = (uint32_t)(size_t)(lds_void_t *)s_buf;  // 4 KB-aligned (BO_LDS_BUF_AT)

    for (int i = 0; i < n; i++) {
        const int at = __builtin_amdgcn_readfirstlane(at_next);
        at_next = s_at[i + 1 < n ? i + 1 : i];
        // tmp = X^{a~} acc - acc + offset, kept in registers for every row's digits
        uint32_t tA[16], tB[16];
        uint32_t xb[16];
        gather_rot(buf_base, t, at, xb, tA, tB);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 16; m++) {
            const uint32_t sg = gather_sign(xb[m]), off_s = P.offset - sg;  // X^a~ wraps past N: negacyclic sign
            tA[m] = tmp_word(tA[m], sg, off_s, accA[m], msbs);
            tB[m] = tmp_word(tB[m], sg, off_s, accB[m], msbs);
        }
        wave_sync();  // the gather's reads precede the exchanges' writes into the buffer
        C2 fa[8], fb[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {  // fmaInFd1024 accumulates from 0.0
            fa[q] = c2(0.0, 0.0);
            fb[q] = c2(0.0, 0.0);
        }
        octo_rows<L, FU>(tA, tB, P.bgbit, T, twist_t, s_x, t, tid, fa, fb, s_bk, (uint32_t)(L * i), bkd, pairs);
        inverse_and_add<SMALL, 64, true, FU>(fa, fb, s_x, T, twist_t, t, accA, accB, near);
        wave_sync();
#pragma unroll
        for (int m = 0; m < 16; m++) {
            s_buf[t + 64 * m] = accA[m];
            s_buf[1024 + t + 64 * m] = accB[m];
        }
        wave_sync();
    }
    if (FU) near_tie_flag(P, near, g, valid);

    if (!valid) return;
    if (out_mode == BR_OUT_LV1) {  // sampleExtractIndex(acc, 0): p[0] = a[0], p[j] = -a[N-j], p[N] = b[0]
        uint32_t *o = out + g * (size_t)1025;
        for (int j = t; j <= 1024; j += 64) o[j] = j == 0 ? s_buf[0] : j < 1024 ? 0u - s_buf[1024 - j] : s_buf[1024];
    } else if (out_mode == BR_OUT_LV0_EXTRACT2) {  // sampleExtractIndex2 (trlwe.zig:165-180)
        uint32_t *o = out + g * (size_t)(n + 1);
        for (int j = t; j <= n; j += 64) o[j] = j == 0 ? s_buf[0] : j < n ? 0u - s_buf[n - j] : s_buf[1024];
    } else {
        uint32_t *o = out + g * (size_t)2048;
        for (int j = t; j < 2048; j += 64) o[j] = s_buf[j];
    }
}

// The split form (two waves per item, each transforming every other row) and
// the pair form (two waves per item, one per accumulator polynomial, with the
// regrouped row sums the duo form kept) were removed in round 4: measured
// slower than the whole form at every batch and parameter set since rounds 1
// and 2 (DESIGN.md §4.3, §4.3b record their measurements).

// term = D * BK row part (fmaInFd1024's (a_re*b_re - a_im*b_im, a_re*b_im + a_im*b_re));
// FU: one multiply and one fma per component
template <bool FU = false>
DEV C2 cmul_bk(C2 d, double2 k) {
    if (FU) return c2(fmad(d.x, k.x, -(d.y * k.y)), fmad(d.x, k.y, d.y * k.x));
    return c2(d.x * k.x - d.y * k.y, d.x * k.y + d.y * k.x);
}

// ---------------------------------------------------------------------------
// Blind rotation, "duo" form (round 4): TWO computing waves per item on ONE
// SIMD, 4 items per 512-thread workgroup, so a 1,024-item batch (one item per
// SIMD) runs two f64 instruction streams on every SIMD instead of one (the
// whole form's gate wave issues f64 at ~2.6 ns per instruction alone, ~2.1
// with a second computing wave beside it).  Wave (g, h) owns
// accumulator polynomial h (0: a, 1: b) and its L decomposition rows:
//   1. rotation gather of its own polynomial from its own LDS buffer (the
//      rotation never mixes the polynomials) -> tmp words in registers;
//   2. per level l: digits, one forward FFT, and the MAC of row hL + l against
//      both output parts into partial sums P_h,a / P_h,b (fused chains from
//      0.0, rows in the reference's order within each half);
//   3. hand-off: P_h,(1-h) goes into the partner's buffer once the partner's
//      forward FFTs are done (an LDS counter per wave), the partner's partial
//      comes back into its own buffer; output h = P_0,h + P_1,h (the pair
//      form's regrouped sum, exact-integer regime only: DESIGN.md §6.1);
//   4. inverse FFT of output h, untwist, guarded conversion, acc_h update.
// No workgroup barrier in the step loop.  BK level slots (rows l and L+l of
// one BK[i], 32 KB) double-buffered and shared by the 8 waves; every wave
// issues its 4 x 1 KB share of each level's LDS-DMA right after its forward
// FFT of the level before, publishes it (pub) once landed,
// and a refill waits until all 8 waves are done with the slot (done).  Every
// wait is a bounded poll (spin_until_ge).
// LDS: BK 2 x 32 KB + tables 16 KB + 8 wave buffers x 8 KB (accumulator copy /
// FFT exchange / hand-off) + 4 x 2 KB a~ + counters = 152 KB.
// ---------------------------------------------------------------------------
constexpr int BD_GATES = 4;
constexpr int BD_WAVES = 2 * BD_GATES;
constexpr int BD_LDS_BK = 2 * 2048 * 16;  // two level slots of rows (l, L+l), double2
constexpr int BD_LDS_BUF = 512 * 16;      // per wave
constexpr int BD_LDS_AT = 1024 * 2;       // per item
constexpr int BD_LDS_SYNC = 128;          // pub[2] done[2] fwd[8] hand[8] bt[4]
constexpr int BD_LDS_BUF_AT = BD_LDS_BK + BR_LDS_TW + BR_LDS_TWIST;
constexpr int BD_LDS_TOTAL = BD_LDS_BUF_AT + BD_WAVES * BD_LDS_BUF + BD_GATES * BD_LDS_AT + BD_LDS_SYNC;
static_assert(BD_LDS_TOTAL <= 160 * 1024, "duo form LDS");
static_assert(BD_LDS_BUF_AT % 4096 == 0 && BD_LDS_BUF % 4096 == 0, "gather_rot1 needs 4 KB-aligned buffers");

// Rotation gather of ONE polynomial (1,024 words at the 4 KB-aligned byte
// address `base`): lane word m = coefficient t + 64m of X^a~ * p, sign in bit
// 12 of xb[m] (gather_sign), as gather_rot.
DEV void gather_rot1(uint32_t base, int t, int at, uint32_t *xb, uint32_t *v) {
    const uint32_t rbb = (uint32_t)((t - at) & 2047) << 2;
    const uint32_t mask = __builtin_amdgcn_readfirstlane(0xFFCu);
    uint32_t vmask;
    asm volatile("v_mov_b32 %0, %1" : "=v"(vmask) : "s"(mask));
#pragma unroll
    for (int m = 0; m < 16; m++) {
        xb[m] = rbb + 256u * m;
        uint32_t a;
        asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(a) : "v"(xb[m]), "v"(vmask), "s"(base));
        v[m] = lds_read_u32(a);
    }
}

// This wave's share of one level's LDS-DMA: the level slot holds row lo (the
// a polynomial's row, 16 KB) then row hi (the b polynomial's), 32 pieces of
// 1 KB; wave w issues pieces w, w + 8 (row lo) and w + 16, w + 24 (row hi),
// SGPR base + 32-bit lane offset, hand-counted completion (vmcnt).
DEV void issue_level_share(const double2 *__restrict__ row_lo, const double2 *__restrict__ row_hi, double2 *slot,
                           int w, int t) {
    const uint32_t base = (uint32_t)(size_t)(lds_void_t *)slot;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const int j = w + 8 * c;
        const double2 *row = c < 2 ? row_lo : row_hi;
        const uint32_t voff = (uint32_t)((j & 15) * 1024 + t * 16);
        const uint32_t dst = __builtin_amdgcn_readfirstlane(base + 1024u * (uint32_t)j);
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(voff), "s"(dst), "s"(row)
            : "memory");
    }
}

// One level's whole LDS-DMA by ONE wave (duo form, claimed by the wave that
// found the slot free first): the level slot holds row lo (the a polynomial's
// row, 16 KB) then row hi (the b polynomial's), 32 pieces of 1 KB; SGPR base
// per piece + the lane's 16-B offset, hand-counted completion (vmcnt).
DEV void issue_level_full(const double2 *__restrict__ row_lo, const double2 *__restrict__ row_hi, double2 *slot,
                          int t) {
    const uint32_t base = (uint32_t)(size_t)(lds_void_t *)slot;
    const uint32_t voff = (uint32_t)t * 16u;
#pragma unroll
    for (int j = 0; j < 32; j++) {
        const double2 *piece = (j < 16 ? row_lo : row_hi) + (j & 15) * 64;
        const uint32_t dst = __builtin_amdgcn_readfirstlane(base + 1024u * (uint32_t)j);
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(voff), "s"(dst), "s"(piece)
            : "memory");
    }
}

// ds_cmpst_rtn_b32 by lane 0 (if *p == cmp: *p = val); the old value, uniform.
DEV uint32_t lds_cas_u32(uint32_t *p, uint32_t cmp, uint32_t val) {
    const uint32_t addr = (uint32_t)(size_t)(lds_void_t *)p;
    uint32_t old;
    uint64_t save;
    asm volatile(
        "s_mov_b64 %[save], exec\n\t"
        "s_mov_b64 exec, 1\n\t"
        "ds_cmpst_rtn_b32 %[old], %[addr], %[cmp], %[val]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_mov_b64 exec, %[save]"
        : [old] "=&v"(old), [save] "=&s"(save)
        : [addr] "v"(addr), [cmp] "v"(cmp), [val] "v"(val)
        : "memory");
    return __builtin_amdgcn_readfirstlane(old);
}
// A plain LDS word read, uniform (polled counters).
DEV uint32_t lds_peek_u32(const uint32_t *p) {
    const uint32_t addr = (uint32_t)(size_t)(const lds_void_t *)p;
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return __builtin_amdgcn_readfirstlane(v);
}

// MAC of one row for the duo form's two partial sums: `po` takes the part at
// bk_own, `px` the part at bk_oth ([q][a|b][lane] rows: the two parts of
// frequency group q at (2q)*64 and (2q+1)*64), BK words two groups ahead.
template <bool FU>
DEV void mac_row_roles(C2 *po, C2 *px, const C2 *d, const double2 *bk_own, const double2 *bk_oth, int t) {
    double2 k[3][2];
    k[0][0] = bk_own[t];
    k[0][1] = bk_oth[t];
    k[1][0] = bk_own[128 + t];
    k[1][1] = bk_oth[128 + t];
#pragma unroll
    for (int q = 0; q < 8; q++) {
        if (q + 2 < 8) {
            k[(q + 2) % 3][0] = bk_own[(q + 2) * 128 + t];
            k[(q + 2) % 3][1] = bk_oth[(q + 2) * 128 + t];
        }
        const C2 x = d[q];
        const double2 ko = k[q % 3][0], kx = k[q % 3][1];
        if (FU) {
            po[q] = c2(fmad(x.x, ko.x, fmad(-x.y, ko.y, po[q].x)), fmad(x.x, ko.y, fmad(x.y, ko.x, po[q].y)));
            px[q] = c2(fmad(x.x, kx.x, fmad(-x.y, kx.y, px[q].x)), fmad(x.x, kx.y, fmad(x.y, kx.x, px[q].y)));
        } else {
            const C2 to = c2(x.x * ko.x - x.y * ko.y, x.x * ko.y + x.y * ko.x);
            const C2 tx = c2(x.x * kx.x - x.y * kx.y, x.x * kx.y + x.y * kx.x);
            po[q] = c2(po[q].x + to.x, po[q].y + to.y);
            px[q] = c2(px[q].x + tx.x, px[q].y + tx.y);
        }
    }
}

#ifndef TFHE_KO_DUO_WAIT  // knock-out timing builds only: every duo-form wait removed (wrong words)
#define DUO_SPIN(...) spin_until_ge(__VA_ARGS__)
#else
#define DUO_SPIN(...) ((void)0)
#endif
#ifndef TFHE_DUO_PROTO  // BK protocol: 2 = LDS slots, every wave's share after a per-level wait (default),
#define TFHE_DUO_PROTO 2  // 1 = LDS slots by claims, 3 = no LDS slots: each wave loads its row from L2 into registers
#endif

// Duo protocol 3: wave h's BK row for level k (row hL + k % L of BK[k / L]),
// parts [q][a|b][lane]: kr[q][0] = frequency t + 64q of output part h (own),
// kr[q][1] of part 1 - h (the partner's); 16 x 16 B per lane, coalesced 1 KB
// per wave-instruction, landing under the next forward transform (the 4 items
// of a workgroup read the same row: L1/L2 hits)
// (wave-uniform piece bases in SGPRs, one shared 32-bit lane offset: hipcc
// otherwise hoists 16 64-bit per-lane addresses out of the step loop and spills)
DEV const double2 *sgpr_ptr(const double2 *p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return reinterpret_cast<const double2 *>(((uint64_t)hi << 32) | lo);
}
DEV void duo_row_load(double2 (*kr)[2], const double2 *__restrict__ row, int h, int t) {
#pragma unroll
    for (int q = 0; q < 8; q++) {
        kr[q][0] = sgpr_ptr(row + (2 * q + h) * 64)[t];
        kr[q][1] = sgpr_ptr(row + (2 * q + 1 - h) * 64)[t];
    }
}
template <bool FU>
DEV void mac_row_regs(C2 *po, C2 *px, const C2 *d, const double2 (*kr)[2]) {
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const C2 x = d[q];
        const double2 ko = kr[q][0], kx = kr[q][1];
        if (FU) {
            po[q] = c2(fmad(x.x, ko.x, fmad(-x.y, ko.y, po[q].x)), fmad(x.x, ko.y, fmad(x.y, ko.x, po[q].y)));
            px[q] = c2(fmad(x.x, kx.x, fmad(-x.y, kx.y, px[q].x)), fmad(x.x, kx.y, fmad(x.y, kx.x, px[q].y)));
        } else {
            const C2 to = c2(x.x * ko.x - x.y * ko.y, x.x * ko.y + x.y * ko.x);
            const C2 tx = c2(x.x * kx.x - x.y * kx.y, x.x * kx.y + x.y * kx.x);
            po[q] = c2(po[q].x + to.x, po[q].y + to.y);
            px[q] = c2(px[q].x + tx.x, px[q].y + tx.y);
        }
    }
}
#ifndef TFHE_DUO_EX2_REGS  // A/B: 1 = exchange 2 of every transform by permlane / DPP moves (ex2_regs)
#define TFHE_DUO_EX2_REGS 0
#endif

// Protocol 3: the lane index as a value hipcc cannot hoist out of the step
// loop, so the transforms' swizzled exchange addresses are computed where they
// are used instead of living (and spilling) beside the prefetched BK row.
DEV int duo_lane(int t) {
#if TFHE_DUO_PROTO == 3
    asm volatile("" : "+v"(t));
#endif
    return t;
}

template <int L, bool SMALL, bool FU>
__global__ __launch_bounds__(512, 1) void k_blind_rotate_duo(
    KParams P, DevTables TT, const uint8_t *__restrict__ ops, const uint32_t *__restrict__ in_a,
    const uint32_t *__restrict__ in_b, const uint32_t *__restrict__ idx, const uint32_t *__restrict__ testvec,
    const double2 *__restrict__ bkd, uint32_t *__restrict__ out, int out_mode, size_t B) {
    static_assert(FU || L == 1, "regrouped row sums need the exact-integer regime");
    constexpr bool EX2LDS = TFHE_DUO_EX2_REGS == 0;
    __shared__ __attribute__((aligned(16))) unsigned char smem[BD_LDS_TOTAL];
    const int tid = threadIdx.x;
    const int t = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int gs = w & 3;  // item slot: waves gs and gs + 4 share a SIMD
    const int h = w >> 2;  // polynomial owned by this wave
    const int pw = w ^ 4;  // partner wave
    double2 *s_bk = reinterpret_cast<double2 *>(smem);
    C2 *s_tw = reinterpret_cast<C2 *>(smem + BD_LDS_BK);
    C2 *s_twist = reinterpret_cast<C2 *>(smem + BD_LDS_BK + BR_LDS_TW);
    unsigned char *bufs = smem + BD_LDS_BUF_AT;
    uint32_t *s_buf = reinterpret_cast<uint32_t *>(bufs + w * BD_LDS_BUF);
    C2 *s_x = reinterpret_cast<C2 *>(s_buf);
    C2 *s_xp = reinterpret_cast<C2 *>(bufs + pw * BD_LDS_BUF);  // partner's buffer (hand-off target)
    uint16_t *s_at = reinterpret_cast<uint16_t *>(bufs + BD_WAVES * BD_LDS_BUF + gs * BD_LDS_AT);
    uint32_t *s_sync = reinterpret_cast<uint32_t *>(smem + BD_LDS_TOTAL - BD_LDS_SYNC);
    uint32_t *s_pub = s_sync, *s_done = s_sync + 2, *s_fwd = s_sync + 4, *s_hand = s_sync + 12;
#if TFHE_DUO_PROTO == 1
    uint32_t *s_cl = s_sync + 24;  // the next unclaimed level
#endif
    int *s_bt = reinterpret_cast<int *>(s_sync + 20);

    if (lds_layout_bad(smem)) {
        if (tid == 0) __hip_atomic_fetch_or(P.err, (uint32_t)DEV_ERR_LDS_LAYOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const int n = P.n;
    const size_t g_raw = (size_t)blockIdx.x * BD_GATES + gs;
    const bool valid = g_raw < B;
    const size_t g = valid ? g_raw : B - 1;  // ragged tail: compute a copy, store nothing
    const size_t ia = idx ? idx[2 * g] : g, ib = idx ? idx[2 * g + 1] : g;
    const uint32_t *A = in_a + ia * (size_t)(n + 1);
    const uint32_t *Bv = in_b ? in_b + ib * (size_t)(n + 1) : A;
    const int op = ops ? (int)ops[g] : 255;
    const size_t step = (size_t)2 * L * 1024;  // double2 per BK[i]
    const uint32_t levels = (uint32_t)n * L;

    auto level_lo = [&](uint32_t k) { return bkd + (size_t)(k / L) * step + (size_t)(k % L) * 1024; };
    auto level_hi = [&](uint32_t k) { return bkd + (size_t)(k / L) * step + (size_t)(L + k % L) * 1024; };
#if TFHE_DUO_PROTO == 1
    if (w == 0) {  // levels 0 and 1 (claimed: cl = 2) and the zeroed counters
        issue_level_full(level_lo(0), level_hi(0), s_bk, t);
        if (levels > 1) issue_level_full(level_lo(1), level_hi(1), s_bk + 2048, t);
        if (t < 20) s_sync[t] = 0u;  // pub, done, fwd, hand (bt: written by the h = 0 waves)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (t == 0) {
            s_pub[0] = 1u;
            s_pub[1] = levels > 1 ? 1u : 0u;
            *s_cl = levels > 1 ? 2u : 1u;
        }
    }
#elif TFHE_DUO_PROTO == 3
    if (w == 0 && t < 20) s_sync[t] = 0u;  // fwd, hand (pub, done unused)
    double2 kr[8][2];
    duo_row_load(kr, bkd + (size_t)h * L * 1024, h, t);  // level 0: row hL of BK[0]
#else
    // every wave's share of levels 0 and 1; published (8 adds per level) before the
    // prologue's second barrier
    if (w == 0 && t < 20) s_sync[t] = 0u;  // pub, done, fwd, hand (bt: written by the h = 0 waves)
    __syncthreads();
    issue_level_share(level_lo(0), level_hi(0), s_bk, w, t);
    if (levels > 1) issue_level_share(level_lo(1), level_hi(1), s_bk + 2048, w, t);
#endif
    for (int x = tid; x < 511; x += 512) s_tw[x] = TT.tw[x];
    for (int x = tid; x < 512; x += 512) s_twist[x] = TT.twist[x];
    if (h == 0) {  // a~_i, b~ (trgsw.zig:297, :312), 64-bit adds
        for (int i = t; i <= n; i += 64) {
            const uint32_t c = gate_combine(op, A[i], Bv[i], i == n);
            const uint32_t tl = (uint32_t)(((uint64_t)c + (1ull << 20)) >> 21);
            if (i < n) s_at[i] = (uint16_t)tl;
            else s_bt[gs] = 2048 - (int)tl;
        }
    }
#if TFHE_DUO_PROTO == 2
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    counter_add(s_pub);
    if (levels > 1) counter_add(s_pub + 1);
#endif
    __syncthreads();  // tables, a~, b~ and the zeroed counters visible to every wave
    const int bt = __builtin_amdgcn_readfirstlane(s_bt[gs]);
    // protocol 3 keeps no BK in LDS: the former slots hold each wave's accumulator
    // (4 KB-aligned), and acc lives in registers only from the hand-off to the
    // step's end (the prefetched BK row takes its registers during the forward phase)
    constexpr bool ACC_LDS = TFHE_DUO_PROTO == 3;
    uint32_t *s_acc = ACC_LDS ? reinterpret_cast<uint32_t *>(smem) + w * 1024 : s_buf;
    uint32_t *s_tmpw = reinterpret_cast<uint32_t *>(smem) + (8 + w) * 1024;  // protocol 3: tmp words too
    uint32_t acc[16];  // acc_h = X^{b~} * testvec_h (trgsw.zig:300-306), lane word m = coefficient t + 64m
#pragma unroll
    for (int m = 0; m < 16; m++) {
        acc[m] = rot_read(testvec + h * 1024, t + 64 * m, bt);
        s_acc[t + 64 * m] = acc[m];
    }
    wave_sync();
    LdsTwAtPass T;
    T.init(s_tw, TT);
    const C2 *twist_t = s_twist + t;
    int at_next = s_at[0];
    uint32_t near = NEAR_NONE;
    uint32_t fail = 0;
    // after one wait gave up (wrong words follow, reported through the device
    // error word), every later wait polls once: a broken protocol ends fast
    const uint32_t spin_cap = P.spin_cap ? P.spin_cap : BR_SPIN_CAP_DEFAULT;
    const uint32_t msbs = digit_msbs(L, P.bgbit);
    const uint32_t buf_base = (uint32_t)(size_t)(lds_void_t *)s_acc;  // 4 KB-aligned (BD_LDS_BUF_AT; smem)
#if TFHE_DUO_PROTO == 1
    // BK levels this wave claimed and has not published yet (at most two: k and k + 1)
    uint32_t owe0 = ~0u, owe1 = ~0u;
    auto publish_owed = [&]() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // my claimed levels' pieces landed
        if (owe0 != ~0u) counter_add(s_pub + (owe0 & 1));
        if (owe1 != ~0u) counter_add(s_pub + (owe1 & 1));
        owe0 = owe1 = ~0u;
    };
    // claim level j (the next unclaimed, cl == j) if its slot is free (all 8 waves done with
    // level j - 2) and issue its whole DMA; false if the slot is busy or another wave won it
    auto try_claim = [&](uint32_t j) {
        if (j >= levels || lds_peek_u32(s_done + (j & 1)) < 8u * (j >> 1)) return false;
        if (lds_cas_u32(s_cl, j, j + 1) != j) return false;
        issue_level_full(level_lo(j), level_hi(j), s_bk + (j & 1) * 2048, t);
        if (owe0 == ~0u) owe0 = j;
        else owe1 = j;
        return true;
    };
#endif

    PhaseProf pp;  // TFHE_PHASE_PROF (tools/phase_prof.hip): per-phase s_memtime per wave
    pp.start();
    for (int i = 0; i < n; i++) {
        pp.mark(0);
        const int at = __builtin_amdgcn_readfirstlane(at_next);
        at_next = s_at[i + 1 < n ? i + 1 : i];
        // tmp_h = X^{a~} acc_h - acc_h + offset (flipped digit fields), in registers
        uint32_t tmp[16], xb[16];
        gather_rot1(buf_base, t, at, xb, tmp);
        if (ACC_LDS) {
#pragma unroll
            for (int m = 0; m < 16; m++) acc[m] = s_acc[t + 64 * m];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 16; m++) {
            const uint32_t sg = gather_sign(xb[m]), off_s = P.offset - sg;
            tmp[m] = tmp_word(tmp[m], sg, off_s, acc[m], msbs);
        }
        if (ACC_LDS) {
#pragma unroll
            for (int m = 0; m < 16; m++) s_tmpw[t + 64 * m] = tmp[m];
        }
        wave_sync();  // the gather's reads precede the exchanges' writes into the buffer
        // partial sums over this wave's rows: po for output h (kept), px for
        // output 1 - h (handed to the partner); fmaInFd1024 accumulates from 0.0
        C2 po[8], px[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            po[q] = c2(0.0, 0.0);
            px[q] = c2(0.0, 0.0);
        }
        pp.mark(1);
#pragma unroll 1
        for (int l = 0; l < L; l++) {
            const uint32_t k = (uint32_t)(L * i + l);  // level k of the launch lives in slot k & 1
            C2 d[1][8];
            if (ACC_LDS) {
#pragma unroll
                for (int m = 0; m < 16; m++) tmp[m] = s_tmpw[t + 64 * m];
            }
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const int m = br3(q);
                d[0][q] = twist_in<FU>(digit_f64_flipped(tmp[m], l, P.bgbit), digit_f64_flipped(tmp[m + 8], l, P.bgbit),
                                       twist_t[64 * m]);
            }
#ifndef TFHE_KO_FFT
            fft512<1, false, FU, LdsTwAtPass, EX2LDS>(d, s_x, T, duo_lane(t));
#endif
            if (l == L - 1) counter_add(s_fwd + w);  // my exchanges are done: the partner may write my buffer
            pp.mark(2);
#if TFHE_DUO_PROTO == 1
            // checkpoint: publish the levels I claimed (they had a forward FFT's time to
            // land), then claim levels k and k + 1 if their slots are free and nobody has
            if (owe0 != ~0u) publish_owed();
            pp.mark(3);
            {
                uint32_t c = lds_peek_u32(s_cl);
                if (c == k && try_claim(k)) c = k + 1;
                if (c == k + 1) try_claim(k + 1);
            }
            if (owe0 == k) publish_owed();  // I claimed level k only now: it must land before my MAC
            pp.mark(4);
            // level k published (by its claimer); if nobody could claim it (slot busy), claim it here
            {
                uint32_t cap = fail ? 1u : spin_cap;
                while (lds_peek_u32(s_pub + (k & 1)) < (k >> 1) + 1u) {
                    if (lds_peek_u32(s_cl) == k && try_claim(k)) {
                        publish_owed();
                        continue;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    if (--cap == 0) {
                        fail = 1;
                        break;
                    }
                }
            }
#elif TFHE_DUO_PROTO == 2
            // level k was published at the end of level k - 1 by every wave
            DUO_SPIN(s_pub + (k & 1), 8u * ((k >> 1) + 1u), fail ? 1u : spin_cap, fail);
#endif
            __builtin_amdgcn_sched_barrier(0);
            pp.mark(5);
#if TFHE_DUO_PROTO == 3
#ifndef TFHE_KO_MAC
            mac_row_regs<FU>(po, px, d[0], kr);
#endif
#ifndef TFHE_KO_DUO_LOAD  // knock-out timing build: the prologue's row reused (wrong words)
            if (k + 1 < levels)  // the next level's row, under the next transform (or the inverse)
                duo_row_load(kr, bkd + (size_t)((k + 1) / L) * step + (size_t)(h * L + (k + 1) % L) * 1024, h, t);
#endif
#else
#ifndef TFHE_KO_MAC
            // row hL + l, parts [q][a|b][lane]: output h's part at +64h, the other's at +64(1-h)
            mac_row_roles<FU>(po, px, d[0], s_bk + (k & 1) * 2048 + h * 1024 + 64 * h, s_bk + (k & 1) * 2048 + h * 1024 + 64 * (1 - h), t);
#endif
            __builtin_amdgcn_sched_barrier(0);
            counter_add(s_done + (k & 1));
#endif
#if TFHE_DUO_PROTO == 2
            pp.mark(3);
            // end of level k: its slot takes level k + 2 once all 8 waves are through
            // level k (this wait is the level's one synchronisation), and level k + 1,
            // issued a level ago, is published
            if (k + 2 < levels) {
                DUO_SPIN(s_done + (k & 1), 8u * ((k >> 1) + 1u), fail ? 1u : spin_cap, fail);
                issue_level_share(level_lo(k + 2), level_hi(k + 2), s_bk + (k & 1) * 2048, w, t);
                if (k >= 1) {
                    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                    counter_add(s_pub + ((k + 1) & 1));
                }
            } else if (k >= 1 && k + 1 < levels) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                counter_add(s_pub + ((k + 1) & 1));
            }
#endif
            pp.mark(1);
        }
        pp.mark(6);
        // hand-off: P_h,(1-h) into the partner's buffer, the partner's into mine
        DUO_SPIN(s_fwd + pw, (uint32_t)i + 1u, fail ? 1u : spin_cap, fail);
#pragma unroll
        for (int q = 0; q < 8; q++) s_xp[t + 64 * q] = px[q];
        counter_add(s_hand + w);
        DUO_SPIN(s_hand + pw, (uint32_t)i + 1u, fail ? 1u : spin_cap, fail);
        __builtin_amdgcn_sched_barrier(0);
        // output h = (rows 0..L-1) + (rows L..2L-1); IEEE addition commutes, so
        // mine + other is that sum for either h
        C2 e[1][8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const int m = br3(q);
            const C2 o = s_x[t + 64 * m];
            const C2 mine = po[m];
            e[0][q] = c2(mine.x + o.x, mine.y + o.y);
        }
        if (ACC_LDS) {  // back into registers for the update, landing under the inverse transform
#pragma unroll
            for (int m = 0; m < 16; m++) acc[m] = s_acc[t + 64 * m];
        }
        wave_sync();  // the partial's reads precede the inverse's exchange writes
        pp.mark(7);
#ifndef TFHE_KO_INV
        fft512<1, true, FU, LdsTwAtPass, EX2LDS>(e, s_x, T, duo_lane(t));
#endif
        uint32_t nq[2] = {NEAR_NONE, NEAR_NONE};
#pragma unroll
        for (int q = 0; q < 8; q++) {
            double re, im;
            untwist_out<false, FU>(e[0][q], twist_t[64 * q], re, im);
            acc[q] += to_torus<SMALL, FU>(re, nq[0]);
            acc[q + 8] += to_torus<SMALL, FU>(im, nq[1]);
        }
        near &= nq[0] & nq[1];
        wave_sync();
#pragma unroll
        for (int m = 0; m < 16; m++) s_acc[t + 64 * m] = acc[m];
        wave_sync();
    }
    pp.mark(0);
#ifdef TFHE_PHASE_PROF
    if (t == 0)
        for (int k = 0; k < 8; k++) atomicAdd(&g_phase_cycles[k], (unsigned long long)pp.acc[k]);
#endif
    report_wait_failure(P, fail, DEV_ERR_GATE_WAIT);
    if (FU) near_tie_flag(P, near, g, valid);

    if (!valid) return;
    if (out_mode == BR_OUT_LV1) {  // sampleExtractIndex(acc, 0): p[0] = a[0], p[j] = -a[N-j], p[N] = b[0]
        uint32_t *o = out + g * (size_t)1025;
        if (h == 0) {
            for (int j = t; j < 1024; j += 64) o[j] = j == 0 ? s_acc[0] : 0u - s_acc[1024 - j];
        } else if (t == 0) {
            o[1024] = s_acc[0];
        }
    } else if (out_mode == BR_OUT_LV0_EXTRACT2) {  // sampleExtractIndex2 (trlwe.zig:165-180)
        uint32_t *o = out + g * (size_t)(n + 1);
        if (h == 0) {
            for (int j = t; j < n; j += 64) o[j] = j == 0 ? s_acc[0] : 0u - s_acc[n - j];
        } else if (t == 0) {
            o[n] = s_acc[0];
        }
    } else {
        uint32_t *o = out + g * (size_t)2048 + h * 1024;
        for (int j = t; j < 1024; j += 64) o[j] = s_acc[j];
    }
}

// ---------------------------------------------------------------------------
// Blind rotation, latency form ("wide"): ONE item per 512-thread workgroup,
// for batches too small to give every SIMD a gate (circuit levels, single
// gates).  Per CMUX step:
//   waves r < 2L : row r's digits (rotation gathered from the LDS accumulator)
//                  and forward transform, spectrum published in slot r
//   all 8 waves  : MAC of 64 frequencies each (t + 64w) over rows 0..2L-1 in
//                  the reference's order, BK words streamed from HBM/L2 into
//                  registers one step ahead; products written over slots 0/1
//   waves 0, 1   : inverse transform of polynomial w and the CMUX add
// Same arithmetic as the other forms, bit for bit.
// ---------------------------------------------------------------------------
constexpr int BW_WAVES = 8;
constexpr size_t BR_WIDE_MAX_ITEMS = 512;  // measured: 1 gate 4.3 vs 9.9 ms; 512 gates 8.8 vs 10.2 ms; 1024: 17.1 vs 10.4 ms

// Row wave w's BK row of the coming step: parts a|b, every frequency t + 64q.
DEV void wide_prefetch(double2 (*kr)[2], const double2 *__restrict__ nb, int w, int t) {
#pragma unroll
    for (int q = 0; q < 8; q++)
#pragma unroll
        for (int h = 0; h < 2; h++) kr[q][h] = nb[((size_t)w * 8 + q) * 128 + h * 64 + t];
}
#ifndef WIDE_INV_W0  // A/B: 0 = the round-2 inverse waves 0, 1
#define WIDE_INV_W0 2
#endif
#ifndef WIDE_ROW45_PRIO  // A/B: issue priority of the row waves 4 and 5 (0 = the default, as every wave)
#define WIDE_ROW45_PRIO 1
#endif
#ifndef WIDE_PF_LATE_MASK  // A/B: 0 = every row wave prefetches right after its terms (round-2 schedule)
#define WIDE_PF_LATE_MASK 0xff
#endif

template <int L, bool SMALL, bool FU = false>
__global__ __launch_bounds__(512, 1) void k_blind_rotate_wide(
    KParams P, DevTables TT, const uint8_t *__restrict__ ops, const uint32_t *__restrict__ in_a,
    const uint32_t *__restrict__ in_b, const uint32_t *__restrict__ idx, const uint32_t *__restrict__ testvec,
    const double2 *__restrict__ bkd, uint32_t *__restrict__ out, int out_mode, size_t B) {
    __shared__ __attribute__((aligned(16))) C2 s_tw[512];
    __shared__ __attribute__((aligned(16))) C2 s_twist[512];
    // row r's product spectra (a, b) in s_prod[0/1][r]; s_prod[0][r] is also row
    // wave r's FFT exchange buffer, and slots 0/1 of s_prod[0] receive the sums
    __shared__ __attribute__((aligned(16))) C2 s_prod[2][2 * L][512];
    __shared__ __attribute__((aligned(16))) uint32_t s_acc[2048];
    __shared__ uint16_t s_at[1024];
    __shared__ int s_bt;
    const int tid = threadIdx.x;
    const int t = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n = P.n;
    const size_t g = blockIdx.x;
    const size_t ia = idx ? idx[2 * g] : g, ib = idx ? idx[2 * g + 1] : g;
    const uint32_t *A = in_a + ia * (size_t)(n + 1);
    const uint32_t *Bv = in_b ? in_b + ib * (size_t)(n + 1) : A;
    const int op = ops ? (int)ops[g] : 255;
    const size_t trgsw = (size_t)2 * L * 1024;  // double2 per BK[i]

    for (int x = tid; x < 511; x += 512) s_tw[x] = TT.tw[x];
    for (int x = tid; x < 512; x += 512) s_twist[x] = TT.twist[x];
    if (w == 0) {
        for (int i = t; i <= n; i += 64) {
            uint32_t c = gate_combine(op, A[i], Bv[i], i == n);
            uint32_t tl = (uint32_t)(((uint64_t)c + (1ull << 20)) >> 21);
            if (i < n) s_at[i] = (uint16_t)tl;
            else s_bt = 2048 - (int)tl;
        }
    }
    // row wave r's BK words of step 0: row r, parts a|b, every frequency t + 64q
    double2 kr[8][2];
    if (w < 2 * L) {
#pragma unroll
        for (int q = 0; q < 8; q++)
#pragma unroll
            for (int h = 0; h < 2; h++) kr[q][h] = bkd[((size_t)w * 8 + q) * 128 + h * 64 + t];
    }
    __syncthreads();
    const int bt = __builtin_amdgcn_readfirstlane(s_bt);
    if (w < 2) {
#pragma unroll
        for (int m = 0; m < 16; m++) s_acc[w * 1024 + t + 64 * m] = rot_read(testvec + w * 1024, t + 64 * m, bt);
    }
    LdsTw T;
    T.init(s_tw, TT);
    const C2 *twist_t = s_twist + t;
    __syncthreads();
    // inverse waves: WIDE_INV_W0 and WIDE_INV_W0 + 1 transform polynomials 0 and 1.
    // Waves 2 and 3 by default: their SIMDs carry one row wave, those of waves
    // 0 and 1 two (rows 4, 5), and the other row waves' BK prefetch issues during
    // the inverse phase on SIMDs the inverse does not use.
    const int ipoly = w - WIDE_INV_W0;
    const bool is_inv = ipoly == 0 || ipoly == 1;
    // row waves that issue their BK prefetch in the inverse phase (the others
    // right after their terms)
    const bool pf_late = w < 2 * L && !is_inv && ((WIDE_PF_LATE_MASK >> w) & 1);
    // the inverse waves keep their polynomial's 16 accumulator words per lane
    // in registers: the update then waits for no LDS read
    uint32_t accr[16];
    if (is_inv) {
#pragma unroll
        for (int m = 0; m < 16; m++) accr[m] = s_acc[ipoly * 1024 + t + 64 * m];
    }

#if WIDE_ROW45_PRIO
    // rows 4 and 5 share their SIMDs with rows 0 and 1 and finish the forward
    // phase last; at a higher issue priority they take the VALU first
    if (w == 4 || w == 5) __builtin_amdgcn_s_setprio(WIDE_ROW45_PRIO);
#endif
    int at_next = s_at[0];  // a~ read one step ahead (its wait would drain every LDS op)
    uint32_t near = NEAR_NONE;  // FU: margin guard (the inverse waves)
    PhaseProf pp;  // development timing (TFHE_PHASE_PROF), per wave
    pp.start();
    for (int i = 0; i < n; i++) {
        pp.mark(0);
        const int at = __builtin_amdgcn_readfirstlane(at_next);
        at_next = s_at[i + 1 < n ? i + 1 : i];
        if (w < 2 * L) {
            const int poly = w >= L ? 1 : 0;
            const int level = w - poly * L;
            const uint32_t *pa = s_acc + poly * 1024;
            // gathers and own words first, arithmetic after (one wait)
            uint32_t rot[16], own[16];
            pp.mark(8);
            const int rb = (t - at) & 2047;
#pragma unroll
            for (int m = 0; m < 16; m++) {
                rot[m] = pa[(rb + 64 * m) & 1023];
                own[m] = pa[t + 64 * m];
            }
            __builtin_amdgcn_sched_barrier(0);
            pp.mark(9);
            C2 d[1][8];
            const uint32_t msbs = digit_msbs(L, P.bgbit);  // flipped tmp words: one v_bfe_i32 per digit
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const int m = br3(q);
                const bool n0 = ((rb + 64 * m) & 1024) != 0, n1 = ((rb + 64 * (m + 8)) & 1024) != 0;
                const uint32_t x0 = ((n0 ? 0u - rot[m] : rot[m]) - own[m] + P.offset) ^ msbs;
                const uint32_t x1 = ((n1 ? 0u - rot[m + 8] : rot[m + 8]) - own[m + 8] + P.offset) ^ msbs;
                d[0][q] = twist_in<FU>(digit_f64_flipped(x0, level, P.bgbit), digit_f64_flipped(x1, level, P.bgbit),
                                       twist_t[64 * m]);
            }
            pp.mark(10);
            fft512<1, false, FU>(d, s_prod[0][w], T, t);
            pp.mark(11);
            // this row's terms of fmaInFd1024 for both outputs, every frequency
            // (after this wave's exchanges in s_prod[0][w])
#pragma unroll
            for (int q = 0; q < 8; q++) {
                s_prod[0][w][t + 64 * q] = cmul_bk<FU>(d[0][q], kr[q][0]);
                s_prod[1][w][t + 64 * q] = cmul_bk<FU>(d[0][q], kr[q][1]);
            }
            pp.mark(14);
#ifndef TFHE_KO_WIDE_PREFETCH
            // next step's BK row, landing under the sum, inverse and forward
            // phases.  The inverse waves (2, 3) issue it here; the other row
            // waves wait for the inverse phase, where they are idle: 16 KB per
            // wave through the CU's vector-memory path no longer queues behind
            // 5 other waves' at the end of the forward phase, which is the
            // critical path (rows 4 and 5 share SIMDs with rows 0 and 1):
            // 104.7 -> 101.8 ms per 16-bit adder with the inverse on waves 2, 3
            // (profiles/r03q_wide_prefetch_inverse.txt).
            if (i + 1 < n && !pf_late) wide_prefetch(kr, bkd + (size_t)(i + 1) * trgsw, w, t);
#endif
        }
        pp.mark(1);
        __syncthreads();  // every row's terms are in place
        pp.mark(2);
        // sum in the reference's row order 0..2L-1 (fmaInFd1024 starts from 0.0: 0.0 + x == x)
        const int f = t + 64 * w;
        C2 fa = s_prod[0][0][f], fb = s_prod[1][0][f];
#pragma unroll
        for (int r = 1; r < 2 * L; r++) {
            const C2 ta = s_prod[0][r][f], tb = s_prod[1][r][f];
            fa = c2(fa.x + ta.x, fa.y + ta.y);
            fb = c2(fb.x + tb.x, fb.y + tb.y);
        }
        // frequency f of slots 0/1 is read above and rewritten here by this lane only
        s_prod[0][0][f] = fa;
        s_prod[0][1][f] = fb;
        pp.mark(3);
        __syncthreads();  // both product spectra complete
        pp.mark(4);
#ifndef TFHE_KO_WIDE_PREFETCH
        if (pf_late && i + 1 < n) wide_prefetch(kr, bkd + (size_t)(i + 1) * trgsw, w, t);
#endif
        if (is_inv) {
            C2 e[1][8];
#pragma unroll
            for (int q = 0; q < 8; q++) e[0][q] = s_prod[0][ipoly][t + 64 * br3(q)];
            C2 twr[8];  // untwist factors, read before the transform: their latency hides behind it
#pragma unroll
            for (int q = 0; q < 8; q++) twr[q] = twist_t[64 * q];
            pp.mark(12);
            fft512<1, true, FU>(e, s_prod[0][ipoly], T, t);
            pp.mark(13);
            uint32_t *pa = s_acc + ipoly * 1024;
#pragma unroll
            for (int q = 0; q < 8; q++) {
                double re, im;
                untwist_out<false, FU>(e[0][q], twr[q], re, im);
                accr[q] += to_torus<SMALL, FU>(re, near);
                accr[q + 8] += to_torus<SMALL, FU>(im, near);
                pa[t + 64 * q] = accr[q];
                pa[t + 64 * q + 512] = accr[q + 8];
            }
        }
        pp.mark(5);
        __syncthreads();  // accumulator updated
    }
    pp.mark(6);
#ifdef TFHE_PHASE_PROF
    if (t == 0)
        for (int k = 0; k < 16; k++) atomicAdd(&g_phase_cycles[w * 16 + k], (unsigned long long)pp.acc[k]);
#endif
    if (FU) near_tie_flag(P, near, g, true);

    if (w != 0) return;
    if (out_mode == BR_OUT_LV1) {
        uint32_t *o = out + g * (size_t)1025;
        for (int j = t; j <= 1024; j += 64) o[j] = j == 0 ? s_acc[0] : j < 1024 ? 0u - s_acc[1024 - j] : s_acc[1024];
    } else if (out_mode == BR_OUT_LV0_EXTRACT2) {
        uint32_t *o = out + g * (size_t)(n + 1);
        for (int j = t; j <= n; j += 64) o[j] = j == 0 ? s_acc[0] : j < n ? 0u - s_acc[n - j] : s_acc[1024];
    } else {
        uint32_t *o = out + g * (size_t)2048;
        for (int j = t; j < 2048; j += 64) o[j] = s_acc[j];
    }
}

// ---------------------------------------------------------------------------
// Identity key switching (trgsw.zig:471-502):
//   res = (0,...,0, b) - sum_{i<N, j<t} KSK[i][j][digit_j(a_i + 2^(32-(1+basebit*t)))]
// Integer gather-subtract; the k = 0 rows of the device KSK are zero (the
// reference skips them, trgsw.zig:490), so every (i, j) subtracts
// unconditionally.  Lane = output word (n+1 words per item), G items per
// block.  All t digits of a_i are the top basebit*t bits of a_i + prec, so
// one shift gives them packed.
// ---------------------------------------------------------------------------
// Select form (2^basebit <= 4): per (i, j) a lane loads the 3 non-zero
// candidate words once; each of the G items then picks its word by its
// wave-uniform digit (readlane -> SGPR), so KSK traffic is per block, not per
// item.
// ---------------------------------------------------------------------------
// Latency form with split transforms (round 4, "wide2"; L = 3): the 6 forward
// transforms of a step occupy the 4 SIMDs evenly and the 2 inverse transforms
// all 4, because rows 4 and 5 and both inverse transforms each run as TWO half
// transforms on two waves of different SIMDs (the round-3
// form put rows 4 and 5 beside rows 0 and 1 and the inverse on 2 SIMDs).
// Half h of a 512-point transform holds positions 256h .. 256h + 255 of the
// bit-reversed DIT array, 4 per lane: stages 1-8 never mix the halves (4 register
// passes of 2 stages, 3 exchanges through the half's own 4 KB), and stage 9
// pairs position p with p + 256 through a 4 KB buffer per half and an LDS counter
// per half.  Every butterfly is the reference's, with its recurrence twiddle,
// in the same arithmetic as fft512 (the general butterfly equals bf1 / bf_m1 on
// the exact (1, 0) and (x, -1) twiddles), so the words are the whole form's.
// Layouts of a half (position bits b0..b7 within it; r = register, t = lane):
//   P1: r = (b0, b1), t = (b2..b7):           p = r + 4t
//   P2: r = (b2, b3), t = (b0, b1, b4..b7):   p = (t & 3) + 4r + 16(t >> 2)
//   P3: r = (b4, b5), t = (b0..b3, b6, b7):   p = (t & 15) + 16r + 64(t >> 4)
//   P4: r = (b6, b7), t = (b0..b5):           p = t + 64r  (output order)
// The input of P1 at (t, r) is transform index k = bitrev9(p + 256h) =
// h + 2 br6(t) + 128 br2(r).  Exchange e stores position p at 16-B slot
// swz_h<e>(p), an XOR swizzle (searched) under which both its ds_write_b128
// (P_e) and its ds_read_b128 (P_e+1) are bank-conflict-free.
// ---------------------------------------------------------------------------
constexpr uint32_t HSWZ[3][4] = {{0xba, 0xbc, 0x28, 0xe0}, {0x9c, 0xc8, 0x50, 0x50}, {0x88, 0x00, 0xc0, 0x40}};
template <int E>
DEV constexpr uint32_t swz_h(uint32_t p) {
    uint32_t x = 0;
    for (int i = 0; i < 4; i++) x |= (uint32_t)(__builtin_popcount(p & HSWZ[E][i]) & 1) << i;
    return p ^ x;
}
DEV int br2(int r) { return ((r & 1) << 1) | (r >> 1); }
DEV uint32_t hp1(int t, int r) { return (uint32_t)(r + 4 * t); }
DEV uint32_t hp2(int t, int r) { return (uint32_t)((t & 3) + 4 * r + 16 * (t >> 2)); }
DEV uint32_t hp3(int t, int r) { return (uint32_t)((t & 15) + 16 * r + 64 * (t >> 4)); }
DEV uint32_t hp4(int t, int r) { return (uint32_t)(t + 64 * r); }

// exchange E of a half: this lane's 4 points at their slots, then the next layout's
template <int E>
DEV void half_exchange(C2 *d, C2 *xb, int t) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const uint32_t p = E == 0 ? hp1(t, r) : E == 1 ? hp2(t, r) : hp3(t, r);
        xb[swz_h<E>(p)] = d[r];
    }
    wave_sync();
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const uint32_t p = E == 0 ? hp2(t, r) : E == 1 ? hp3(t, r) : hp4(t, r);
        d[r] = xb[swz_h<E>(p)];
    }
    wave_sync();
}

// Stages 1-8 of half a transform (forward, or INV with the conjugate twiddles).
// In: P1 with d[r] = point k(t, r); out: P4.  tw = the LDS stage table
// (index len/2 - 1 + j), a1 = W4[1]'s real part (imaginary part exactly -1).
template <bool INV, bool FU>
DEV void half_fft_1to8(C2 *d, C2 *xb, const C2 *tw, double a1, int t) {
    // pass 1: len 2 (b0), len 4 (b1): the twiddles are lane-uniform, as in passA
    bf1<FU>(d[0], d[1]);
    bf1<FU>(d[2], d[3]);
    bf1<FU>(d[0], d[2]);
    bf_m1<INV, FU>(d[1], d[3], a1);
    half_exchange<0>(d, xb, t);
    {  // pass 2: len 8 (b2 = r bit 0), len 16 (b3 = r bit 1); j0 = b0 + 2 b1 = t & 3
        const int j0 = t & 3;
        const C2 w8 = tw[3 + j0], w16a = tw[7 + j0], w16b = tw[7 + j0 + 4];
        bf<INV, FU>(d[0], d[1], w8);
        bf<INV, FU>(d[2], d[3], w8);
        bf<INV, FU>(d[0], d[2], w16a);
        bf<INV, FU>(d[1], d[3], w16b);
    }
    half_exchange<1>(d, xb, t);
    {  // pass 3: len 32 (b4), len 64 (b5); j0 = b0..b3 = t & 15
        const int j0 = t & 15;
        const C2 w32 = tw[15 + j0], w64a = tw[31 + j0], w64b = tw[31 + j0 + 16];
        bf<INV, FU>(d[0], d[1], w32);
        bf<INV, FU>(d[2], d[3], w32);
        bf<INV, FU>(d[0], d[2], w64a);
        bf<INV, FU>(d[1], d[3], w64b);
    }
    half_exchange<2>(d, xb, t);
    {  // pass 4: len 128 (b6), len 256 (b7); j0 = b0..b5 = t
        const C2 w128 = tw[63 + t], w256a = tw[127 + t], w256b = tw[127 + t + 64];
        bf<INV, FU>(d[0], d[1], w128);
        bf<INV, FU>(d[2], d[3], w128);
        bf<INV, FU>(d[0], d[2], w256a);
        bf<INV, FU>(d[1], d[3], w256b);
    }
}

// Stage 9 (len 512) across the two halves: position p = t + 64r of half 0 pairs
// with p + 256 of half 1 (twiddle W512[p]).  Both halves write their P4 points
// to their own 4 KB (mine), publish a counter, wait for the partner's, and
// compute the butterfly from (half 0's, half 1's) points: half 0 keeps a, half 1
// b = 2u - a (it computes a too: the same expression, the same bits).
template <bool INV, bool FU>
DEV void half_fft_9(C2 *d, C2 *mine, const C2 *other, uint32_t *cnt_mine, const uint32_t *cnt_other,
                    uint32_t target, const C2 *tw, int h, int t, uint32_t cap, uint32_t &fail) {
#pragma unroll
    for (int r = 0; r < 4; r++) mine[t + 64 * r] = d[r];
    counter_add(cnt_mine);  // in order after this wave's stores
    spin_until_ge(cnt_other, target, cap, fail);
    __builtin_amdgcn_sched_barrier(0);
    // a uniform branch, not selects (a select of the C2 objects went through scratch)
    if (h == 0) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            C2 x = other[t + 64 * r];
            bf<INV, FU>(d[r], x, tw[255 + t + 64 * r]);
        }
    } else {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            C2 u = other[t + 64 * r];
            bf<INV, FU>(u, d[r], tw[255 + t + 64 * r]);
        }
    }
}

template <int L, bool SMALL, bool FU = false>
__global__ __launch_bounds__(512, 1) void k_blind_rotate_wide2(
    KParams P, DevTables TT, const uint8_t *__restrict__ ops, const uint32_t *__restrict__ in_a,
    const uint32_t *__restrict__ in_b, const uint32_t *__restrict__ idx, const uint32_t *__restrict__ testvec,
    const double2 *__restrict__ bkd, uint32_t *__restrict__ out, int out_mode, size_t B) {
    static_assert(L == 3, "split rows 4 and 5: 2L = 6");
    __shared__ __attribute__((aligned(16))) C2 s_tw[512];
    __shared__ __attribute__((aligned(16))) C2 s_twist[512];
    // row r's term spectra (a, b) in s_prod[0/1][r]; s_prod[0][r] is also row r's
    // exchange buffer (split rows: half h uses its 4 KB); slots 0/1 of s_prod[0]
    // receive the sums; the inverse halves exchange through s_prod[1][poly]
    __shared__ __attribute__((aligned(16))) C2 s_prod[2][2 * L][512];
    __shared__ __attribute__((aligned(16))) C2 s_x9[2][512];  // stage 9: [split row or inverse poly][half]
    __shared__ __attribute__((aligned(16))) uint32_t s_acc[2048];
    __shared__ uint16_t s_at[1024];
    __shared__ uint32_t s_cnt[2][2][2];  // stage-9 counters [forward / inverse][row or poly][half]
    __shared__ int s_bt;
    const int tid = threadIdx.x;
    const int t = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n = P.n;
    const size_t g = blockIdx.x;
    const size_t ia = idx ? idx[2 * g] : g, ib = idx ? idx[2 * g + 1] : g;
    const uint32_t *A = in_a + ia * (size_t)(n + 1);
    const uint32_t *Bv = in_b ? in_b + ib * (size_t)(n + 1) : A;
    const int op = ops ? (int)ops[g] : 255;
    const size_t trgsw = (size_t)2 * L * 1024;  // double2 per BK[i]
    // roles: waves 0-3 transform rows 0-3 whole and run the inverse halves
    // (wave 2p + h: polynomial p, half h); waves 4-7 transform rows 4 and 5 in
    // halves (wave 4 + 2h + s: row 4 + s, half h), one beside each full row on its SIMD
    const bool full = w < 4;
    const int hrow = 4 + (w & 1), hh = (w >> 1) & 1;  // split-row role of waves 4-7
    const int ipoly = w >> 1, ih = w & 1;             // inverse role of waves 0-3
    const uint32_t spin_cap = P.spin_cap ? P.spin_cap : BR_SPIN_CAP_DEFAULT;
    uint32_t fail = 0;

    for (int x = tid; x < 511; x += 512) s_tw[x] = TT.tw[x];
    for (int x = tid; x < 512; x += 512) s_twist[x] = TT.twist[x];
    if (tid < 8) (&s_cnt[0][0][0])[tid] = 0u;
    if (w == 0) {
        for (int i = t; i <= n; i += 64) {
            uint32_t c = gate_combine(op, A[i], Bv[i], i == n);
            uint32_t tl = (uint32_t)(((uint64_t)c + (1ull << 20)) >> 21);
            if (i < n) s_at[i] = (uint16_t)tl;
            else s_bt = 2048 - (int)tl;
        }
    }
    // BK words of step 0: full rows every frequency t + 64q, split halves q = 4h + r
    double2 kr[8][2];
    if (full) {
        wide_prefetch(kr, bkd, w, t);
    } else {
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int p = 0; p < 2; p++) kr[r][p] = bkd[((size_t)hrow * 8 + 4 * hh + r) * 128 + p * 64 + t];
    }
    __syncthreads();
    const int bt = __builtin_amdgcn_readfirstlane(s_bt);
    if (w < 2) {
#pragma unroll
        for (int m = 0; m < 16; m++) s_acc[w * 1024 + t + 64 * m] = rot_read(testvec + w * 1024, t + 64 * m, bt);
    }
    LdsTw T;
    T.init(s_tw, TT);
    const C2 *twist_t = s_twist + t;
    __syncthreads();
    // inverse halves keep their 8 accumulator words per lane in registers:
    // coefficients p = 256 ih + t + 64r (r < 4) and p + 512
    uint32_t accr[8];
    if (full) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            accr[r] = s_acc[ipoly * 1024 + 256 * ih + t + 64 * r];
            accr[r + 4] = s_acc[ipoly * 1024 + 512 + 256 * ih + t + 64 * r];
        }
    }
    const uint32_t msbs = digit_msbs(L, P.bgbit);
    const double a1 = TT.twa[0].x;  // W4[1] = (a1, -1)

    int at_next = s_at[0];
    uint32_t near = NEAR_NONE;
    for (int i = 0; i < n; i++) {
        const int at = __builtin_amdgcn_readfirstlane(at_next);
        at_next = s_at[i + 1 < n ? i + 1 : i];
        if (full) {  // row w, whole transform (as k_blind_rotate_wide)
            const int poly = w >= L ? 1 : 0;
            const int level = w - poly * L;
            const uint32_t *pa = s_acc + poly * 1024;
            uint32_t rot[16], own[16];
            const int rb = (t - at) & 2047;
#pragma unroll
            for (int m = 0; m < 16; m++) {
                rot[m] = pa[(rb + 64 * m) & 1023];
                own[m] = pa[t + 64 * m];
            }
            __builtin_amdgcn_sched_barrier(0);
            C2 d[1][8];
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const int m = br3(q);
                const bool n0 = ((rb + 64 * m) & 1024) != 0, n1 = ((rb + 64 * (m + 8)) & 1024) != 0;
                const uint32_t x0 = ((n0 ? 0u - rot[m] : rot[m]) - own[m] + P.offset) ^ msbs;
                const uint32_t x1 = ((n1 ? 0u - rot[m + 8] : rot[m + 8]) - own[m + 8] + P.offset) ^ msbs;
                d[0][q] = twist_in<FU>(digit_f64_flipped(x0, level, P.bgbit), digit_f64_flipped(x1, level, P.bgbit),
                                       twist_t[64 * m]);
            }
            fft512<1, false, FU>(d, s_prod[0][w], T, t);
#pragma unroll
            for (int q = 0; q < 8; q++) {
                s_prod[0][w][t + 64 * q] = cmul_bk<FU>(d[0][q], kr[q][0]);
                s_prod[1][w][t + 64 * q] = cmul_bk<FU>(d[0][q], kr[q][1]);
            }
#ifndef TFHE_KO_WIDE_PREFETCH
            if (i + 1 < n) wide_prefetch(kr, bkd + (size_t)(i + 1) * trgsw, w, t);
#endif
        } else {  // row hrow, half hh
            const uint32_t *pa = s_acc + 1024;  // rows 4, 5: polynomial b, levels 1, 2
            const int level = hrow - L;
            const int kb = hh + 2 * br6(t);  // P1 point (t, r) = transform index kb + 128 br2(r)
            uint32_t rot[8], own[8];
#pragma unroll
            for (int m = 0; m < 8; m++) {  // coefficients kb + 128m: k for m < 4, k + 512 for m >= 4
                const int c = kb + 128 * m;
                rot[m] = pa[(c - at) & 1023];
                own[m] = pa[c];
            }
            __builtin_amdgcn_sched_barrier(0);
            C2 d[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int m = br2(r), c0 = kb + 128 * m, c1 = c0 + 512;
                const bool n0 = ((c0 - at) & 1024) != 0, n1 = ((c1 - at) & 1024) != 0;
                const uint32_t x0 = ((n0 ? 0u - rot[m] : rot[m]) - own[m] + P.offset) ^ msbs;
                const uint32_t x1 = ((n1 ? 0u - rot[m + 4] : rot[m + 4]) - own[m + 4] + P.offset) ^ msbs;
                d[r] = twist_in<FU>(digit_f64_flipped(x0, level, P.bgbit), digit_f64_flipped(x1, level, P.bgbit),
                                    s_twist[c0]);
            }
            C2 *xb = &s_prod[0][hrow][256 * hh];
#ifndef TFHE_KO_FFT
            half_fft_1to8<false, FU>(d, xb, s_tw, a1, t);
            half_fft_9<false, FU>(d, &s_x9[hrow - 4][256 * hh], &s_x9[hrow - 4][256 * (1 - hh)],
                                  &s_cnt[0][hrow - 4][hh], &s_cnt[0][hrow - 4][1 - hh], (uint32_t)i + 1u, s_tw, hh, t,
                                  fail ? 1u : spin_cap, fail);
#endif
            // terms at frequencies f = 256 hh + t + 64r (after this wave's exchanges in xb)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                s_prod[0][hrow][256 * hh + t + 64 * r] = cmul_bk<FU>(d[r], kr[r][0]);
                s_prod[1][hrow][256 * hh + t + 64 * r] = cmul_bk<FU>(d[r], kr[r][1]);
            }
        }
        __syncthreads();  // every row's terms are in place
        // sum in the reference's row order 0..2L-1 (fmaInFd1024 starts from 0.0: 0.0 + x == x)
        const int f = t + 64 * w;
        C2 fa = s_prod[0][0][f], fb = s_prod[1][0][f];
#pragma unroll
        for (int r = 1; r < 2 * L; r++) {
            const C2 ta = s_prod[0][r][f], tb = s_prod[1][r][f];
            fa = c2(fa.x + ta.x, fa.y + ta.y);
            fb = c2(fb.x + tb.x, fb.y + tb.y);
        }
        s_prod[0][0][f] = fa;
        s_prod[0][1][f] = fb;
        __syncthreads();  // both product spectra complete
        if (!full) {
#ifndef TFHE_KO_WIDE_PREFETCH
            if (i + 1 < n) {  // next step's BK half row, issued in the inverse phase (these waves are idle)
#pragma unroll
                for (int r = 0; r < 4; r++)
#pragma unroll
                    for (int p = 0; p < 2; p++)
                        kr[r][p] = bkd[(size_t)(i + 1) * trgsw + ((size_t)hrow * 8 + 4 * hh + r) * 128 + p * 64 + t];
            }
#endif
        } else {  // inverse half ih of polynomial ipoly
            const int kb = ih + 2 * br6(t);
            C2 e[4], twr[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                e[r] = s_prod[0][ipoly][kb + 128 * br2(r)];
                twr[r] = twist_t[256 * ih + 64 * r];  // untwist of output coefficient 256 ih + t + 64r
            }
            C2 *xb = &s_prod[1][ipoly][256 * ih];
#ifndef TFHE_KO_INV
            half_fft_1to8<true, FU>(e, xb, s_tw, a1, t);
            half_fft_9<true, FU>(e, &s_x9[ipoly][256 * ih], &s_x9[ipoly][256 * (1 - ih)], &s_cnt[1][ipoly][ih],
                                 &s_cnt[1][ipoly][1 - ih], (uint32_t)i + 1u, s_tw, ih, t, fail ? 1u : spin_cap, fail);
#endif
            uint32_t *pa = s_acc + ipoly * 1024 + 256 * ih;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                double re, im;
                untwist_out<false, FU>(e[r], twr[r], re, im);
                accr[r] += to_torus<SMALL, FU>(re, near);
                accr[r + 4] += to_torus<SMALL, FU>(im, near);
                pa[t + 64 * r] = accr[r];
                pa[t + 64 * r + 512] = accr[r + 4];
            }
        }
        __syncthreads();  // accumulator updated
    }
    report_wait_failure(P, fail, DEV_ERR_GATE_WAIT);
    if (FU) near_tie_flag(P, near, g, true);

    if (w != 0) return;
    if (out_mode == BR_OUT_LV1) {
        uint32_t *o = out + g * (size_t)1025;
        for (int j = t; j <= 1024; j += 64) o[j] = j == 0 ? s_acc[0] : j < 1024 ? 0u - s_acc[1024 - j] : s_acc[1024];
    } else if (out_mode == BR_OUT_LV0_EXTRACT2) {
        uint32_t *o = out + g * (size_t)(n + 1);
        for (int j = t; j <= n; j += 64) o[j] = j == 0 ? s_acc[0] : j < n ? 0u - s_acc[n - j] : s_acc[1024];
    } else {
        uint32_t *o = out + g * (size_t)2048;
        for (int j = t; j < 2048; j += 64) o[j] = s_acc[j];
    }
}

template <int T, int G>
__global__ __launch_bounds__(256) void k_key_switch_sel(KParams P, const uint32_t *__restrict__ lv1,
                                                        const uint32_t *__restrict__ ksk,
                                                        uint32_t *__restrict__ out, size_t B) {
    const size_t g0 = (size_t)blockIdx.y * G;
    const int w = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const int n1 = P.n + 1;
    const bool active = w < n1;
    const int wc = active ? w : 0;
    uint32_t res[G];
#pragma unroll
    for (int g = 0; g < G; g++) res[g] = (w == P.n && g0 + g < B) ? lv1[(g0 + g) * 1025 + 1024] : 0u;
    const uint32_t prec = 1u << (32 - (1 + 2 * T));
    const size_t rs = (size_t)P.ks_stride;
    const size_t stride_i = (size_t)T * 4 * rs;
    const uint32_t *rows0 = ksk + wc;
    for (int i0 = 0; i0 < 1024; i0 += 64) {
        // packed digits of a_{i0+lane} for every item: pkv[g] in lane l is item g's i0+l
        uint32_t pkv[G];
#pragma unroll
        for (int g = 0; g < G; g++) {
            const uint32_t a = (g0 + g < B) ? lv1[(g0 + g) * 1025 + i0 + lane] : 0u;
            pkv[g] = (a + prec) >> (32 - 2 * T);  // digit j at bits 2(T-1-j)
        }
        for (int ii = 0; ii < 64; ii++) {
            const uint32_t *rows = rows0 + (size_t)(i0 + ii) * stride_i;
            uint32_t r[T][3];
#pragma unroll
            for (int j = 0; j < T; j++)
#pragma unroll
                for (int k = 0; k < 3; k++) r[j][k] = rows[(size_t)(4 * j + k + 1) * rs];
#pragma unroll
            for (int g = 0; g < G; g++) {
                const uint32_t pk = __builtin_amdgcn_readlane(pkv[g], ii);
#pragma unroll
                for (int j = 0; j < T; j++) {
                    const uint32_t k = (pk >> (2 * (T - 1 - j))) & 3u;
                    const uint32_t v = (k & 2u) ? ((k & 1u) ? r[j][2] : r[j][1]) : ((k & 1u) ? r[j][0] : 0u);
                    res[g] -= v;
                }
            }
        }
    }
    if (active) {
#pragma unroll
        for (int g = 0; g < G; g++)
            if (g0 + g < B) out[(g0 + g) * n1 + w] = res[g];
    }
}

// Gather form (any base): per (i, j) each item loads its selected row word;
// the G*t loads of one i are independent and issued together (no branches),
// candidates are shared across the block's items through L1/L2.
template <int T, int G>
__global__ __launch_bounds__(256) void k_key_switch_gather(KParams P, const uint32_t *__restrict__ lv1,
                                                           const uint32_t *__restrict__ ksk,
                                                           uint32_t *__restrict__ out, size_t B) {
    const size_t g0 = (size_t)blockIdx.y * G;
    const int w = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const int n1 = P.n + 1;
    const bool active = w < n1;
    const int wc = active ? w : 0;
    const int basebit = P.basebit, base = 1 << basebit;
    uint32_t res[G];
#pragma unroll
    for (int g = 0; g < G; g++) res[g] = (w == P.n && g0 + g < B) ? lv1[(g0 + g) * 1025 + 1024] : 0u;
    const uint32_t prec = 1u << (32 - (1 + basebit * T));
    const size_t rs = (size_t)P.ks_stride;
    const size_t stride_i = (size_t)T * base * rs;
    const uint32_t *rows0 = ksk + wc;
    for (int i0 = 0; i0 < 1024; i0 += 64) {
        uint32_t pkv[G];
#pragma unroll
        for (int g = 0; g < G; g++) {
            const uint32_t a = (g0 + g < B) ? lv1[(g0 + g) * 1025 + i0 + lane] : 0u;
            pkv[g] = (a + prec) >> (32 - basebit * T);
        }
#pragma unroll 2
        for (int ii = 0; ii < 64; ii++) {
            const uint32_t *rows = rows0 + (size_t)(i0 + ii) * stride_i;
            uint32_t v[G][T];
#pragma unroll
            for (int g = 0; g < G; g++) {
                const uint32_t pk = __builtin_amdgcn_readlane(pkv[g], ii);
#pragma unroll
                for (int j = 0; j < T; j++) {
                    const uint32_t k = (pk >> (basebit * (T - 1 - j))) & (uint32_t)(base - 1);
                    v[g][j] = rows[(size_t)(base * j + k) * rs];
                }
            }
#pragma unroll
            for (int g = 0; g < G; g++)
#pragma unroll
                for (int j = 0; j < T; j++) res[g] -= v[g][j];
        }
    }
    if (active) {
#pragma unroll
        for (int g = 0; g < G; g++)
            if (g0 + g < B) out[(g0 + g) * n1 + w] = res[g];
    }
}

// ---------------------------------------------------------------------------
// Identity key switch as a one-hot integer GEMM on the matrix cores ("gemm"
// form, basebit 2).  out[m][w] = [w = n]·b_m − Σ_{i,j}
// KSK[i][j][k_{m,i,j}][w] (keyswitch, key.zig / tlwe identityKeySwitch) is
// C = A·K with A[m][(i,j,k)] = [k = digit j of item m's a_i] (0/1) and K the
// KSK rows, mod 2^32.  K is split into its 4 byte planes, stored as int8
// (byte − 128); per plane v_mfma_i32_32x32x32_i8 sums exactly in int32
// (|Σ| ≤ N·t·128), and out = b − Σ_b (C_b << 8b) − N·t·128·0x01010101 (every
// (i, j) selects exactly one row, k = 0 included: its zero row reads −128).
// K-order per MFMA step: one level j, 8 coefficients i0..i0+7; lane half h
// holds coefficients i0 + 4h + (e >> 2), candidate k = e & 3 in its 16 bytes
// e (A and B pair by (h, e): tools/mfma_i8_probe.hip shows any common k
// permutation is exact).  Workgroup: 8 waves (2 per SIMD), 512 items, one
// 32-word output tile; wave v takes items 64v..64v+63 as two 32-row MFMA
// tiles, 2 x 4 accumulators (128 VGPRs).  The B fragments of a coefficient
// block (t levels x 4 planes x 1 KB) and the block's input words of the 512
// items come by LDS-DMA into a 3-slot ring, two blocks ahead, one barrier per
// block; K splits over blockIdx.z write partial sums that k_ks_gemm_reduce adds.
constexpr int KG_WAVES = 8;
constexpr int KG_ITEMS = 64 * KG_WAVES;  // items per workgroup
typedef int kg_v4i __attribute__((ext_vector_type(4)));
typedef int kg_v16i __attribute__((ext_vector_type(16)));

// MFMA-layout key, built from the device KSK (k = 0 rows zeroed), in blocks
// of CB coefficients (kg_cb): kg[j][ib][wt][s][b][lane][e] int8, lane = 32h + c,
// s < KS = kg_ksteps the MFMA K-steps of one level of one block:
//   basebit 2: CB = 8, KS = 1, coefficient i = 8ib + 4h + (e >> 2), k = e & 3;
//   basebit 5: CB = 4, KS = 4, coefficient i = 4ib + s, k = 16h + e;
// byte b of KSK[i][j][k][w = 32wt + c] − 128 (w > n or i >= n_in: 0 − 128).
__host__ __device__ __forceinline__ int kg_cb(int basebit) { return basebit == 2 ? 8 : 4; }
__host__ __device__ __forceinline__ int kg_ksteps(int basebit) { return basebit == 2 ? 1 : 4; }
__host__ __device__ __forceinline__ int kg_blocks(int n_in, int basebit) { return (n_in + kg_cb(basebit) - 1) / kg_cb(basebit); }
size_t ks_gemm_bytes(const KParams &P, int n_in, int t, int basebit) {
    const size_t w32 = (size_t)(P.n + 1 + 31) / 32;
    return (size_t)t * kg_blocks(n_in, basebit) * w32 * kg_ksteps(basebit) * 4 * 1024;
}
__global__ void k_ksk_to_gemm(KParams P, const uint32_t *__restrict__ ksk, uint32_t *__restrict__ kg, size_t words,
                              int n_in, int t, int basebit) {
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // one u32 = bytes e = 4q .. 4q+3
    if (x >= words) return;
    const int w32 = (P.n + 1 + 31) / 32, nib = kg_blocks(n_in, basebit), ks = kg_ksteps(basebit);
    const int base = 1 << basebit;
    const int q = (int)(x & 3), lane = (int)((x >> 2) & 63), b = (int)((x >> 8) & 3);
    size_t r = x >> 10;
    const int st = (int)(r % ks);
    r /= ks;
    const int wt = (int)(r % w32);
    r /= w32;
    const int ib = (int)(r % nib), j = (int)(r / nib);
    const int h = lane >> 5, c = lane & 31, w = 32 * wt + c;
    const size_t rs = (size_t)P.ks_stride;
    uint32_t v = 0;
#pragma unroll
    for (int e4 = 0; e4 < 4; e4++) {
        const int e = 4 * q + e4;
        const int i = basebit == 2 ? 8 * ib + 4 * h + (e >> 2) : 4 * ib + st;
        const int k = basebit == 2 ? (e & 3) : 16 * h + e;
        const uint32_t word =
            (w <= P.n && i < n_in) ? ksk[((size_t)(base * t) * i + (size_t)base * j + k) * rs + w] : 0u;
        v |= (((word >> (8 * b)) & 255u) ^ 128u) << (8 * e4);  // byte − 128 as int8
    }
    kg[x] = v;
}

// s_waitcnt vmcnt(N) (an immediate per case)
template <int N>
DEV void kg_wait() {
    static_assert(N >= 0 && N <= 15, "kg_wait");
#define KG_W(n_) if constexpr (N == n_) asm volatile("s_waitcnt vmcnt(" #n_ ")" ::: "memory");
    KG_W(0) KG_W(1) KG_W(2) KG_W(3) KG_W(4) KG_W(5) KG_W(6) KG_W(7)
    KG_W(8) KG_W(9) KG_W(10) KG_W(11) KG_W(12) KG_W(13) KG_W(14) KG_W(15)
#undef KG_W
}

template <int T, int BASEBIT>
__global__ __launch_bounds__(64 * KG_WAVES, 1) void k_key_switch_gemm(KParams P, const uint32_t *__restrict__ lv1,
                                                                   const uint32_t *__restrict__ kg,
                                                                   uint32_t *__restrict__ part, size_t B,
                                                                   int ib_per_split, int n_in, int in_stride) {
    constexpr int CB = BASEBIT == 2 ? 8 : 4;             // coefficients per block
    constexpr int KS = BASEBIT == 2 ? 1 : 4;             // MFMA K-steps per level per block
    constexpr int STEP_BYTES = KS * 4 * 1024;            // one level's K-steps x 4 planes of one 32-word tile
    constexpr int WORDS_BYTES = CB * KG_ITEMS * 4;       // the block's CB input words of the 512 items
    constexpr int WORD_DMAS = CB / 4;                    // 16-B pieces per item per block
    constexpr int BUF_BYTES = T * STEP_BYTES + WORDS_BYTES;
    constexpr int STAGES = 3 * BUF_BYTES <= 160 * 1024 ? 3 : 2;  // blocks read, landing (, issued)
    constexpr int LOADER_DMAS = T * KS + WORD_DMAS;      // per block: waves 0-3 (KSK pieces + words) ...
    constexpr int OTHER_DMAS = WORD_DMAS;                // ... and waves 4-7 (words)
    static_assert(STAGES * BUF_BYTES <= 160 * 1024, "gemm key-switch LDS");
    __shared__ __attribute__((aligned(16))) unsigned char smem[STAGES * BUF_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int v = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool loader = v < 4;  // waves 0-3 also issue the KSK pieces: 4 KB per instruction, 256 threads x 16 B
    const int w32 = (P.n + 1 + 31) / 32;
    const int wt = blockIdx.x;
    const int nib = kg_blocks(n_in, BASEBIT);
    const int ib_lo = blockIdx.z * ib_per_split, ib_hi = min(nib, ib_lo + ib_per_split);
    const size_t m_wg = (size_t)blockIdx.y * KG_ITEMS;
    const int h = lane >> 5, c = lane & 31;
    // the block's input words: piece r of item (CB = 8) 256r + tid/2, half tid & 1, or (CB = 4) tid
    const uint32_t *a_src[WORD_DMAS];
#pragma unroll
    for (int r = 0; r < WORD_DMAS; r++) {
        const size_t m = m_wg + (CB == 8 ? 256 * r + (tid >> 1) : tid);
        a_src[r] = lv1 + (m < B ? m : B - 1) * (size_t)in_stride + (CB == 8 ? 4 * (tid & 1) : 0);
    }
    const uint32_t lds0 = (uint32_t)(size_t)(lds_void_t *)smem;
    // In flight per wave, oldest first: block ib's pieces, then block ib + 1's
    // (LOADER_DMAS or OTHER_DMAS per block), all by LDS-DMA: no VGPR holds a
    // load in flight, so the only waits are the kg_wait below.
    auto issue = [&](int ib, int slot) {
        const uint32_t base = lds0 + slot * BUF_BYTES;
        if (loader) {
#pragma unroll
            for (int j = 0; j < T; j++)
#pragma unroll
                for (int st = 0; st < KS; st++) {
                    // block (j, ib, wt) is KS x 4 KB; thread tid's 16 B of K-step st at word 1,024 st + 4 tid
                    const uint32_t *src = kg + ((((size_t)j * nib + ib) * w32 + wt) * KS + st) * 1024 + tid * 4;
                    const uint32_t dst =
                        __builtin_amdgcn_readfirstlane(base + j * STEP_BYTES + st * 4096 + (tid & ~63) * 16);
                    uint32_t keep;
                    asm volatile(
                        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                        : "=&s"(keep)
                        : "v"(src), "s"(dst)
                        : "memory");
                }
        }
        // words [item][CB], 16 B per lane.  Coefficients past n_in select zero
        // rows, so what a block's last words read there (the next row, or the
        // caller's slack past the last one: launch_ks_gemm) is unused.
#pragma unroll
        for (int r = 0; r < WORD_DMAS; r++) {
            const uint32_t dst =
                __builtin_amdgcn_readfirstlane(base + T * STEP_BYTES + r * 256 * 32 + (tid & ~63) * 16);
            uint32_t keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(a_src[r] + CB * ib), "s"(dst)
                : "memory");
        }
    };
    kg_v16i acc[2][4];
#pragma unroll
    for (int s = 0; s < 2; s++)
#pragma unroll
        for (int b = 0; b < 4; b++) acc[s][b] = kg_v16i{};
    const uint32_t prec = 1u << (32 - (1 + BASEBIT * T));
#pragma unroll
    for (int k = 0; k < STAGES - 1; k++)
        if (ib_lo + k < ib_hi) issue(ib_lo + k, k);
    for (int ib = ib_lo; ib < ib_hi; ib++) {
        const int slot = (ib - ib_lo) % STAGES;
        // blocks ib + 1 .. ib + STAGES - 2 may stay in flight
        const int ahead = min(STAGES - 2, ib_hi - 1 - ib);
        if (ahead == 1) {
            if (loader) kg_wait<LOADER_DMAS>();
            else kg_wait<OTHER_DMAS>();
        } else {
            kg_wait<0>();
        }
        __syncthreads();  // block ib landed for every wave; every wave done with block ib - 1
        if (ib + STAGES - 1 < ib_hi) issue(ib + STAGES - 1, (slot + STAGES - 1) % STAGES);  // block ib - 1's slot
        const unsigned char *buf = smem + slot * BUF_BYTES;
        const uint32_t *words = reinterpret_cast<const uint32_t *>(buf + T * STEP_BYTES);
        if constexpr (BASEBIT == 2) {
            uint32_t pk[2][4];
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const kg_v4i wv = *reinterpret_cast<const kg_v4i *>(words + (64 * v + 32 * s + c) * 8 + 4 * h);
#pragma unroll
                for (int q = 0; q < 4; q++) pk[s][q] = ((uint32_t)wv[q] + prec) >> (32 - 2 * T);
            }
#pragma unroll
            for (int j = 0; j < T; j++) {
                kg_v4i a[2];
#pragma unroll
                for (int s = 0; s < 2; s++)
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        a[s][q] = (int)(1u << (8u * ((pk[s][q] >> (2 * (T - 1 - j))) & 3u)));
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const kg_v4i bf = *reinterpret_cast<const kg_v4i *>(buf + j * STEP_BYTES + b * 1024 + lane * 16);
#pragma unroll
                    for (int s = 0; s < 2; s++)
                        acc[s][b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], bf, acc[s][b], 0, 0, 0);
                }
            }
        } else {  // basebit 5: one K-step per (coefficient, level), lane half h holds k = 16h .. 16h+15
            uint32_t pk[2][4];
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const kg_v4i wv = *reinterpret_cast<const kg_v4i *>(words + (64 * v + 32 * s + c) * 4);
#pragma unroll
                for (int q = 0; q < 4; q++) pk[s][q] = ((uint32_t)wv[q] + prec) >> (32 - BASEBIT * T);
            }
#pragma unroll
            for (int j = 0; j < T; j++)
#pragma unroll
                for (int st = 0; st < KS; st++) {
                    kg_v4i a[2];
#pragma unroll
                    for (int s = 0; s < 2; s++) {
                        const uint32_t d = (pk[s][st] >> (BASEBIT * (T - 1 - j))) & 31u;
                        const uint32_t one = 1u << (8u * (d & 3u));
                        const int word = (int)(d >> 2) - 4 * h;  // 0..3 when k = d sits in this lane half
#pragma unroll
                        for (int q = 0; q < 4; q++) a[s][q] = word == q ? (int)one : 0;
                    }
#pragma unroll
                    for (int b = 0; b < 4; b++) {
                        const kg_v4i bf = *reinterpret_cast<const kg_v4i *>(buf + j * STEP_BYTES + st * 4096 +
                                                                            b * 1024 + lane * 16);
#pragma unroll
                        for (int s = 0; s < 2; s++)
                            acc[s][b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], bf, acc[s][b], 0, 0, 0);
                    }
                }
        }
    }
    // partial sums of this K split: part[z][m][w], w < n + 1
    const int n1 = P.n + 1;
    uint32_t *pz = part + (size_t)blockIdx.z * B * n1;
    const int w = 32 * wt + c;
    const size_t m_base = m_wg + 64 * v;
#pragma unroll
    for (int s = 0; s < 2; s++)
#pragma unroll
        for (int reg = 0; reg < 16; reg++) {
            const size_t m = m_base + 32 * s + (reg & 3) + 8 * (reg >> 2) + 4 * h;
            const uint32_t val = (uint32_t)acc[s][0][reg] + ((uint32_t)acc[s][1][reg] << 8) +
                                 ((uint32_t)acc[s][2][reg] << 16) + ((uint32_t)acc[s][3][reg] << 24);
            if (m < B && w < n1) pz[m * n1 + w] = val;
        }
}

// out[m][w] = [w = n]·b_m − Σ_z part[z][m][w] − CB·blocks·t·128·0x01010101 (mod 2^32)
__global__ void k_ks_gemm_reduce(KParams P, const uint32_t *__restrict__ lv1, const uint32_t *__restrict__ part,
                                 uint32_t *__restrict__ out, size_t B, int splits, int n_in, int in_stride, int t,
                                 int basebit) {
    const int n1 = P.n + 1;
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= B * n1) return;
    const size_t m = x / n1;
    const int w = (int)(x % n1);
    uint32_t r = (uint32_t)(kg_cb(basebit) * kg_blocks(n_in, basebit) * t) * 128u * 0x01010101u;
    for (int z = 0; z < splits; z++) r += part[(size_t)z * B * n1 + x];
    out[x] = (w == P.n ? lv1[m * (size_t)in_stride + n_in] : 0u) - r;
}

// Zero the k = 0 rows of a device KSK (left undefined by the reference, key.zig:156).
__global__ void k_ksk_zero_k0(uint32_t *__restrict__ ksk, int rs, int base, size_t groups) {
    size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= groups * rs) return;
    size_t grp = idx / rs, x = idx % rs;
    ksk[grp * base * rs + x] = 0u;
}

// Lane form (any base; default): lane = item (64 items per block), block =
// one chunk of KL_CHUNK output words x all N*t digits, the 4 waves splitting
// the coefficient range i and reducing through LDS at the end.  Per i, a wave
// LDS-DMAs the chunk of all 2^basebit candidate rows of all t levels
// ([j][16-B piece][k] slots; the zero k = 0 rows come along) into a private
// double buffer, and every lane subtracts its digit's slots.  One KSK row
// chunk serves 64 items (the select form's 8), and the candidates of one (j,
// piece) sit in consecutive 16-B slots, so the lane-dependent ds_read_b128
// touch distinct banks.
constexpr int KL_CHUNK = 32;  // output words per block (8 pieces of 16 B)
constexpr int KL_WAVES = 4;
// Balanced variant for the 128-bit set at B = 1024: 44-word chunks (16 per
// 704-word padded row) x 8 waves -> exactly 256 blocks, one per CU, instead of
// 352 blocks of which 96 share a CU (launch_ks_lanes picks per batch).
constexpr int KL_CHUNK_WIDE = 44;
constexpr int KL_WAVES_WIDE = 8;

template <int T, int BASEBIT, int CHUNK = KL_CHUNK, int WAVES = KL_WAVES, int GW = 1>
// n_in / in_stride: input dimension and words per input ciphertext — N and
// N+1 for the identity key switch (TLWELv1 in), n and n+1 for the proxy
// re-encryption of proxy_reenc.zig:267-306 (TLWELv0 in, same algorithm).
// GW: waves that take different 64-item groups (64*GW items per block) and
// walk the same coefficients in the same order, so their DMAs of one KSK
// chunk meet in L2; the other WAVES/GW split the coefficient range.  GW > 1
// cuts KSK reads from HBM when the key does not stay cached (UINT4: 323 MB).
__global__ __launch_bounds__(64 * WAVES) void k_key_switch_lanes(KParams P, const uint32_t *__restrict__ lv1,
                                                          const uint32_t *__restrict__ ksk,
                                                          uint32_t *__restrict__ out, size_t B, int n_in,
                                                          int in_stride) {
    constexpr int BASE = 1 << BASEBIT;
    constexpr int PIECES = CHUNK / 4;
    constexpr int SLOTS = T * PIECES * BASE;    // 16-B slots per coefficient i
    constexpr int NDMA = (SLOTS + 63) / 64;     // LDS-DMA instructions per i
    constexpr int BUF = NDMA * 64 + 16;         // 16-B slots per buffer: KSK slots + 64 digits words
    constexpr int RING = 2 * BUF;               // double buffer
    constexpr int RED = WAVES * CHUNK * 64;     // reduction words
    constexpr int LDS_BYTES = (RING * 16 * WAVES > RED * 4) ? RING * 16 * WAVES : RED * 4;
    static_assert(LDS_BYTES <= 160 * 1024, "key-switch LDS");
    __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int IW = WAVES / GW;  // waves splitting the coefficient range
    static_assert(WAVES % GW == 0, "GW divides WAVES");
    const int gw = w % GW, iw = w / GW;
    uint4 *ring = reinterpret_cast<uint4 *>(smem) + w * RING;
    const size_t g_raw = (size_t)blockIdx.y * (64 * GW) + gw * 64 + lane;
    const bool valid = g_raw < B;
    const size_t g = valid ? g_raw : B - 1;
    const int w0 = blockIdx.x * CHUNK;
    const size_t rs = (size_t)P.ks_stride;
    const size_t step_i = (size_t)BASE * T * rs;  // words between consecutive i
    const int per = (n_in + IW - 1) / IW;
    const int ilo = min(n_in, iw * per), ihi = min(n_in, ilo + per);
    // this lane's DMA sources relative to row (i, 0, 0): slot s = c*64 + lane
    uint32_t src_off[NDMA];
#pragma unroll
    for (int c = 0; c < NDMA; c++) {
        const int sl = min(c * 64 + lane, SLOTS - 1);  // padding slots re-load the last one
        const int k = sl % BASE, piece = (sl / BASE) % PIECES, j = sl / (BASE * PIECES);
        src_off[c] = (uint32_t)((BASE * j + k) * rs + w0 + 4 * piece);
    }
    // Per i, one buffer receives the KSK slots and, by a 4-byte LDS-DMA, a_i
    // of the 64 items (lane g's word).  The DMAs are inline asm
    // (cdna_hip_programming.md §5.7): as builtins hipcc would guard every
    // ds_read of one buffer with vmcnt(0) against the fill of the other, so
    // their completion is counted by hand (vmcnt(0) at the top of step i, when
    // only buffer i's fill is in flight).
    const uint32_t ring_lds = (uint32_t)(size_t)(lds_void_t *)ring;
    const uint32_t *a_src = lv1 + g * (size_t)in_stride;
    auto issue = [&](int i, int which) {
        const uint32_t *r = ksk + (size_t)i * step_i;
#pragma unroll
        for (int c = 0; c < NDMA; c++) {
            const uint32_t dst = __builtin_amdgcn_readfirstlane(ring_lds + (which * BUF + c * 64) * 16);
            uint32_t keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(r + src_off[c]), "s"(dst)
                : "memory");
        }
        const uint32_t dst = __builtin_amdgcn_readfirstlane(ring_lds + (which * BUF + NDMA * 64) * 16);
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(a_src + i), "s"(dst)
            : "memory");
    };
    const uint32_t prec = 1u << (32 - (1 + BASEBIT * T));
    uint32_t acc[CHUNK];
#pragma unroll
    for (int x = 0; x < CHUNK; x++) acc[x] = 0u;
    if (ilo < ihi) issue(ilo, 0);
    for (int i = ilo; i < ihi; i++) {
        const int cur = (i - ilo) & 1;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // buffer i landed
        wave_sync();
        if (i + 1 < ihi) issue(i + 1, cur ^ 1);
        const uint4 *buf = ring + cur * BUF;
        const uint32_t a = reinterpret_cast<const uint32_t *>(buf + NDMA * 64)[lane];
        const uint32_t pk = (a + prec) >> (32 - BASEBIT * T);  // digit j at bits BASEBIT*(T-1-j)
#pragma unroll
        for (int j = 0; j < T; j++) {
            const uint32_t k = (pk >> (BASEBIT * (T - 1 - j))) & (uint32_t)(BASE - 1);
            const uint4 *sl = buf + j * PIECES * BASE + k;
#pragma unroll
            for (int pc = 0; pc < PIECES; pc++) {
                const uint4 v = sl[pc * BASE];
                acc[4 * pc + 0] -= v.x;
                acc[4 * pc + 1] -= v.y;
                acc[4 * pc + 2] -= v.z;
                acc[4 * pc + 3] -= v.w;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this buffer's reads done before its re-fill
    }
    __syncthreads();  // every wave done with its ring: reuse LDS for the reduction
    uint32_t *red = reinterpret_cast<uint32_t *>(smem);
#pragma unroll
    for (int x = 0; x < CHUNK; x++) red[(w * CHUNK + x) * 64 + lane] = acc[x];
    __syncthreads();
    const int n1 = P.n + 1;
    for (int x = iw; x < CHUNK; x += IW) {  // wave (gw, iw) reduces words iw, iw + IW, ... of group gw
        uint32_t r = 0u;
#pragma unroll
        for (int v = 0; v < IW; v++) r += red[((v * GW + gw) * CHUNK + x) * 64 + lane];
        const int word = w0 + x;
        if (valid && word < n1) out[g * n1 + word] = (word == P.n ? a_src[n_in] : 0u) + r;  // r = -(sum of rows)
    }
}

// Ring form for keys that stream from HBM (UINT4: 323 MB, beyond the MALL).
// The lane form's per-wave double buffer leaves one coefficient of DMA in
// flight, and at basebit 5 a coefficient's subtractions (~150 instructions)
// take far less than an HBM round trip: 2.65 ms per 4,096 items, latency
// bound.  Here the GW waves of a block (one 64-item group each) share ONE ring
// of DEPTH buffers, since they read the same chunk of the same coefficient:
// each wave DMAs 1/GW of a buffer's KSK slots plus its own items' a_i, and a
// block barrier per coefficient publishes buffer i (every wave waited for its
// own pieces) and retires buffer i - 1, which is refilled DEPTH - 1 ahead.
// A quarter of the LDS per block lets 3 blocks share a CU, and DEPTH - 1
// coefficients are in flight per block.  Same subtractions in the same order.
#ifndef KS_RING_DEPTH
#define KS_RING_DEPTH 4
#endif
template <int N>
DEV void wait_vmcnt_le() {  // s_waitcnt vmcnt(N), expcnt / lgkmcnt untouched
    static_assert(N >= 0 && N < 64, "vmcnt field");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
template <int T, int BASEBIT, int CHUNK, int GW, int DEPTH>
__global__ __launch_bounds__(64 * GW) void k_key_switch_ring(KParams P, const uint32_t *__restrict__ lv1,
                                                           const uint32_t *__restrict__ ksk,
                                                           uint32_t *__restrict__ out, size_t B, int n_in,
                                                           int in_stride) {
    constexpr int BASE = 1 << BASEBIT;
    constexpr int PIECES = CHUNK / 4;
    constexpr int SLOTS = T * PIECES * BASE;  // 16-B KSK slots per coefficient
    static_assert(SLOTS % 64 == 0, "whole DMA instructions");
    constexpr int NDMA = SLOTS / 64;             // LDS-DMA instructions per buffer, all waves
    constexpr int MINE = (NDMA + GW - 1) / GW;   // per wave (+ 1 for its a_i words); when GW does not
                                                 // divide NDMA, some waves repeat another's piece
                                                 // (the same bytes into the same slot)
    constexpr int BUF = SLOTS + GW * 16;      // 16-B slots per buffer: KSK slots, then GW x 64 a_i words
    static_assert(DEPTH >= 3 && (MINE + 1) * (DEPTH - 2) < 64, "ring depth");
    __shared__ __attribute__((aligned(16))) uint4 ring[DEPTH * BUF];
    const int lane = threadIdx.x & 63;
    const int gw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const size_t g_raw = (size_t)blockIdx.y * (64 * GW) + gw * 64 + lane;
    const bool valid = g_raw < B;
    const size_t g = valid ? g_raw : B - 1;
    const int w0 = blockIdx.x * CHUNK;
    const size_t rs = (size_t)P.ks_stride;
    const size_t step_i = (size_t)BASE * T * rs;
    uint32_t src_off[MINE];
#pragma unroll
    for (int cc = 0; cc < MINE; cc++) {
        const int sl = ((cc * GW + gw) % NDMA) * 64 + lane;
        const int k = sl % BASE, piece = (sl / BASE) % PIECES, j = sl / (BASE * PIECES);
        src_off[cc] = (uint32_t)((BASE * j + k) * rs + w0 + 4 * piece);
    }
    const uint32_t ring_lds = (uint32_t)(size_t)(lds_void_t *)ring;
    const uint32_t *a_src = lv1 + g * (size_t)in_stride;
    auto issue = [&](int i, int slot) {
        const uint32_t *r = ksk + (size_t)i * step_i;
#pragma unroll
        for (int cc = 0; cc < MINE; cc++) {
            const uint32_t dst = __builtin_amdgcn_readfirstlane(ring_lds + (slot * BUF + ((cc * GW + gw) % NDMA) * 64) * 16);
            uint32_t keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(r + src_off[cc]), "s"(dst)
                : "memory");
        }
        const uint32_t dst = __builtin_amdgcn_readfirstlane(ring_lds + (slot * BUF + SLOTS + gw * 16) * 16);
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(a_src + i), "s"(dst)
            : "memory");
    };
    const uint32_t prec = 1u << (32 - (1 + BASEBIT * T));
    uint32_t acc[CHUNK];
#pragma unroll
    for (int x = 0; x < CHUNK; x++) acc[x] = 0u;
    for (int i = 0; i < DEPTH - 1 && i < n_in; i++) issue(i, i);
    for (int i = 0; i < n_in; i++) {
        // this wave's pieces of buffer i landed: only buffers i+1 .. i+DEPTH-2 may still be in flight
        if (i + DEPTH - 2 < n_in) wait_vmcnt_le<(MINE + 1) * (DEPTH - 2)>();
        else wait_vmcnt_le<0>();
        // every wave's pieces of buffer i landed, and every wave is done reading buffer i - 1
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (i + DEPTH - 1 < n_in) issue(i + DEPTH - 1, (i + DEPTH - 1) % DEPTH);
        const uint4 *buf = ring + (i % DEPTH) * BUF;
        const uint32_t a = reinterpret_cast<const uint32_t *>(buf + SLOTS + gw * 16)[lane];
        const uint32_t pk = (a + prec) >> (32 - BASEBIT * T);  // digit j at bits BASEBIT*(T-1-j)
#pragma unroll
        for (int j = 0; j < T; j++) {
            const uint32_t k = (pk >> (BASEBIT * (T - 1 - j))) & (uint32_t)(BASE - 1);
            const uint4 *sl = buf + j * PIECES * BASE + k;
#pragma unroll
            for (int pc = 0; pc < PIECES; pc++) {
                const uint4 v = sl[pc * BASE];
                acc[4 * pc + 0] -= v.x;
                acc[4 * pc + 1] -= v.y;
                acc[4 * pc + 2] -= v.z;
                acc[4 * pc + 3] -= v.w;
            }
        }
    }
    const int n1 = P.n + 1;
    if (!valid) return;
#pragma unroll
    for (int x = 0; x < CHUNK; x++) {
        const int word = w0 + x;
        if (word < n1) out[g * n1 + word] = (word == P.n ? a_src[n_in] : 0u) + acc[x];  // acc = -(sum of rows)
    }
}

// ---------------------------------------------------------------------------
// Stage kernels (parity tests and key generation); same device FFT.
// ---------------------------------------------------------------------------
// ifft1024: u32 -> f64 [re(512) | im(512)], ×2 (fft.zig:293-366)
__global__ __launch_bounds__(64) void k_fft_forward(DevTables TT, const uint32_t *__restrict__ in,
                                                    double *__restrict__ out) {
    __shared__ C2 s_x[512];
    const int t = threadIdx.x;
    const uint32_t *x = in + (size_t)blockIdx.x * 1024;
    RegTw T;
    T.init(TT.tw, t);
    C2 d[1][8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
        int k = t + 64 * br3(q);
        d[0][q] = twist_in((double)(int32_t)x[k], (double)(int32_t)x[k + 512], TT.twist[k]);
    }
    fft512<1, false>(d, s_x, T, t);
    double *o = out + (size_t)blockIdx.x * 1024;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        o[t + 64 * q] = d[0][q].x * 2.0;
        o[512 + t + 64 * q] = d[0][q].y * 2.0;
    }
}

// fft1024: f64 -> u32 (fft.zig:370-443).  Input ×0.5 folded into 1/1024.
__global__ __launch_bounds__(64) void k_fft_inverse(DevTables TT, const double *__restrict__ in,
                                                    uint32_t *__restrict__ out) {
    __shared__ C2 s_x[512];
    const int t = threadIdx.x;
    const double *f = in + (size_t)blockIdx.x * 1024;
    RegTw T;
    T.init(TT.tw, t);
    C2 d[1][8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
        int k = t + 64 * br3(q);
        d[0][q] = c2(f[k], f[k + 512]);
    }
    fft512<1, true>(d, s_x, T, t);
    uint32_t *o = out + (size_t)blockIdx.x * 1024;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        double tr, ti;
        untwist_out(d[0][q], TT.twist[t + 64 * q], tr, ti);
        o[t + 64 * q] = torus_from_f64(tr);
        o[512 + t + 64 * q] = torus_from_f64(ti);
    }
}

// poly_mul (fft.zig:458-492): ifft(a), ifft(b), (ar*br - ai*bi)*0.5, fft.
// With the ×2 of both ifft outputs and the ×0.5s folded: P = A*B computed on
// the unscaled transforms equals ref/2 exactly; fft's ×0.5 then cancels it.
__global__ __launch_bounds__(64) void k_poly_mul(DevTables TT, const uint32_t *__restrict__ a,
                                                 const uint32_t *__restrict__ b, size_t b_stride,
                                                 uint32_t *__restrict__ out) {
    __shared__ C2 s_x[2 * 512];
    const int t = threadIdx.x;
    const uint32_t *x = a + (size_t)blockIdx.x * 1024;
    const uint32_t *y = b + (size_t)blockIdx.x * b_stride;
    RegTw T;
    T.init(TT.tw, t);
    C2 twl[8];
#pragma unroll
    for (int m = 0; m < 8; m++) twl[m] = TT.twist[t + 64 * m];
    C2 d[2][8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
        int m = br3(q), k = t + 64 * m;
        d[0][q] = twist_in((double)(int32_t)x[k], (double)(int32_t)x[k + 512], twl[m]);
        d[1][q] = twist_in((double)(int32_t)y[k], (double)(int32_t)y[k + 512], twl[m]);
    }
    fft512<2, false>(d, s_x, T, t);
    // reference: r = (2A_r*2B_r - 2A_i*2B_i)*0.5 = 2*(A_r*B_r - A_i*B_i) exactly;
    // fft then multiplies by 0.5, so the inverse input is P below, unscaled,
    // and the final normalisation is 1/512 (not 1/1024).
    C2 e[1][8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
        C2 p = c2(d[0][q].x * d[1][q].x - d[0][q].y * d[1][q].y,
                  d[0][q].x * d[1][q].y + d[0][q].y * d[1][q].x);
        e[0][br3(q)] = p;
    }
    fft512<1, true>(e, s_x, T, t);
    uint32_t *o = out + (size_t)blockIdx.x * 1024;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        C2 f = e[0][q], w = twl[q];
        const double norm = 1.0 / 512.0;
        double tr = (f.x * w.x + f.y * w.y) * norm;
        double ti = (f.y * w.x - f.x * w.y) * norm;
        o[t + 64 * q] = torus_from_f64(tr);
        o[512 + t + 64 * q] = torus_from_f64(ti);
    }
}

// externalProductWithFft (trgsw.zig:111-154) of B TRLWEs against one
// device-layout TRGSW row.
template <int L>
__global__ __launch_bounds__(64) void k_external_product(KParams P, DevTables TT,
                                                         const double2 *__restrict__ bkrow,
                                                         const uint32_t *__restrict__ in,
                                                         uint32_t *__restrict__ out) {
    __shared__ C2 s_x[2 * 512];
    const int t = threadIdx.x;
    const uint32_t *x = in + (size_t)blockIdx.x * 2048;
    RegTw T;
    T.init(TT.tw, t);
    C2 twl[8];
#pragma unroll
    for (int m = 0; m < 8; m++) twl[m] = TT.twist[t + 64 * m];
    uint32_t tA[16], tB[16], accA[16], accB[16];
#pragma unroll
    for (int m = 0; m < 16; m++) {
        tA[m] = x[t + 64 * m] + P.offset;
        tB[m] = x[1024 + t + 64 * m] + P.offset;
        accA[m] = 0;
        accB[m] = 0;
    }
    C2 fa[8], fb[8];
    ext_pairs_global<L>(tA, tB, bkrow, P.bgbit, T, twl, s_x, t, fa, fb);
    uint32_t near = NEAR_NONE;
    inverse_and_add<false, 1>(fa, fb, s_x, T, twl, t, accA, accB, near);
    uint32_t *o = out + (size_t)blockIdx.x * 2048;
#pragma unroll
    for (int m = 0; m < 16; m++) {
        o[t + 64 * m] = accA[m];
        o[1024 + t + 64 * m] = accB[m];
    }
}

// BK layout permutation: reference [rows][a|b][1024] (each re[512] ++ im[512])
// <-> device [rows][q][a|b][64] double2 (re, im) at frequency t + 64q.
__global__ void k_bk_permute(const double *__restrict__ ref, double2 *__restrict__ dev, size_t rows,
                             int dir) {
    size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= rows * 512) return;
    size_t row = idx / 512;
    int pos = (int)(idx % 512);
    int q = pos >> 6, t = pos & 63;  // pos = t + 64q
    const size_t rb = row * 2048;
    double2 *da = dev + row * 1024 + (size_t)(2 * q) * 64 + t;
    double2 *db = da + 64;
    // device copy scaled by 2^-10 (exact): the untwist's 1/1024 moves into
    // the key (untwist_out<false>)
    const double down = 1.0 / 1024.0, up = 1024.0;
    if (dir == 0) {
        *da = make_double2(ref[rb + pos] * down, ref[rb + 512 + pos] * down);
        *db = make_double2(ref[rb + 1024 + pos] * down, ref[rb + 1536 + pos] * down);
    } else {
        double *r = const_cast<double *>(ref);
        double2 a = *da, b = *db;
        r[rb + pos] = a.x * up;
        r[rb + 512 + pos] = a.y * up;
        r[rb + 1024 + pos] = b.x * up;
        r[rb + 1536 + pos] = b.y * up;
    }
}

// Ciphertext gather dst[k] = (NEG ? -1 : 1) * src[idx[k]]: TLWELv0.neg
// (tlwe.zig:120-239, gates.zig:132-135 notGate) is the circuit evaluator's
// free NOT; the plain form collects its outputs.  One block per ciphertext.
template <bool NEG>
__global__ __launch_bounds__(256) void k_tlwe_gather(const uint32_t *__restrict__ src,
                                                     const uint32_t *__restrict__ idx, uint32_t *__restrict__ dst,
                                                     int n1) {
    const uint32_t *x = src + (size_t)idx[blockIdx.x] * n1;
    uint32_t *y = dst + (size_t)blockIdx.x * n1;
    for (int j = threadIdx.x; j < n1; j += 256) y[j] = NEG ? 0u - x[j] : x[j];
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
hipError_t launch_tlwe_gather(const KParams &P, const uint32_t *src, const uint32_t *idx, uint32_t *dst,
                              size_t count, bool negate, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (negate)
        hipLaunchKernelGGL(k_tlwe_gather<true>, dim3((unsigned)count), dim3(256), 0, s, src, idx, dst, P.n + 1);
    else
        hipLaunchKernelGGL(k_tlwe_gather<false>, dim3((unsigned)count), dim3(256), 0, s, src, idx, dst, P.n + 1);
    return hipGetLastError();
}

// The pair form: fused (exact-integer regime) for any L, the reference's trees
// only for L = 1 (where its regrouped sum is the reference's order).

// |external product| <= 2L * N * Bg/2 * 2^31 below 2^49: the SMALL conversions
// and the fused arithmetic's guarded conversion hold (the L=3 / Bg=2^6 sets:
// 2^48.6; UINT4: 2^63, never)
static bool small_products(const KParams &P) {
    return std::ldexp(2.0 * P.L * 1024.0, P.bgbit - 1 + 31) < std::ldexp(1.0, 49);
}

// The default whole-form kernel lives in its own unit (launch_whole_default,
// tfhe_kernels_whole.hip); single-file builds of this source (tools/phase_prof.hip,
// tools/fft_bench.hip) define TFHE_SINGLE_TU and launch it here.
#ifdef TFHE_SINGLE_TU
#define WHOLE_DEFAULT_LAUNCH(L_, S_)                                                                              \
    hipLaunchKernelGGL((k_blind_rotate<L_, S_, true, S_, true>), grid, block, 0, s, P, T, ops, in_a, in_b, idx,   \
                       testvec, bk2, out, out_mode, B)
#else
#define WHOLE_DEFAULT_LAUNCH(L_, S_)                                                                              \
    do {  /* fused implies SMALL: the kernel is never instantiated in this unit */                              \
        if (!(S_)) return hipErrorInvalidValue;                                                                   \
        const hipError_t e_ = launch_whole_default(L_, grid, block, s, P, T, ops, in_a, in_b, idx, testvec, bk2,  \
                                                   out, out_mode, B);                                             \
        if (e_ != hipSuccess) return e_;                                                                          \
    } while (0)
#endif
static hipError_t launch_blind_rotate_form(const KParams &P, const DevTables &T, const uint8_t *ops,
                               const uint32_t *in_a, const uint32_t *in_b, const uint32_t *idx,
                               const uint32_t *testvec, const double *bkd, uint32_t *out, int out_mode, size_t B,
                               hipStream_t s, char form, const LaunchOpts &O, const char **used) {
    if (B == 0) return hipSuccess;
    const double2 *bk2 = reinterpret_cast<const double2 *>(bkd);
    const bool small = small_products(P);
    // form: 'W' latency (8 waves per item),
    // 'w' whole (1 wave per item; loader waves unless LaunchOpts::br_loader = 0)
    const bool wide = form == 'W';
    const bool loader = !wide && O.br_loader != 0;
    // fused arithmetic in the exact-integer regime (SMALL) unless the
    // reference expression trees are requested (TFHE_OPT_ARITH)
    const bool fused = small && fused_allowed(O);
    if (form == 'o') {  // octo form: 8 items per workgroup, two gate waves per SIMD
        const dim3 grid((unsigned)((B + BO_GATES - 1) / BO_GATES)), block(64 * BO_GATES);
#define BO_LAUNCH(L_, S_)                                                                                            \
        do {                                                                                                         \
            if (fused) {                                                                                             \
                hipLaunchKernelGGL((k_blind_rotate_octo<L_, S_, S_>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, \
                                   testvec, bk2, out, out_mode, B);                                                  \
                if (used) *used = "k_blind_rotate_octo<" #L_ "," #S_ ",true> (octo form, fused)";                    \
            } else {                                                                                                 \
                hipLaunchKernelGGL((k_blind_rotate_octo<L_, S_, false>), grid, block, 0, s, P, T, ops, in_a, in_b,   \
                                   idx, testvec, bk2, out, out_mode, B);                                             \
                if (used) *used = "k_blind_rotate_octo<" #L_ "," #S_ ",false> (octo form)";                          \
            }                                                                                                        \
        } while (0)
        switch (P.L) {
        case 1: if (small) BO_LAUNCH(1, true); else BO_LAUNCH(1, false); break;
        case 2: if (small) BO_LAUNCH(2, true); else BO_LAUNCH(2, false); break;
        case 3: if (small) BO_LAUNCH(3, true); else BO_LAUNCH(3, false); break;
        default: return hipErrorInvalidValue;
        }
#undef BO_LAUNCH
        return hipGetLastError();
    }
    if (form == 'd') {  // duo form (2 computing waves per item); falls back to the whole form where not exact
        const dim3 grid((unsigned)((B + BD_GATES - 1) / BD_GATES)), block(64 * BD_WAVES);
        bool ok = true;
        if (P.L == 3 && small && fused) {
            hipLaunchKernelGGL((k_blind_rotate_duo<3, true, true>), grid, block, 0, s, P, T, ops, in_a, in_b, idx,
                               testvec, bk2, out, out_mode, B);
            if (used) *used = "k_blind_rotate_duo<3,true,true> (duo form, fused)";
        } else if (P.L == 1 && small && fused) {
            hipLaunchKernelGGL((k_blind_rotate_duo<1, true, true>), grid, block, 0, s, P, T, ops, in_a, in_b, idx,
                               testvec, bk2, out, out_mode, B);
            if (used) *used = "k_blind_rotate_duo<1,true,true> (duo form, fused)";
        } else if (P.L == 1 && !small) {
            hipLaunchKernelGGL((k_blind_rotate_duo<1, false, false>), grid, block, 0, s, P, T, ops, in_a, in_b, idx,
                               testvec, bk2, out, out_mode, B);
            if (used) *used = "k_blind_rotate_duo<1,false,false> (duo form)";
        } else {
            ok = false;
        }
        if (ok) return hipGetLastError();
        form = 'w';
    }
    dim3 grid, block;
    if (wide) {
        grid = dim3((unsigned)B);
        block = dim3(64 * BW_WAVES);
    } else {
        grid = dim3((unsigned)((B + BR_WAVES - 1) / BR_WAVES));
        block = dim3(64 * BR_WAVES * (loader ? 2 : 1));
    }
#define BR_LAUNCH(L_, S_)                                                                                         \
    do {                                                                                                          \
        if (wide && L_ == 3 && O.br_form == 7) {  /* split transforms (k_blind_rotate_wide2), forced only */     \
            if (fused) {                                                                                          \
                hipLaunchKernelGGL((k_blind_rotate_wide2<3, S_, S_>), grid, block, 0, s, P, T, ops, in_a, in_b,   \
                                   idx, testvec, bk2, out, out_mode, B);                                          \
                if (used) *used = "k_blind_rotate_wide2<3," #S_ ",true> (latency form, split transforms, fused)"; \
            } else {                                                                                              \
                hipLaunchKernelGGL((k_blind_rotate_wide2<3, S_, false>), grid, block, 0, s, P, T, ops, in_a,      \
                                   in_b, idx, testvec, bk2, out, out_mode, B);                                    \
                if (used) *used = "k_blind_rotate_wide2<3," #S_ ",false> (latency form, split transforms)";      \
            }                                                                                                     \
        } else if (wide && fused) {                                                                               \
            hipLaunchKernelGGL((k_blind_rotate_wide<L_, S_, S_>), grid, block, 0, s, P, T, ops, in_a, in_b, idx,  \
                               testvec, bk2, out, out_mode, B);                                                   \
            if (used) *used = "k_blind_rotate_wide<" #L_ "," #S_ ",true> (latency form, fused)";                  \
        } else if (wide) {                                                                                        \
            hipLaunchKernelGGL((k_blind_rotate_wide<L_, S_, false>), grid, block, 0, s, P, T, ops, in_a, in_b,    \
                               idx, testvec, bk2, out, out_mode, B);                                              \
            if (used) *used = "k_blind_rotate_wide<" #L_ "," #S_ ",false> (latency form)";                        \
        } else if (loader && fused && O.br_flags) {                                                               \
            WHOLE_DEFAULT_LAUNCH(L_, S_);                                                                         \
            if (used) *used = "k_blind_rotate<" #L_ "," #S_ ",true,true,true> (whole form, loader waves, slot counters, fused)"; \
        } else if (loader && O.br_flags) {                                                                        \
            hipLaunchKernelGGL((k_blind_rotate<L_, S_, true, false, true>), grid, block, 0, s, P, T, ops, in_a,   \
                               in_b, idx, testvec, bk2, out, out_mode, B);                                        \
            if (used) *used = "k_blind_rotate<" #L_ "," #S_ ",true,false,true> (whole form, loader waves, slot counters)"; \
        } else if (loader && fused) {                                                                             \
            hipLaunchKernelGGL((k_blind_rotate<L_, S_, true, S_>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, \
                               testvec, bk2, out, out_mode, B);                                                   \
            if (used) *used = "k_blind_rotate<" #L_ "," #S_ ",true,true> (whole form, loader waves, fused)";      \
        } else if (loader) {                                                                                      \
            hipLaunchKernelGGL((k_blind_rotate<L_, S_, true, false>), grid, block, 0, s, P, T, ops, in_a, in_b,   \
                               idx, testvec, bk2, out, out_mode, B);                                              \
            if (used) *used = "k_blind_rotate<" #L_ "," #S_ ",true,false> (whole form, loader waves)";            \
        } else if (fused) {                                                                                       \
            hipLaunchKernelGGL((k_blind_rotate<L_, S_, false, S_>), grid, block, 0, s, P, T, ops, in_a, in_b,     \
                               idx, testvec, bk2, out, out_mode, B);                                              \
            if (used) *used = "k_blind_rotate<" #L_ "," #S_ ",false,true> (whole form, fused)";                   \
        } else {                                                                                                  \
            hipLaunchKernelGGL((k_blind_rotate<L_, S_, false, false>), grid, block, 0, s, P, T, ops, in_a, in_b,  \
                               idx, testvec, bk2, out, out_mode, B);                                              \
            if (used) *used = "k_blind_rotate<" #L_ "," #S_ ",false,false> (whole form)";                         \
        }                                                                                                         \
    } while (0)
    switch (P.L) {
    case 1: if (small) BR_LAUNCH(1, true); else BR_LAUNCH(1, false); break;
    case 2: if (small) BR_LAUNCH(2, true); else BR_LAUNCH(2, false); break;
    case 3: if (small) BR_LAUNCH(3, true); else BR_LAUNCH(3, false); break;
    default: return hipErrorInvalidValue;
    }
#undef BR_LAUNCH
    return hipGetLastError();
}

// Modelled blind-rotation time on a device with `cus` CUs, in whole-form
// rounds (BR_WAVES x cus items), of the launch plans launch_blind_rotate picks
// from; the cheapest wins (ties: the earlier plan).  LaunchOpts::br_form
// (TFHE_OPT_BR_FORM) instead forces one form for the whole batch (A/B runs, tests).
//  - latency form for the whole batch (at most BR_WIDE_MAX_ITEMS): per item per
//    CU 0.43 of a round at L = 3 (4.1 ms for up to 256 items, 8.1 ms for 512, a
//    round 9.6 ms), BR_WIDE_COST_L1 at L = 1 (a round 6.05 ms);
//  - whole form for the whole batch, ceil(B / round) rounds;
//  - whole form for the full rounds and the latency form for a ragged tail of at
//    most BR_TAIL_WIDE_MAX items (a circuit level of 10,256 gates: 99 vs 106 ms);
//  - L = 1: the octo form for the whole batch, BO_ROUND_COST_L1 per octo round
//    (8 x cus items).  One octo round costs 1.9 whole-form rounds (2,048 items:
//    11.50 vs 12.09 ms, 4,096: 22.6 vs 23.9, 8,192: 44.9 vs 47.3).  At L = 3 the
//    octo form is 4-5 % slower than the whole form.  Octo rounds
//    followed by a tail launch measured 2 ms worse than modelled (2,348 items:
//    19.5 ms against 17.6 for three whole-form rounds), so that split is no plan
//    (profiles/r03g_octo_dispatch.txt).
constexpr size_t BR_TAIL_WIDE_MAX = BR_WIDE_MAX_ITEMS;
constexpr double BO_ROUND_COST_L1 = 1.9;
constexpr double BR_WIDE_COST_L1 = 0.66;

size_t device_cus() {
    static int cus = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return 256;
        return v > 0 ? v : 256;
    }();
    return (size_t)cus;
}

enum BrPlan { PLAN_NONE, PLAN_WIDE, PLAN_WHOLE, PLAN_WHOLE_TAIL, PLAN_OCTO };

static BrPlan blind_rotate_plan(size_t B, size_t cus, int L, double *cost_out) {
    if (B == 0) {
        if (cost_out) *cost_out = 0.0;
        return PLAN_NONE;
    }
    const size_t round = BR_WAVES * cus, tail = B % round;
    const double kw = L == 1 ? BR_WIDE_COST_L1 : 0.43;
    auto wide = [&](size_t b) { return kw * (double)((b + cus - 1) / cus); };
    BrPlan best = PLAN_WHOLE;
    double c = (double)((B + round - 1) / round);
    auto consider = [&](BrPlan p, double v) {
        if (v < c) best = p, c = v;
    };
    if (B <= BR_WIDE_MAX_ITEMS && wide(B) <= c) best = PLAN_WIDE, c = wide(B);
    if (tail != 0 && tail <= BR_TAIL_WIDE_MAX && B >= round) consider(PLAN_WHOLE_TAIL, (double)(B / round) + wide(tail));
    if (L == 1) {
        const size_t octo_round = (size_t)BO_GATES * cus;
        consider(PLAN_OCTO, BO_ROUND_COST_L1 * (double)((B + octo_round - 1) / octo_round));
    }
    if (cost_out) *cost_out = c;
    return best;
}

double blind_rotate_cost(size_t B, size_t cus, int L) {
    double c = 0.0;
    blind_rotate_plan(B, cus, L, &c);
    return c;
}

// Items [start, start + count) of a batch through one form: their ops / idx
// entries / inputs / outputs / near-tie flags.
static hipError_t launch_blind_rotate_range(const KParams &P, const DevTables &T, const uint8_t *ops,
                                            const uint32_t *in_a, const uint32_t *in_b, const uint32_t *idx,
                                            const uint32_t *testvec, const double *bkd, uint32_t *out, int out_mode,
                                            size_t start, size_t count, hipStream_t s, char form, const LaunchOpts &O,
                                            const char **used) {
    const size_t in_words = (size_t)P.n + 1;
    const size_t out_words = out_mode == BR_OUT_LV1 ? (size_t)P.N + 1 : out_mode == BR_OUT_TRLWE ? 2 * (size_t)P.N : in_words;
    KParams Q = P;
    if (Q.tie_flags) Q.tie_flags += start;
    return launch_blind_rotate_form(Q, T, ops ? ops + start : nullptr, idx ? in_a : in_a + start * in_words,
                                    idx ? in_b : (in_b ? in_b + start * in_words : nullptr),
                                    idx ? idx + 2 * start : nullptr, testvec, bkd, out + start * out_words, out_mode,
                                    count, s, form, O, used);
}

static hipError_t launch_blind_rotate_forms(const KParams &P, const DevTables &T, const uint8_t *ops,
                                            const uint32_t *in_a, const uint32_t *in_b, const uint32_t *idx,
                                            const uint32_t *testvec, const double *bkd, uint32_t *out, int out_mode,
                                            size_t B, hipStream_t s, const LaunchOpts &O, const char **used) {
    if (O.br_form) {  // forced form (TFHE_OPT_BR_FORM): the whole batch in one launch
        const char f = O.br_form == 3 || O.br_form == 7 ? 'W' : O.br_form == 5 ? 'o' : O.br_form == 6 ? 'd' : 'w';
        return launch_blind_rotate_form(P, T, ops, in_a, in_b, idx, testvec, bkd, out, out_mode, B, s, f, O, used);
    }
    const size_t round = BR_WAVES * device_cus(), tail = B % round;
    switch (blind_rotate_plan(B, device_cus(), P.L, nullptr)) {
    case PLAN_NONE: return hipSuccess;
    case PLAN_WIDE:
        return launch_blind_rotate_form(P, T, ops, in_a, in_b, idx, testvec, bkd, out, out_mode, B, s, 'W', O, used);
    case PLAN_OCTO:
        return launch_blind_rotate_form(P, T, ops, in_a, in_b, idx, testvec, bkd, out, out_mode, B, s, 'o', O, used);
    case PLAN_WHOLE_TAIL: {
        hipError_t e = launch_blind_rotate_range(P, T, ops, in_a, in_b, idx, testvec, bkd, out, out_mode, 0, B - tail,
                                                 s, 'w', O, used);
        if (e != hipSuccess) return e;
        return launch_blind_rotate_range(P, T, ops, in_a, in_b, idx, testvec, bkd, out, out_mode, B - tail, tail, s,
                                         'W', O, nullptr);
    }
    default:
        return launch_blind_rotate_form(P, T, ops, in_a, in_b, idx, testvec, bkd, out, out_mode, B, s, 'w', O, used);
    }
}

// The margin guard's recompute: the whole form in the
// reference's expression trees over the same B items, whose workgroups return
// at once unless one of their 4 items was flagged by the fused launch.
static hipError_t launch_br_recompute(const KParams &P, const DevTables &T, const uint8_t *ops, const uint32_t *in_a,
                                      const uint32_t *in_b, const uint32_t *idx, const uint32_t *testvec,
                                      const double2 *bk2, uint32_t *out, int out_mode, size_t B, hipStream_t s) {
    KParams Q = P;
    Q.fallback = 1;
    const dim3 grid((unsigned)((B + BR_WAVES - 1) / BR_WAVES)), block(64 * BR_WAVES * 2);
    switch (P.L) {
    case 1: hipLaunchKernelGGL((k_blind_rotate<1, true, true, false, true>), grid, block, 0, s, Q, T, ops, in_a, in_b, idx, testvec, bk2, out, out_mode, B); break;
    case 2: hipLaunchKernelGGL((k_blind_rotate<2, true, true, false, true>), grid, block, 0, s, Q, T, ops, in_a, in_b, idx, testvec, bk2, out, out_mode, B); break;
    case 3: hipLaunchKernelGGL((k_blind_rotate<3, true, true, false, true>), grid, block, 0, s, Q, T, ops, in_a, in_b, idx, testvec, bk2, out, out_mode, B); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_blind_rotate(const KParams &P, const DevTables &T, const uint8_t *ops,
                               const uint32_t *in_a, const uint32_t *in_b, const uint32_t *idx,
                               const uint32_t *testvec, const double *bkd, uint32_t *out, int out_mode, size_t B,
                               hipStream_t s, const LaunchOpts &O, const char **used) {
    if (B == 0) return hipSuccess;
    KParams Q = P;
    Q.fallback = 0;
    const bool fused = small_products(P) && fused_allowed(O);
    if (!fused) Q.tie_flags = nullptr;
    hipError_t e = launch_blind_rotate_forms(Q, T, ops, in_a, in_b, idx, testvec, bkd, out, out_mode, B, s, O, used);
#ifdef TFHE_FU_UNGUARDED  // A/B builds: the fused arithmetic without its margin guard
    return e;
#endif
    if (e != hipSuccess || !fused || !Q.tie_flags) return e;
    return launch_br_recompute(Q, T, ops, in_a, in_b, idx, testvec, reinterpret_cast<const double2 *>(bkd), out,
                               out_mode, B, s);
}

// lane-form key switch over an input of n_in coefficients (+ b); false if
// (t, basebit) has no instantiation
static bool launch_ks_lanes(const KParams &P, int t_, int basebit, const uint32_t *in, int n_in, int in_stride,
                            const uint32_t *key, uint32_t *out, size_t B, hipStream_t s, const LaunchOpts &O,
                            const char **used) {
    const unsigned groups = (unsigned)((B + 63) / 64);
    dim3 grid((unsigned)((P.ks_stride + KL_CHUNK - 1) / KL_CHUNK), groups), block(64 * KL_WAVES);
    // basebit 2 (128/80-bit): the 44-word x 8-wave blocks when they spread the
    // work more evenly over the 256 CUs (rounds of one block per CU x pieces per
    // block); 1024 gates at 128-bit: 1 round x 11 pieces instead of 2 x 8
    const unsigned wide_chunks = (unsigned)((P.ks_stride + KL_CHUNK_WIDE - 1) / KL_CHUNK_WIDE);
    const size_t rounds = (grid.x * (size_t)groups + 255) / 256, rounds_w = (wide_chunks * (size_t)groups + 255) / 256;
    const bool wide = basebit == 2 && !O.ks_narrow && rounds_w * (KL_CHUNK_WIDE / 4) < rounds * (KL_CHUNK / 4);
    if (wide) {
        dim3 gw(wide_chunks, groups), bw(64 * KL_WAVES_WIDE);
#define KS_WIDE(T_)                                                                                                     \
    do {                                                                                                                \
        hipLaunchKernelGGL((k_key_switch_lanes<T_, 2, KL_CHUNK_WIDE, KL_WAVES_WIDE>), gw, bw, 0, s, P, in, key, out, B, \
                           n_in, in_stride);                                                                            \
        if (used) *used = "k_key_switch_lanes<" #T_ ",2,44,8,1>";                                                       \
    } while (0)
        if (t_ == 9) KS_WIDE(9);
        else if (t_ == 8) KS_WIDE(8);
        else if (t_ == 7) KS_WIDE(7);
        else return false;
#undef KS_WIDE
        return true;
    }
    // UINT4 (basebit 5): the 323 MB KSK streams from HBM once per item group, so
    // 4 groups per block share each chunk through L2, and (default) one ring of
    // 4 buffers per block keeps 3 coefficients in flight (k_key_switch_ring).
    // LaunchOpts::ks_groups forces the lane form with 1, 2, 4 or 8 groups.
    if (!O.ks_groups && basebit == 5 && B > 64 && (t_ == 3 || t_ == 2)) {
        dim3 gr(grid.x, (unsigned)((B + 255) / 256)), br(256);
        if (t_ == 3) hipLaunchKernelGGL((k_key_switch_ring<3, 5, KL_CHUNK, 4, KS_RING_DEPTH>), gr, br, 0, s, P, in, key, out, B, n_in, in_stride);
        else hipLaunchKernelGGL((k_key_switch_ring<2, 5, KL_CHUNK, 4, KS_RING_DEPTH>), gr, br, 0, s, P, in, key, out, B, n_in, in_stride);
        if (used) *used = t_ == 3 ? "k_key_switch_ring<3,5,32,4,4>" : "k_key_switch_ring<2,5,32,4,4>";
        return true;
    }
    const int gw = O.ks_groups ? O.ks_groups : (basebit >= 5 ? 4 : 1);
    if (gw == 8 && basebit == 5 && t_ == 3 && B > 64) {  // 16-word chunks: 8 rings fit the LDS
        dim3 g8((unsigned)((P.ks_stride + 15) / 16), (unsigned)((B + 511) / 512)), b8(512);
        hipLaunchKernelGGL((k_key_switch_lanes<3, 5, 16, 8, 8>), g8, b8, 0, s, P, in, key, out, B, n_in, in_stride);
        if (used) *used = "k_key_switch_lanes<3,5,16,8,8>";
        return true;
    }
    if (gw == 4 && basebit == 5 && B > 64) {
        dim3 g4(grid.x, (unsigned)((B + 255) / 256)), b4(256);
        if (t_ == 3) hipLaunchKernelGGL((k_key_switch_lanes<3, 5, KL_CHUNK, 4, 4>), g4, b4, 0, s, P, in, key, out, B, n_in, in_stride);
        else if (t_ == 2) hipLaunchKernelGGL((k_key_switch_lanes<2, 5, KL_CHUNK, 4, 4>), g4, b4, 0, s, P, in, key, out, B, n_in, in_stride);
        else return false;
        if (used) *used = t_ == 3 ? "k_key_switch_lanes<3,5,32,4,4>" : "k_key_switch_lanes<2,5,32,4,4>";
        return true;
    }
    if (gw == 2 && basebit == 5 && B > 64) {
        dim3 g2(grid.x, (unsigned)((B + 127) / 128)), b2(256);
        if (t_ == 3) hipLaunchKernelGGL((k_key_switch_lanes<3, 5, KL_CHUNK, 4, 2>), g2, b2, 0, s, P, in, key, out, B, n_in, in_stride);
        else if (t_ == 2) hipLaunchKernelGGL((k_key_switch_lanes<2, 5, KL_CHUNK, 4, 2>), g2, b2, 0, s, P, in, key, out, B, n_in, in_stride);
        else return false;
        if (used) *used = t_ == 3 ? "k_key_switch_lanes<3,5,32,4,2>" : "k_key_switch_lanes<2,5,32,4,2>";
        return true;
    }
#define KS_LANES(T_, BB_)                                                                                     \
    do {                                                                                                      \
        hipLaunchKernelGGL((k_key_switch_lanes<T_, BB_>), grid, block, 0, s, P, in, key, out, B, n_in, in_stride); \
        if (used) *used = "k_key_switch_lanes<" #T_ "," #BB_ ",32,4,1>";                                      \
    } while (0)
    if (basebit == 2 && t_ == 9) KS_LANES(9, 2);
    else if (basebit == 2 && t_ == 8) KS_LANES(8, 2);
    else if (basebit == 2 && t_ == 7) KS_LANES(7, 2);
    else if (basebit == 3 && t_ == 4) KS_LANES(4, 3);
    else if (basebit == 4 && t_ == 3) KS_LANES(3, 4);
    else if (basebit == 4 && t_ == 4) KS_LANES(4, 4);
    else if (basebit == 5 && t_ == 3) KS_LANES(3, 5);
    else if (basebit == 5 && t_ == 2) KS_LANES(2, 5);
    else return false;
#undef KS_LANES
    return true;
}

static hipError_t launch_ks_gemm(const KParams &P, int t, int basebit, int n_in, int in_stride, const uint32_t *in,
                                 const KsGemm &G, uint32_t *out, size_t B, hipStream_t s, const char **used);

hipError_t launch_reencrypt(const KParams &P, int t_, int basebit, const uint32_t *in, const uint32_t *key,
                            uint32_t *out, size_t B, hipStream_t s, const LaunchOpts &O, const char **used,
                            const KsGemm *KG) {
    if (B == 0) return hipSuccess;
    if (KG && KG->kg && KG->part && ks_gemm_supported(t_, basebit) &&
        (O.ks_form == 2 || (O.ks_form == 3 && ks_gemm_auto(t_, basebit))))
        return launch_ks_gemm(P, t_, basebit, P.n, P.n + 1, in, *KG, out, B, s, used);
    if (!launch_ks_lanes(P, t_, basebit, in, P.n, P.n + 1, key, out, B, s, O, used)) return hipErrorInvalidValue;
    return hipGetLastError();
}

bool reencrypt_supported(int t_, int basebit) {
    return (basebit == 2 && t_ >= 7 && t_ <= 9) || (basebit == 3 && t_ == 4) || (basebit == 4 && (t_ == 3 || t_ == 4)) ||
           (basebit == 5 && (t_ == 2 || t_ == 3));
}

// K splits of the gemm form: enough workgroups for one per CU.
static int ks_gemm_splits(const KParams &P, size_t B, int n_in, int basebit) {
    const size_t tiles = (size_t)(P.n + 1 + 31) / 32 * ((B + KG_ITEMS - 1) / KG_ITEMS);
    const size_t z = std::max<size_t>(1, device_cus() / tiles);
    return (int)std::min<size_t>(z, (size_t)kg_blocks(n_in, basebit));
}
size_t ks_gemm_part_bytes(const KParams &P, size_t B, int n_in, int basebit) {
    return (size_t)ks_gemm_splits(P, B, n_in, basebit) * B * (P.n + 1) * 4;
}

// One-hot GEMM key switch of B inputs of in_stride words (n_in coefficients, then b)
// against a MFMA-layout key of t levels of basebit (ks_gemm_supported).  The
// kernel reads whole blocks of coefficients: when they reach past in_stride the
// input buffer needs KS_GEMM_INPUT_SLACK readable bytes past its last row.
static hipError_t launch_ks_gemm(const KParams &P, int t, int basebit, int n_in, int in_stride, const uint32_t *in,
                                 const KsGemm &G, uint32_t *out, size_t B, hipStream_t s, const char **used) {
    const int nib = kg_blocks(n_in, basebit);
    const int z = ks_gemm_splits(P, B, n_in, basebit);
    const int per = (nib + z - 1) / z;
    const int splits = (nib + per - 1) / per;
    dim3 grid((unsigned)((P.n + 1 + 31) / 32), (unsigned)((B + KG_ITEMS - 1) / KG_ITEMS), (unsigned)splits),
        block(64 * KG_WAVES);
#define KG_LAUNCH(T_, BB_)                                                                                       \
    do {                                                                                                         \
        hipLaunchKernelGGL((k_key_switch_gemm<T_, BB_>), grid, block, 0, s, P, in, G.kg, G.part, B, per, n_in, \
                           in_stride);                                                                           \
        if (used) *used = "k_key_switch_gemm<" #T_ "," #BB_ "> + k_ks_gemm_reduce";                              \
    } while (0)
    if (basebit == 2 && t == 9) KG_LAUNCH(9, 2);
    else if (basebit == 2 && t == 8) KG_LAUNCH(8, 2);
    else if (basebit == 2 && t == 7) KG_LAUNCH(7, 2);
    else if (basebit == 5 && t == 3) KG_LAUNCH(3, 5);
    else if (basebit == 5 && t == 2) KG_LAUNCH(2, 5);
    else return hipErrorInvalidValue;
#undef KG_LAUNCH
    const size_t total = B * (size_t)(P.n + 1);
    hipLaunchKernelGGL(k_ks_gemm_reduce, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, P, in, G.part, out, B,
                       splits, n_in, in_stride, t, basebit);
    return hipGetLastError();
}

bool ks_gemm_supported(int t, int basebit) {
    return (basebit == 2 && t >= 7 && t <= 9) || (basebit == 5 && (t == 2 || t == 3));
}
bool ks_gemm_supported(const KParams &P) { return ks_gemm_supported(P.iks_t, P.basebit); }
// Batches from this size take the GEMM under TFHE_OPT_KS_FORM = 3: it is the
// faster form from 64 items up (0.050 vs 0.218 ms at 64, 0.090 vs 0.239 ms at
// 1,024, 0.35 vs 0.94 ms at 4,096; profiles/r03k_ks_gemm.txt), and a batch of
// one still fills 242 workgroups (22 tiles x 11 K splits).
size_t KS_GEMM_MIN_ITEMS = 1;
// TFHE_OPT_KS_FORM = 3 takes the GEMM wherever it applies: at basebit 5 too
// (UINT4, 4,096 items: 0.90 ms against the ring form's 1.24 ms, config 5
// 182.5 k -> 186.0 k/s; profiles/r03m_ks_gemm_uint4.txt)
bool ks_gemm_auto(int t, int basebit) { return ks_gemm_supported(t, basebit); }

hipError_t launch_ksk_to_gemm(const KParams &P, const uint32_t *ksk, uint32_t *kg, int n_in, int t, int basebit,
                              hipStream_t s) {
    const size_t words = ks_gemm_bytes(P, n_in, t, basebit) / 4;
    hipLaunchKernelGGL(k_ksk_to_gemm, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, s, P, ksk, kg, words, n_in,
                       t, basebit);
    return hipGetLastError();
}

hipError_t launch_key_switch(const KParams &P, const uint32_t *lv1, const uint32_t *ksk, uint32_t *out,
                             size_t B, hipStream_t s, const LaunchOpts &O, const char **used, const KsGemm *KG) {
    if (B == 0) return hipSuccess;
    // kernel form (TFHE_OPT_KS_FORM): 3 auto (default) = the one-hot GEMM for
    // basebit 2 from KS_GEMM_MIN_ITEMS items, else lanes; 2 the GEMM wherever it
    // applies; 0 lanes; 1 the select / gather forms
    const bool gemm_ok = KG && KG->kg && KG->part && ks_gemm_supported(P);
    if (gemm_ok && (O.ks_form == 2 || (O.ks_form == 3 && B >= KS_GEMM_MIN_ITEMS && ks_gemm_auto(P.iks_t, P.basebit))))
        return launch_ks_gemm(P, P.iks_t, P.basebit, 1024, 1025, lv1, *KG, out, B, s, used);
    if (O.ks_form != 1 && launch_ks_lanes(P, P.iks_t, P.basebit, lv1, 1024, 1025, ksk, out, B, s, O, used))
        return hipGetLastError();
    // items per block: TFHE_OPT_KS_SEL_ITEMS in {8, 16, 32} (default 8)
    const int G = (O.ks_sel_items == 16 || O.ks_sel_items == 32) ? O.ks_sel_items : 8;
    if (used) *used = P.basebit == 2 ? "k_key_switch_sel" : "k_key_switch_gather";
    dim3 grid((unsigned)((P.n + 1 + 255) / 256), (unsigned)((B + G - 1) / G)), block(256);
#define KS_SEL(T_, G_) hipLaunchKernelGGL((k_key_switch_sel<T_, G_>), grid, block, 0, s, P, lv1, ksk, out, B)
#define KS_GATHER(T_, G_) hipLaunchKernelGGL((k_key_switch_gather<T_, G_>), grid, block, 0, s, P, lv1, ksk, out, B)
#define KS_G(KIND, T_)                  \
    do {                                \
        if (G == 16) KIND(T_, 16);      \
        else if (G == 32) KIND(T_, 32); \
        else KIND(T_, 8);               \
    } while (0)
    if (P.basebit == 2) {
        switch (P.iks_t) {
        case 7: KS_G(KS_SEL, 7); break;
        case 8: KS_G(KS_SEL, 8); break;
        case 9: KS_G(KS_SEL, 9); break;
        default: return hipErrorInvalidValue;
        }
    } else {
        switch (P.iks_t) {
        case 2: KS_G(KS_GATHER, 2); break;
        case 3: KS_G(KS_GATHER, 3); break;
        case 4: KS_G(KS_GATHER, 4); break;
        default: return hipErrorInvalidValue;
        }
    }
#undef KS_SEL
#undef KS_GATHER
#undef KS_G
    return hipGetLastError();
}

hipError_t launch_ksk_zero_k0(const KParams &P, uint32_t *ksk, hipStream_t s) {
    return launch_key_zero_k0(P, ksk, 1024, P.iks_t, P.basebit, s);
}

hipError_t launch_key_zero_k0(const KParams &P, uint32_t *ksk, int n_in, int t_, int basebit, hipStream_t s) {
    const int rs = P.ks_stride, base = 1 << basebit;
    const size_t groups = (size_t)n_in * t_;
    const size_t total = groups * rs;
    hipLaunchKernelGGL(k_ksk_zero_k0, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, ksk, rs, base,
                       groups);
    return hipGetLastError();
}

hipError_t launch_fft_forward(const DevTables &T, const uint32_t *in, double *out, size_t B, hipStream_t s) {
    if (B == 0) return hipSuccess;
    hipLaunchKernelGGL(k_fft_forward, dim3((unsigned)B), dim3(64), 0, s, T, in, out);
    return hipGetLastError();
}

hipError_t launch_fft_inverse(const DevTables &T, const double *in, uint32_t *out, size_t B, hipStream_t s) {
    if (B == 0) return hipSuccess;
    hipLaunchKernelGGL(k_fft_inverse, dim3((unsigned)B), dim3(64), 0, s, T, in, out);
    return hipGetLastError();
}

hipError_t launch_poly_mul(const DevTables &T, const uint32_t *a, const uint32_t *b, size_t b_stride,
                           uint32_t *out, size_t B, hipStream_t s) {
    if (B == 0) return hipSuccess;
    hipLaunchKernelGGL(k_poly_mul, dim3((unsigned)B), dim3(64), 0, s, T, a, b, b_stride, out);
    return hipGetLastError();
}

hipError_t launch_external_product(const KParams &P, const DevTables &T, const double *bkd_row,
                                   const uint32_t *in, uint32_t *out, size_t B, hipStream_t s) {
    if (B == 0) return hipSuccess;
    const double2 *bk2 = reinterpret_cast<const double2 *>(bkd_row);
    switch (P.L) {
    case 1: hipLaunchKernelGGL(k_external_product<1>, dim3((unsigned)B), dim3(64), 0, s, P, T, bk2, in, out); break;
    case 2: hipLaunchKernelGGL(k_external_product<2>, dim3((unsigned)B), dim3(64), 0, s, P, T, bk2, in, out); break;
    case 3: hipLaunchKernelGGL(k_external_product<3>, dim3((unsigned)B), dim3(64), 0, s, P, T, bk2, in, out); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Order-independent 64-bit fingerprint of a device buffer (16-B words; the
// key buffers are multiples of 16 B): sum over words i of a SplitMix64-style
// mix of (word, i), one vector atomic add per wave.  Compares the key copies
// of a multi-device context after its broadcast (HBM-bound, ~35 us per key).
__global__ __launch_bounds__(256) void k_checksum(const uint4 *__restrict__ p, size_t words16, unsigned long long *out) {
    unsigned long long acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < words16; i += (size_t)gridDim.x * 256) {
        const uint4 v = p[i];
        unsigned long long x = (((unsigned long long)v.y << 32) | v.x) ^ (i * 0x9E3779B97F4A7C15ull);
        unsigned long long y = (((unsigned long long)v.w << 32) | v.z) + (i * 0xD1B54A32D192ED03ull);
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
        y = (y ^ (y >> 27)) * 0x94D049BB133111EBull;
        acc += (x ^ (x >> 31)) + (y ^ (y >> 29));
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);
}

// Largest |x| over a buffer of doubles (the fused arithmetic's key admission,
// DESIGN.md §6.1): the bit patterns of non-negative doubles order like their
// values (a NaN above every number), so a 64-bit max per lane, per wave, and
// one atomic max per wave.
__global__ __launch_bounds__(256) void k_absmax_f64(const double2 *__restrict__ p, size_t n2, unsigned long long *out) {
    unsigned long long m = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) {
        const double2 v = p[i];
        const unsigned long long a = (unsigned long long)__double_as_longlong(v.x) & 0x7FFFFFFFFFFFFFFFull;
        const unsigned long long b = (unsigned long long)__double_as_longlong(v.y) & 0x7FFFFFFFFFFFFFFFull;
        m = a > m ? a : m;
        m = b > m ? b : m;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long x = __shfl_xor(m, o);
        m = x > m ? x : m;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

hipError_t launch_absmax(const double *p, size_t count, unsigned long long *out, hipStream_t s) {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(*out), s);
    if (e != hipSuccess || count < 2) return e;
    const size_t n2 = count / 2;
    const unsigned blocks = (unsigned)std::min<size_t>((n2 + 255) / 256, 2048);
    hipLaunchKernelGGL(k_absmax_f64, dim3(blocks), dim3(256), 0, s, reinterpret_cast<const double2 *>(p), n2, out);
    return hipGetLastError();
}

hipError_t launch_checksum(const void *p, size_t bytes, unsigned long long *out, hipStream_t s) {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(*out), s);
    if (e != hipSuccess || bytes < 16) return e;
    const size_t w = bytes / 16;
    const unsigned blocks = (unsigned)std::min<size_t>((w + 255) / 256, 2048);
    hipLaunchKernelGGL(k_checksum, dim3(blocks), dim3(256), 0, s, reinterpret_cast<const uint4 *>(p), w, out);
    return hipGetLastError();
}

hipError_t launch_bk_permute(const KParams &, const double *bk_ref, double *bkd, size_t rows, hipStream_t s) {
    size_t total = rows * 512;
    if (!total) return hipSuccess;
    hipLaunchKernelGGL(k_bk_permute, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, bk_ref,
                       reinterpret_cast<double2 *>(bkd), rows, 0);
    return hipGetLastError();
}

hipError_t launch_bk_unpermute(const KParams &, const double *bkd, double *bk_ref, size_t rows, hipStream_t s) {
    size_t total = rows * 512;
    if (!total) return hipSuccess;
    hipLaunchKernelGGL(k_bk_permute, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, bk_ref,
                       reinterpret_cast<double2 *>(const_cast<double *>(bkd)), rows, 1);
    return hipGetLastError();
}

#endif  // TFHE_WHOLE_TU
}  // namespace tfhe
