// tfhe_ab_forms.hip — blind-rotation forms that lost their A/B runs, kept
// buildable for further A/B work but NOT part of the product library
// (VERDICT r04 item 3).  tools/ab_forms.sh links this unit into an A/B library
// (tools/bin/lib_ab.so, compiled with TFHE_AB_BUILD: tfhe_gpu_create refuses
// it unless TFHE_ALLOW_AB_BUILD=1), where TFHE_OPT_BR_FORM 6 (duo), 7
// (split-transform latency form) and 8 (round 4's whole form at L = 3, whose
// loader waves only issue DMAs: the reference point of the round-5 loader
// assist) reach these kernels through the product launcher's weak hook
// ab_launch_blind_rotate.  Measurements: DESIGN.md §4.2 (wide2: 109.4-109.8 vs
// 99.9 ms per 16-bit adder), §4.3d (duo: 7.93-8.05 vs 6.12-6.18 ms per 1,024
// gates), §4.1b (assist).  The development switches below (TFHE_KO_*,
// TFHE_DUO_*) apply to this unit only.
#include <cmath>

#include "../../zig-tfhe_amd/csrc/tfhe_device.hpp"

namespace tfhe {

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
        pp.flush(g_phase_cycles, 8);
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

hipError_t ab_launch_wide_rc(const KParams &P, const DevTables &T, const uint8_t *ops, const uint32_t *in_a,
                             const uint32_t *in_b, const uint32_t *idx, const uint32_t *testvec, const double2 *bk2,
                             uint32_t *out, int out_mode, size_t B, hipStream_t s, const char **used);  // tfhe_kernels.hip
hipError_t ab_launch_assist_dev(int var, dim3 grid, dim3 block, hipStream_t s, const KParams &P, const DevTables &T,
                                const uint8_t *ops, const uint32_t *in_a, const uint32_t *in_b, const uint32_t *idx,
                                const uint32_t *testvec, const double2 *bk2, uint32_t *out, int out_mode, size_t B,
                                const char **used);  // tfhe_ab_assist_dev.hip

// TFHE_OPT_BR_FORM 6 / 7 / 8 (and 9 + VAR: tfhe_ab_assist_dev.hip) from the product launcher
// (launch_blind_rotate_form).
hipError_t ab_launch_blind_rotate(int br_form, const KParams &P, const DevTables &T, const uint8_t *ops,
                                  const uint32_t *in_a, const uint32_t *in_b, const uint32_t *idx,
                                  const uint32_t *testvec, const double2 *bk2, uint32_t *out, int out_mode, size_t B,
                                  hipStream_t s, bool fused, const char **used) {
    const bool small = std::ldexp(2.0 * P.L * 1024.0, P.bgbit - 1 + 31) < std::ldexp(1.0, 49);
    if (br_form == 30) {  // the latency form with row counters (tfhe_kernels.hip, RC = 1)
        if (!(P.L == 3 && small && fused)) return hipErrorInvalidValue;
        return ab_launch_wide_rc(P, T, ops, in_a, in_b, idx, testvec, bk2, out, out_mode, B, s, used);
    }
    if (br_form == 6) {  // duo: two computing waves per item
        const dim3 grid((unsigned)((B + BD_GATES - 1) / BD_GATES)), block(64 * BD_WAVES);
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
            return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    if (br_form == 8 && P.L == 3 && small && fused) {  // round 4's whole form at L = 3 (loader waves issue DMAs only)
        const dim3 grid((unsigned)((B + BR_WAVES - 1) / BR_WAVES)), block(64 * BR_WAVES * 2);
        hipLaunchKernelGGL((k_blind_rotate<3, true, true>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec, bk2,
                           out, out_mode, B);
        if (used) *used = "k_blind_rotate<3,true,true> (whole form without loader assist, fused)";
        return hipGetLastError();
    }
    if (br_form >= 9 && P.L == 3 && small && fused) {  // development copies of the assist form
        const dim3 grid((unsigned)((B + BR_WAVES - 1) / BR_WAVES)), block(64 * BR_WAVES * 2);
        return ab_launch_assist_dev(br_form - 9, grid, block, s, P, T, ops, in_a, in_b, idx, testvec, bk2, out, out_mode,
                                    B, used);
    }
    if (br_form == 7 && P.L == 3 && small) {  // latency form with split transforms
        const dim3 grid((unsigned)B), block(64 * BW_WAVES);
        if (fused) {
            hipLaunchKernelGGL((k_blind_rotate_wide2<3, true, true>), grid, block, 0, s, P, T, ops, in_a, in_b, idx,
                               testvec, bk2, out, out_mode, B);
            if (used) *used = "k_blind_rotate_wide2<3,true,true> (latency form, split transforms, fused)";
        } else {
            hipLaunchKernelGGL((k_blind_rotate_wide2<3, true, false>), grid, block, 0, s, P, T, ops, in_a, in_b, idx,
                               testvec, bk2, out, out_mode, B);
            if (used) *used = "k_blind_rotate_wide2<3,true,false> (latency form, split transforms)";
        }
        return hipGetLastError();
    }
    return hipErrorInvalidValue;
}

}  // namespace tfhe
