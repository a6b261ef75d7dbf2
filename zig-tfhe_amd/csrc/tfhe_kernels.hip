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
//
// This unit: the octo and latency blind-rotation forms, the reference-tree
// and UINT4 instantiations of the whole form, the key switch, the stage
// kernels and every launcher; the device building blocks are in
// tfhe_device.hpp, the default whole-form kernels in tfhe_kernels_whole.hip.
#include <algorithm>

#include "tfhe_device.hpp"

namespace tfhe {


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
        fft512<1, false, FU, LdsTwAtPass, true>(d, xb, T, t);
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

// The split and pair forms (two waves per item) were removed in round 4, and the
// duo form and the split-transform latency form moved to tools/ab/ in round 5:
// all measured slower than the forms here.


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
constexpr size_t BR_WIDE_MAX_ITEMS = 512;  // measured: 1 gate 4.3 vs 9.9 ms; 512 gates 8.8 vs 10.2 ms; 1024: 17.1 vs 10.4 ms
// measured settings: the inverse on waves 2 and 3 (waves 0, 1 in round 2), the
// row waves 4 and 5 at issue priority 1 (99.7 -> 99.2 ms per adder; 1, 2, 3
// measure the same, profiles/r04_ab_wide_prio.txt)
constexpr int WIDE_INV_W0 = 2;
constexpr int WIDE_ROW45_PRIO = 1;

// RC (row counters, round 6; L = 3): no workgroup barrier between the
// forward and inverse phases.  Each row wave publishes its two term spectra with a per-row LDS
// counter; the inverse waves (2, 3) sum their output's six rows themselves, in the reference's
// row order, each row as soon as its counter says it landed, so most of the sum runs while the
// last rows are still transforming, and the sums stay in registers for the inverse.  Rows 0, 1
// move to waves 2, 3 (the SIMDs that carry one row wave each: the first rows of the order land
// first), rows 2, 3 to waves 0, 1 at issue priority 1 over rows 4, 5 on their shared SIMDs.
// Same row order and arithmetic: the same words.
template <int L, bool SMALL, bool FU = false, int RC = 0>
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
    __shared__ uint32_t s_rows[8];  // RC: terms of row r published for steps < s_rows[r]
    static_assert(!RC || L == 3, "row counters: L = 3");
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
    if (RC && tid < 8) s_rows[tid] = 0u;
    // the row this wave transforms (RC: rows 0, 1 on waves 2, 3; rows 2, 3 on waves 0, 1)
    const int row = RC && w < 4 ? w ^ 2 : w;
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
            for (int h = 0; h < 2; h++) kr[q][h] = bkd[((size_t)row * 8 + q) * 128 + h * 64 + t];
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
    // right after their terms; RC: every row wave right after its terms)
    const bool pf_late = !RC && w < 2 * L && !is_inv;
    // the inverse waves keep their polynomial's 16 accumulator words per lane
    // in registers: the update then waits for no LDS read
    uint32_t accr[16];
    if (is_inv) {
#pragma unroll
        for (int m = 0; m < 16; m++) accr[m] = s_acc[ipoly * 1024 + t + 64 * m];
    }

    // rows 4 and 5 share their SIMDs with rows 0 and 1 and finish the forward
    // phase last; at a higher issue priority they take the VALU first
    // (RC: rows 2 and 3 on waves 0 and 1 instead, ahead of rows 4 and 5 in the sum's order)
    if (RC ? (w == 0 || w == 1) : (w == 4 || w == 5)) __builtin_amdgcn_s_setprio(WIDE_ROW45_PRIO);
    uint32_t fail = 0;  // RC: a row-counter wait gave up (report_wait_failure)
    const uint32_t spin_cap = P.spin_cap ? P.spin_cap : BR_SPIN_CAP_DEFAULT;
    int at_next = s_at[0];  // a~ read one step ahead (its wait would drain every LDS op)
    uint32_t near = NEAR_NONE;  // FU: margin guard (the inverse waves)
    PhaseProf pp;  // development timing (TFHE_PHASE_PROF), per wave
    pp.start();
    for (int i = 0; i < n; i++) {
        pp.mark(0);
        const int at = __builtin_amdgcn_readfirstlane(at_next);
        at_next = s_at[i + 1 < n ? i + 1 : i];
        if (w < 2 * L) {
            const int poly = row >= L ? 1 : 0;
            const int level = row - poly * L;
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
            fft512<1, false, FU>(d, s_prod[0][row], T, t);
            pp.mark(11);
            // this row's terms of fmaInFd1024 for both outputs, every frequency
            // (after this wave's exchanges in s_prod[0][row])
#pragma unroll
            for (int q = 0; q < 8; q++) {
                s_prod[0][row][t + 64 * q] = cmul_bk<FU>(d[0][q], kr[q][0]);
                s_prod[1][row][t + 64 * q] = cmul_bk<FU>(d[0][q], kr[q][1]);
            }
            if (RC) {
                __builtin_amdgcn_sched_barrier(0);
                counter_add(s_rows + row);  // the terms land before the count (one wave's LDS ops run in order)
            }
            pp.mark(14);
            // next step's BK row, landing under the sum, inverse and forward
            // phases.  The inverse waves (2, 3) issue it here; the other row
            // waves wait for the inverse phase, where they are idle: 16 KB per
            // wave through the CU's vector-memory path no longer queues behind
            // 5 other waves' at the end of the forward phase, which is the
            // critical path (rows 4 and 5 share SIMDs with rows 0 and 1):
            // 104.7 -> 101.8 ms per 16-bit adder with the inverse on waves 2, 3
            // (profiles/r03q_wide_prefetch_inverse.txt).
            if (i + 1 < n && !pf_late) wide_prefetch(kr, bkd + (size_t)(i + 1) * trgsw, row, t);
        }
        if (RC) {
            if (is_inv) {
                // this output's sum over rows 0..2L-1 in the reference's order, each row once
                // its counter shows this step's terms (fmaInFd1024 starts from 0.0: 0.0 + x == x)
                C2 fs[8];
                pp.mark(2);
#pragma unroll
                for (int r = 0; r < 2 * L; r++) {
                    uint32_t f = 0;
                    spin_until_ge<1>(s_rows + r, (uint32_t)i + 1u, spin_cap, f);
                    fail |= f;
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        const C2 tq = s_prod[ipoly][r][t + 64 * q];
                        fs[q] = r == 0 ? tq : c2(fs[q].x + tq.x, fs[q].y + tq.y);
                    }
                }
                pp.mark(4);
                C2 e[1][8];
#pragma unroll
                for (int q = 0; q < 8; q++) e[0][q] = fs[br3(q)];
                C2 twr[8];
#pragma unroll
                for (int q = 0; q < 8; q++) twr[q] = twist_t[64 * q];
                pp.mark(12);
                // exchange buffer: row 0's term spectrum of this output, already summed; only
                // this wave reads it this step, and row 0's wave rewrites it after the barrier
                fft512<1, true, FU>(e, s_prod[ipoly][0], T, t);
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
            __syncthreads();  // accumulator updated, every term read
            continue;
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
        if (pf_late && i + 1 < n) wide_prefetch(kr, bkd + (size_t)(i + 1) * trgsw, row, t);
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
        pp.flush(g_phase_cycles + w * 16, 16);
#endif
    if (RC) report_wait_failure(P, fail, DEV_ERR_GATE_WAIT);
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
constexpr int KS_RING_DEPTH = 4;  // ring depths 3-8 measure the same (profiles/r02_ab_ks_ring.txt)
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

// Forms that lost their A/B runs (the duo form, §4.3d, and the split-transform
// latency form, §4.2 of DESIGN.md) are not in the product library: they live in
// tools/ab/tfhe_ab_forms.hip, which an A/B library links in (tools/ab_forms.sh)
// and which then defines this hook.  In the product it stays unresolved (null).
__attribute__((weak)) hipError_t ab_launch_blind_rotate(int br_form, const KParams &P, const DevTables &T,
                                                        const uint8_t *ops, const uint32_t *in_a,
                                                        const uint32_t *in_b, const uint32_t *idx,
                                                        const uint32_t *testvec, const double2 *bk2, uint32_t *out,
                                                        int out_mode, size_t B, hipStream_t s, bool fused,
                                                        const char **used);
bool ab_forms_linked() { return ab_launch_blind_rotate != nullptr; }
#ifdef TFHE_AB_BUILD
bool kernels_ab_build() { return true; }
#else
bool kernels_ab_build() { return false; }
#endif

// form: 'w' whole (default kernels: launch_whole_default), 'W' latency (one
// item per 8-wave workgroup), 'o' octo (L = 1: 8 items per workgroup), 'a' the
// A/B forms (TFHE_OPT_BR_FORM 6-8, A/B libraries only).
static hipError_t launch_blind_rotate_form(const KParams &P, const DevTables &T, const uint8_t *ops,
                                           const uint32_t *in_a, const uint32_t *in_b, const uint32_t *idx,
                                           const uint32_t *testvec, const double *bkd, uint32_t *out, int out_mode,
                                           size_t B, hipStream_t s, char form, const LaunchOpts &O,
                                           const char **used) {
    if (B == 0) return hipSuccess;
    const double2 *bk2 = reinterpret_cast<const double2 *>(bkd);
    const bool small = small_products(P);
    // fused arithmetic in the exact-integer regime (SMALL) unless the
    // reference expression trees are requested (TFHE_OPT_ARITH)
    const bool fused = small && fused_allowed(O);
    if (form == 'a') {  // an A/B form (TFHE_OPT_BR_FORM >= 6)
        if (!ab_launch_blind_rotate) return hipErrorInvalidValue;
        return ab_launch_blind_rotate(O.br_form, P, T, ops, in_a, in_b, idx, testvec, bk2, out, out_mode, B, s, fused,
                                      used);
    }
    if (form == 'o') {  // octo form: 8 items per workgroup, two gate waves per SIMD; L = 1
        if (P.L != 1) return hipErrorInvalidValue;
        const dim3 grid((unsigned)((B + BO_GATES - 1) / BO_GATES)), block(64 * BO_GATES);
        if (fused) {
            hipLaunchKernelGGL((k_blind_rotate_octo<1, true, true>), grid, block, 0, s, P, T, ops, in_a, in_b, idx,
                               testvec, bk2, out, out_mode, B);
            if (used) *used = "k_blind_rotate_octo<1,true,true> (octo form, fused)";
        } else if (small) {
            hipLaunchKernelGGL((k_blind_rotate_octo<1, true, false>), grid, block, 0, s, P, T, ops, in_a, in_b, idx,
                               testvec, bk2, out, out_mode, B);
            if (used) *used = "k_blind_rotate_octo<1,true,false> (octo form)";
        } else {
            hipLaunchKernelGGL((k_blind_rotate_octo<1, false, false>), grid, block, 0, s, P, T, ops, in_a, in_b, idx,
                               testvec, bk2, out, out_mode, B);
            if (used) *used = "k_blind_rotate_octo<1,false,false> (octo form)";
        }
        return hipGetLastError();
    }
    if (form == 'W') {  // latency form: one item per 8-wave workgroup
        const dim3 grid((unsigned)B), block(64 * BW_WAVES);
#define BW_LAUNCH(L_, S_)                                                                                         \
    do {                                                                                                          \
        if (fused) {                                                                                              \
            hipLaunchKernelGGL((k_blind_rotate_wide<L_, S_, S_>), grid, block, 0, s, P, T, ops, in_a, in_b, idx,  \
                               testvec, bk2, out, out_mode, B);                                                   \
            if (used) *used = "k_blind_rotate_wide<" #L_ "," #S_ ",true> (latency form, fused)";                  \
        } else {                                                                                                  \
            hipLaunchKernelGGL((k_blind_rotate_wide<L_, S_, false>), grid, block, 0, s, P, T, ops, in_a, in_b,    \
                               idx, testvec, bk2, out, out_mode, B);                                              \
            if (used) *used = "k_blind_rotate_wide<" #L_ "," #S_ ",false> (latency form)";                        \
        }                                                                                                         \
    } while (0)
        switch (P.L) {
        case 1: if (small) BW_LAUNCH(1, true); else BW_LAUNCH(1, false); break;
        case 2: if (small) BW_LAUNCH(2, true); else BW_LAUNCH(2, false); break;
        case 3: if (small) BW_LAUNCH(3, true); else BW_LAUNCH(3, false); break;
        default: return hipErrorInvalidValue;
        }
#undef BW_LAUNCH
        return hipGetLastError();
    }
    // whole form: 4 items + 4 loader waves per 512-thread workgroup
    const dim3 grid((unsigned)((B + BR_WAVES - 1) / BR_WAVES)), block(64 * BR_WAVES * 2);
    if (fused) {  // the default kernels, in their own unit (fused implies SMALL)
        const hipError_t e = launch_whole_default(P.L, grid, block, s, P, T, ops, in_a, in_b, idx, testvec, bk2, out,
                                                  out_mode, B);
        if (used) {
            static const char *names[4] = {"", "k_blind_rotate<1,true,true> (whole form, fused)",
                                           "k_blind_rotate<2,true,true> (whole form, fused)",
                                           "k_blind_rotate_assist<true> (whole form, loader waves own polynomial b, fused)"};
            *used = P.L >= 1 && P.L <= 3 ? names[P.L] : "";
        }
        return e;
    }
#define BR_LAUNCH(L_, S_)                                                                                         \
    do {                                                                                                          \
        hipLaunchKernelGGL((k_blind_rotate<L_, S_, false>), grid, block, 0, s, P, T, ops, in_a, in_b, idx,        \
                           testvec, bk2, out, out_mode, B);                                                       \
        if (used) *used = "k_blind_rotate<" #L_ "," #S_ ",false> (whole form)";                                   \
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

#ifdef TFHE_AB_BUILD
// A/B builds only (tools/ab/tfhe_ab_forms.hip, TFHE_OPT_BR_FORM 30): the latency form with row
// counters (RC = 1) at L = 3, fused.
hipError_t ab_launch_wide_rc(const KParams &P, const DevTables &T, const uint8_t *ops, const uint32_t *in_a,
                             const uint32_t *in_b, const uint32_t *idx, const uint32_t *testvec, const double2 *bk2,
                             uint32_t *out, int out_mode, size_t B, hipStream_t s, const char **used) {
    if (P.L != 3) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_blind_rotate_wide<3, true, true, 1>), dim3((unsigned)B), dim3(64 * BW_WAVES), 0, s, P, T,
                       ops, in_a, in_b, idx, testvec, bk2, out, out_mode, B);
    if (used) *used = "k_blind_rotate_wide<3,true,true,RC> (latency form, row counters, fused)";
    return hipGetLastError();
}
#endif

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
        const char f = O.br_form == 3 ? 'W' : O.br_form == 5 ? 'o' : O.br_form >= 6 ? 'a' : 'w';  // 6-8: A/B forms
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
    case 1: hipLaunchKernelGGL((k_blind_rotate<1, true, false>), grid, block, 0, s, Q, T, ops, in_a, in_b, idx, testvec, bk2, out, out_mode, B); break;
    case 2: hipLaunchKernelGGL((k_blind_rotate<2, true, false>), grid, block, 0, s, Q, T, ops, in_a, in_b, idx, testvec, bk2, out, out_mode, B); break;
    case 3: hipLaunchKernelGGL((k_blind_rotate<3, true, false>), grid, block, 0, s, Q, T, ops, in_a, in_b, idx, testvec, bk2, out, out_mode, B); break;
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

// Largest energy (sum of squared re/im components) of one TRGSW row's spectrum
// over the device BK (the key admission's row-energy rule):
// one wave per (BK[i], row): lane t reads the row's 16-B words [q][part][t]
// (device layout [i][row][q < 8][a|b][lane < 64] of double2), sums part a and
// part b separately, and the wave's larger sum goes into one 64-bit atomic max
// (non-negative doubles order like their bit patterns).
__global__ __launch_bounds__(256) void k_row_energy_max(const double2 *__restrict__ bk, size_t rows,
                                                        unsigned long long *out) {
    const size_t r = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int t = threadIdx.x & 63;
    if (r >= rows) return;
    const double2 *row = bk + r * 1024;
    double ea = 0.0, eb = 0.0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const double2 a = row[q * 128 + t], b = row[q * 128 + 64 + t];
        ea += a.x * a.x + a.y * a.y;
        eb += b.x * b.x + b.y * b.y;
    }
    for (int o = 32; o > 0; o >>= 1) {
        ea += __shfl_xor(ea, o);
        eb += __shfl_xor(eb, o);
    }
    if (t == 0) atomicMax(out, (unsigned long long)__double_as_longlong(ea > eb ? ea : eb));
}

hipError_t launch_row_energy_max(const double *bkd, size_t rows, unsigned long long *out, hipStream_t s) {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(*out), s);
    if (e != hipSuccess || rows == 0) return e;
    hipLaunchKernelGGL(k_row_energy_max, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s,
                       reinterpret_cast<const double2 *>(bkd), rows, out);
    return hipGetLastError();
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

}  // namespace tfhe
