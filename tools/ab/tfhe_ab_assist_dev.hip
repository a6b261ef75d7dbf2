// tfhe_ab_assist_dev.hip — a development copy of the product's loader-assist whole form
// (csrc/tfhe_kernels_whole.hip, k_blind_rotate_assist) for A/B work in the A/B library only
// (tools/ab_forms.sh).  TFHE_OPT_BR_FORM 9 + VAR: VAR 0 = the product kernel as is (control),
// VAR 1 = knock-out timing build: pair 2 runs ONE forward transform (row 4) and reuses it for
// row 5 (wrong words; the upper bound of moving row 5's transform off the gate wave),
// VAR 2 = the loader wave also transforms row 5 (b's last level) from its tB words and hands
// the spectrum to the gate through Y (counters tb_read, r5_ready); same arithmetic and words;
// VAR 3 = VAR 2 with the loader's row-5 exchange 2 in registers, VAR 4 = VAR 2 with the gate's
// single row-4 transform exchanging through LDS; VAR 5 = VAR 2 with tB handed over as its top 16
// bits (the gate needs only b's levels 0 and 1) in a 2 KB area of its own, so the loader transforms
// row 5 through Y at once instead of waiting for the gate to read tB out of Y; VAR 6 = VAR 0 with
// the gate's pipelined forward pairs exchanging stage 2 in registers (fewer LDS operations);
// VAR 7 / 8 / 9: the same for pair 0 / pair 2 / pairs 1-2 only; VAR 10 = knock-out timing build:
// the forward pairs skip exchange 2 altogether (wrong words; what half the exchange traffic is worth);
// VAR 11 = VAR 0 with the slot counter and the MAC's first BK group read under the pair's last pass;
// VAR 12 = VAR 5 with pair 1's exchange 2 in registers; VAR 13 = VAR 0 with each forward pair's
// transform 0 exchanging stage 2 in registers and transform 1 through LDS; VAR 14 = knock-out
// timing build: VAR 13 with transform 0's exchange 2 skipped (wrong words); VAR 15 / 16 = VAR 0 with
// the odd gate waves started ~2 k / ~4 k cycles late (exchange bursts interleaved across gates).  (Until this fix VAR 6-10 also carried
// VAR 5's row-5 split: R5 was VAR >= 2; profiles/r05_ab_ex2_regs.txt records both.)
#include "../../zig-tfhe_amd/csrc/tfhe_device.hpp"

namespace tfhe {

constexpr int BAD_LDS_X = 512 * 16;  // per gate
constexpr int BAD_LDS_Y = 512 * 16;  // per gate (its loader's)
constexpr int BAD_LDS_AT = 768 * 2;  // a~ of n <= 768 steps (the launcher checks)
constexpr int BAD_LDS_SYNC = 128;  // pub[2] done[2] fb_ready[4] tb_ready[4] tb_read[4] r5_ready[4]
constexpr int BAD_X_AT = BR_LDS_BK + BR_LDS_TW + BR_LDS_TWIST;
constexpr int BAD_Y_AT = BAD_X_AT + BR_WAVES * BAD_LDS_X;
constexpr int BAD_AT_AT = BAD_Y_AT + BR_WAVES * BAD_LDS_Y;
constexpr int BAD_LDS_T16 = 1024 * 2;  // VAR 5: tB's top 16 bits per coefficient
constexpr int BAD_T16_AT = BAD_AT_AT + BR_WAVES * BAD_LDS_AT;
constexpr int BAD_LDS_TOTAL = BAD_T16_AT + BR_WAVES * BAD_LDS_T16 + BAD_LDS_SYNC;
static_assert(BAD_LDS_TOTAL <= 160 * 1024, "assist form LDS");
static_assert(BAD_X_AT % 4096 == 0 && BAD_Y_AT % 4096 == 0 && BAD_LDS_X % 4096 == 0, "gathers need 4 KB-aligned copies");

// Rotation gather of ONE polynomial (1,024 words at the 4 KB-aligned byte address
// `base`), as gather_rot: lane word m = coefficient t + 64m of X^a~ p, sign in bit
// 12 of xb[m].
DEV void gather_rot_one_d(uint32_t base, int t, int at, uint32_t *xb, uint32_t *v) {
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

// Inverse transform of ONE accumulated spectrum (fft1024), untwist, guarded
// conversion and the CMUX add into acc (lane-local); exchange 1 through xb,
// exchange 2 in registers (the single-transform fft512).
template <bool FU, bool EX2LDS = false>
DEV void inverse_one_d(const C2 *f, C2 *xb, const LdsTw &T, const C2 *twist_t, int t, uint32_t *acc, uint32_t &near) {
    C2 e[1][8];
#pragma unroll
    for (int q = 0; q < 8; q++) e[0][q] = f[br3(q)];
    fft512<1, true, FU, LdsTw, EX2LDS>(e, xb, T, t);
    uint32_t nq[2] = {NEAR_NONE, NEAR_NONE};
#pragma unroll
    for (int q = 0; q < 8; q++) {
        double re, im;
        untwist_out<false, FU>(e[0][q], twist_t[64 * q], re, im);
        acc[q] += to_torus<true, FU>(re, nq[0]);
        acc[q + 8] += to_torus<true, FU>(im, nq[1]);
    }
    near &= nq[0] & nq[1];
}

// Bounded poll with a short sleep (hand-offs between a gate and its loader).
// Its own SGPR flag, ORed into `fail` through a vector value (one shared "+s"
// flag across this loop's asm blocks made hipcc emit an illegal VGPR-to-SGPR copy).
DEV void spin_short_d(const uint32_t *p, uint32_t target, uint32_t cap, uint32_t &fail) {
    uint32_t f = 0;
    spin_until_ge<1>(p, target, cap, f);
    fail |= f;
}

// The pipelined transform pair of fft512_x2 (tfhe_device.hpp, one buffer) with exchange 2 in
// registers (ex2_regs: permlane swaps + DPP) instead of LDS: 16 ds_write/read_b128 fewer per
// transform for 80 VALU moves each.  Same values (pure data movement).
template <bool INV, bool FU, class TW>
DEV void fft512_x2_ex2r(C2 (*d)[8], C2 *xb, const TW &T, int t) {
    C2 wb_[7], wc_[7];
    passA<INV, FU>(d[0], T.a);
    ex1_write(d[0], xb, t);
    wave_sync();
    passA<INV, FU>(d[1], T.a);
    ex1_read(d[0], xb, t);
    ex1_write(d[1], xb, t);
    wave_sync();
    T.pass_b(wb_, t);
    passBC<INV, FU>(d[0], wb_);
    ex1_read(d[1], xb, t);
    ex2_regs(d[0]);
    passBC<INV, FU>(d[1], wb_);
    T.pass_c(wc_, t);
    ex2_regs(d[1]);
    passBC<INV, FU>(d[0], wc_);
    passBC<INV, FU>(d[1], wc_);
}

// VAR 13: fft512_x2 (one buffer) with the MAC's slot counter and first BK frequency group read
// EARLY, right behind transform 1's exchange-2 reads and before its last pass, so their LDS
// latency runs under that pass instead of in front of the MAC.  The wave's LDS operations
// execute in order, so BK words read behind a counter value that says "published" are the
// published ones; a counter that does not yet say so sends the caller to the usual wait.
template <bool INV, bool FU, class TW>
DEV void fft512_x2_early(C2 (*d)[8], C2 *xb, const TW &T, int t, const uint32_t *pubp, const double2 *slot_t,
                         uint32_t &cnt, double2 *kpre) {
    C2 wb_[7], wc_[7];
    passA<INV, FU>(d[0], T.a);
    ex1_write(d[0], xb, t);
    wave_sync();
    passA<INV, FU>(d[1], T.a);
    ex1_read(d[0], xb, t);
    ex1_write(d[1], xb, t);
    wave_sync();
    T.pass_b(wb_, t);
    passBC<INV, FU>(d[0], wb_);
    ex1_read(d[1], xb, t);
    ex2_write(d[0], xb, t);
    wave_sync();
    passBC<INV, FU>(d[1], wb_);
    T.pass_c(wc_, t);
    ex2_read(d[0], xb, t);
    ex2_write(d[1], xb, t);
    wave_sync();
    passBC<INV, FU>(d[0], wc_);
    ex2_read(d[1], xb, t);
    wave_sync();
    cnt = *(volatile const uint32_t *)pubp;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_sched_barrier(0);
    kpre[0] = slot_t[0];
    kpre[1] = slot_t[64];
    kpre[2] = slot_t[1024];
    kpre[3] = slot_t[1088];
    __builtin_amdgcn_sched_barrier(0);
    passBC<INV, FU>(d[1], wc_);
}

// VAR 13: the pair with transform 0's exchange 2 in registers and transform 1's through LDS, its
// LDS round trip running under transform 0's register moves and last pass.
template <bool INV, bool FU, class TW, bool KO = false>
DEV void fft512_x2_half(C2 (*d)[8], C2 *xb, const TW &T, int t) {
    C2 wb_[7], wc_[7];
    passA<INV, FU>(d[0], T.a);
    ex1_write(d[0], xb, t);
    wave_sync();
    passA<INV, FU>(d[1], T.a);
    ex1_read(d[0], xb, t);
    ex1_write(d[1], xb, t);
    wave_sync();
    T.pass_b(wb_, t);
    passBC<INV, FU>(d[0], wb_);
    ex1_read(d[1], xb, t);
    wave_sync();
    passBC<INV, FU>(d[1], wb_);
    ex2_write(d[1], xb, t);
    wave_sync();
    if (!KO) ex2_regs(d[0]);  // KO (VAR 14, timing only, wrong words): transform 0's exchange 2 skipped
    T.pass_c(wc_, t);
    passBC<INV, FU>(d[0], wc_);
    ex2_read(d[1], xb, t);
    wave_sync();
    passBC<INV, FU>(d[1], wc_);
}

// Knock-out (VAR 10, timing only, wrong words): the pair with exchange 2 skipped entirely.
template <bool INV, bool FU, class TW>
DEV void fft512_x2_noex2(C2 (*d)[8], C2 *xb, const TW &T, int t) {
    C2 wb_[7], wc_[7];
    passA<INV, FU>(d[0], T.a);
    ex1_write(d[0], xb, t);
    wave_sync();
    passA<INV, FU>(d[1], T.a);
    ex1_read(d[0], xb, t);
    ex1_write(d[1], xb, t);
    wave_sync();
    T.pass_b(wb_, t);
    passBC<INV, FU>(d[0], wb_);
    ex1_read(d[1], xb, t);
    passBC<INV, FU>(d[1], wb_);
    T.pass_c(wc_, t);
    passBC<INV, FU>(d[0], wc_);
    passBC<INV, FU>(d[1], wc_);
}

template <bool FU, int VAR>
__global__ __launch_bounds__(512, 1) void k_blind_rotate_assist_dev(
    KParams P, DevTables TT, const uint8_t *__restrict__ ops, const uint32_t *__restrict__ in_a,
    const uint32_t *__restrict__ in_b, const uint32_t *__restrict__ idx, const uint32_t *__restrict__ testvec,
    const double2 *__restrict__ bkd, uint32_t *__restrict__ out, int out_mode, size_t B) {
    constexpr int L = 3;
    constexpr bool R5 = (VAR >= 2 && VAR <= 5) || VAR == 12;  // the loader transforms row 5
    constexpr bool R5_EX2LDS = VAR != 3;       // its exchange 2 through LDS (3: in registers)
    constexpr bool G4_EX2LDS = VAR == 4;       // the gate's single row-4 transform: exchange 2 through LDS
    constexpr bool T16F = VAR == 5 || VAR == 12;  // tB handed over as its top 16 bits in T16 (Y free at once)
    __shared__ __attribute__((aligned(16))) unsigned char smem[BAD_LDS_TOTAL];
    const int tid = threadIdx.x;
    const int t = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool loader = w >= BR_WAVES;
    const int gi = loader ? w - BR_WAVES : w;  // the gate this wave serves
    double2 *s_bk = reinterpret_cast<double2 *>(smem);
    C2 *s_tw = reinterpret_cast<C2 *>(smem + BR_LDS_BK);
    C2 *s_twist = reinterpret_cast<C2 *>(smem + BR_LDS_BK + BR_LDS_TW);
    C2 *X = reinterpret_cast<C2 *>(smem + BAD_X_AT + gi * BAD_LDS_X);
    C2 *Y = reinterpret_cast<C2 *>(smem + BAD_Y_AT + gi * BAD_LDS_Y);
    uint32_t *X32 = reinterpret_cast<uint32_t *>(X), *Y32 = reinterpret_cast<uint32_t *>(Y);
    uint16_t *s_at = reinterpret_cast<uint16_t *>(smem + BAD_AT_AT + gi * BAD_LDS_AT);
    uint16_t *T16 = reinterpret_cast<uint16_t *>(smem + BAD_T16_AT + gi * BAD_LDS_T16);
    uint32_t *s_sync = reinterpret_cast<uint32_t *>(smem + BAD_LDS_TOTAL - BAD_LDS_SYNC);
    uint32_t *fb_ready = s_sync + 4, *tb_ready = s_sync + 8, *tb_read = s_sync + 12, *r5_ready = s_sync + 16;
    if (lds_layout_bad(smem)) {
        if (tid == 0) __hip_atomic_fetch_or(P.err, (uint32_t)DEV_ERR_LDS_LAYOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const int n = P.n;
    const size_t g_raw = (size_t)blockIdx.x * BR_WAVES + gi;
    const bool valid = g_raw < B;
    const size_t g = valid ? g_raw : B - 1;  // ragged tail: compute a copy, store nothing
    const size_t ia = idx ? idx[2 * g] : g, ib = idx ? idx[2 * g + 1] : g;
    const uint32_t *A = in_a + ia * (size_t)(n + 1);
    const uint32_t *Bv = in_b ? in_b + ib * (size_t)(n + 1) : A;
    const int op = ops ? (int)ops[g] : 255;
    const uint32_t spin_cap = P.spin_cap ? P.spin_cap : BR_SPIN_CAP_DEFAULT;
    const uint32_t msbs = digit_msbs(L, P.bgbit);
    const uint32_t pairs = (uint32_t)n * L;

    if (loader) {
        const int ltid = tid - 64 * BR_WAVES;
        __builtin_amdgcn_s_setprio(LOADER_PRIO);
        const size_t stride = (size_t)L * 2048;
        const uint32_t loader_cap = spin_cap / LOADER_SLEEP > 0 ? spin_cap / LOADER_SLEEP : 1u;
        uint32_t near = NEAR_NONE, fail = 0;
        issue_bk_pair_async(bkd, s_bk, ltid);  // pair 0 into slot 0
        // b~ of this wave's item (trgsw.zig:312), as the gate computes it
        int bt = 0;
        if (t == (n & 63)) {
            const uint32_t c = gate_combine(op, A[n], Bv[n], true);
            bt = 2048 - (int)(uint32_t)(((uint64_t)c + (1ull << 20)) >> 21);
        }
        bt = __builtin_amdgcn_readlane(bt, n & 63);
        uint32_t accB[16];
#pragma unroll
        for (int m = 0; m < 16; m++) accB[m] = rot_read(testvec + 1024, t + 64 * m, bt);
        __syncthreads();  // the gates' prologue: counters zeroed, tables and a~ in LDS
        LdsTw T;
        T.init(s_tw);  // pass-A twiddles from LDS (VGPRs): in SGPRs this loop failed to compile
        const C2 *twist_t = s_twist + t;
        const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lds_void_t *)Y32);  // acc_b copy: Y[0, 4 KB)
        PhaseProf lp;  // tools/phase_prof.hip assist: 0 vmcnt + pub, 1 fb wait, 2 inverse b, 3 gather + tB, 4 refill wait + issue
        lp.start();
        bool pre_pub = false;  // VAR 2: pair k was published inside the row-5 block
        for (uint32_t k = 0; k < pairs; k++) {
            lp.mark(0);
            if (!pre_pub) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of pair k landed
                counter_add(s_sync + (k & 1));
            }
            pre_pub = false;
            uint32_t tbw[16];  // VAR 2: step i's tB words, kept for row 5's digits
            // the b work as soon as the own gate's fb is in, before the wait for the next refill (with its
            // 96-unit sleep): 6.15 vs 6.65 ms after it
            if (k % L == 0) {
                const uint32_t i = k / L;
                if (i > 0) {  // step i - 1's b polynomial: fb from the gate, inverse, CMUX add
                    lp.mark(1);
                    spin_short_d(fb_ready + gi, i, spin_cap, fail);
                    lp.mark(2);
                    C2 f[8];
#pragma unroll
                    for (int q = 0; q < 8; q++) f[q] = Y[q * 64 + t];
                    inverse_one_d<FU, true>(f, Y, T, twist_t, t, accB, near);
                }
                lp.mark(3);
                wave_sync();  // the exchange's reads precede the copy's writes
#pragma unroll
                for (int m = 0; m < 16; m++) Y32[t + 64 * m] = accB[m];
                wave_sync();
                // step i's tB: X^{a~_i} acc_b - acc_b + offset, flipped (tmp_word)
                const int at = __builtin_amdgcn_readfirstlane((int)s_at[i]);
                uint32_t v[16], xb[16];
                gather_rot_one_d(base, t, at, xb, v);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int m = 0; m < 16; m++) {
                    const uint32_t sg = gather_sign(xb[m]), off_s = P.offset - sg;
                    tbw[m] = tmp_word(v[m], sg, off_s, accB[m], msbs);
                    if (T16F)
                        T16[t + 64 * m] = (uint16_t)(tbw[m] >> 16);
                    else
                        Y32[1024 + t + 64 * m] = tbw[m];
                }
                __builtin_amdgcn_sched_barrier(0);
                counter_add(tb_ready + gi);  // tB(i) written (the LDS runs this wave's ops in order)
                lp.mark(0);
            }
            if (k + 1 < pairs) {
                const uint32_t k1 = k + 1;
                lp.mark(4);
                spin_until_ge<LOADER_SLEEP>(s_sync + 2 + (k1 & 1), 4u * (k1 >> 1), loader_cap, fail);
                issue_bk_pair_async(bkd + (size_t)(k1 / L) * stride + (size_t)(k1 % L) * 2048, s_bk + (k1 & 1) * 2048,
                                    ltid);
                if (R5 && k % L == 0) {
                    // row 5 (b's last level) of step i: digits from the tB words, forward transform through Y
                    // once the gate has read tB out of it, spectrum handed over in Y (r5_ready); pair k + 1
                    // is published first (its DMA landed under the digits)
                    const uint32_t i = k / L;
                    C2 e[1][8];
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        const int m = br3(q);
                        e[0][q] = twist_in<FU>((double)(int32_t)__builtin_amdgcn_sbfe(tbw[m], 32 - L * P.bgbit, P.bgbit),
                                               (double)(int32_t)__builtin_amdgcn_sbfe(tbw[m + 8], 32 - L * P.bgbit, P.bgbit),
                                               twist_t[64 * m]);
                    }
                    lp.mark(6);
                    if (!T16F) spin_short_d(tb_read + gi, i + 1, spin_cap, fail);
                    lp.mark(7);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // pair k + 1's pieces landed
                    counter_add(s_sync + (k1 & 1));
                    pre_pub = true;
                    wave_sync();
                    fft512<1, false, FU, LdsTw, R5_EX2LDS>(e, Y, T, t);
                    wave_sync();  // the exchange's reads precede the spectrum's writes
#pragma unroll
                    for (int q = 0; q < 8; q++) Y[q * 64 + t] = e[0][q];
                    __builtin_amdgcn_sched_barrier(0);
                    counter_add(r5_ready + gi);
                    lp.mark(4);
                }
            }
        }
        spin_short_d(fb_ready + gi, (uint32_t)n, spin_cap, fail);  // the last step's b polynomial
        {
            C2 f[8];
#pragma unroll
            for (int q = 0; q < 8; q++) f[q] = Y[q * 64 + t];
            inverse_one_d<FU, true>(f, Y, T, twist_t, t, accB, near);
        }
        lp.mark(5);
#ifdef TFHE_PHASE_PROF
        if (t == 0)
            for (int q = 0; q < 8; q++) atomicAdd(&g_phase_cycles[16 + q], (unsigned long long)lp.acc[q]);
#endif
        report_wait_failure(P, fail, DEV_ERR_LOADER_WAIT);
        if (FU && VAR != 10 && VAR != 14) near_tie_flag(P, near, g, valid);  // VAR 10/14: garbage values
        if (!valid) return;
        // the b parts of the outputs (accB: coefficient t + 64m)
        if (out_mode == BR_OUT_LV1) {
            if (t == 0) out[g * (size_t)1025 + 1024] = accB[0];
        } else if (out_mode == BR_OUT_LV0_EXTRACT2) {
            if (t == 0) out[g * (size_t)(n + 1) + n] = accB[0];
        } else {
            uint32_t *o = out + g * (size_t)2048 + 1024;
#pragma unroll
            for (int m = 0; m < 16; m++) o[t + 64 * m] = accB[m];
        }
        return;
    }

    // ---- gate wave ----
    if (tid < 20) s_sync[tid] = 0u;
    for (int x = tid; x < 511; x += 256) s_tw[x] = TT.tw[x];
    for (int x = tid; x < 512; x += 256) s_twist[x] = TT.twist[x];
    int bt = 0;
    for (int i = t; i <= n; i += 64) {
        const uint32_t c = gate_combine(op, A[i], Bv[i], i == n);
        const uint32_t tl = (uint32_t)(((uint64_t)c + (1ull << 20)) >> 21);
        if (i < n) s_at[i] = (uint16_t)tl;
        else bt = 2048 - (int)tl;
    }
    bt = __builtin_amdgcn_readlane(bt, n & 63);
    uint32_t accA[16];
#pragma unroll
    for (int m = 0; m < 16; m++) {
        accA[m] = rot_read(testvec, t + 64 * m, bt);
        X32[t + 64 * m] = accA[m];
    }
    __syncthreads();  // tables, a~ and counters visible to every wave
    LdsTw T;
    T.init(s_tw, TT);
    const C2 *twist_t = s_twist + t;
    const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lds_void_t *)X32);  // acc_a copy: X[0, 4 KB)
    int at_next = s_at[0];
    uint32_t near = NEAR_NONE, fail = 0;
    PhaseProf pp;  // tools/phase_prof.hip assist: 0 gather + tmp, 1 pair 0 fft, 2 pub waits, 3 macs, 4 tB wait, 5 pairs 1-2 fft, 6 fb hand-off, 7 inverse a
    pp.start();
    // VAR 15 / 16: odd gate waves start ~2 k / ~4 k cycles late, so the four gates' LDS exchange
    // bursts interleave instead of coinciding (the slot protocol keeps them within two pairs)
    if (VAR == 15 && (gi & 1)) __builtin_amdgcn_s_sleep(32);
    if (VAR == 16 && (gi & 1)) __builtin_amdgcn_s_sleep(64);
    for (int i = 0; i < n; i++) {
        pp.mark(0);
        const int at = __builtin_amdgcn_readfirstlane(at_next);
        uint32_t tA[16], xb[16];
        C2 tw0[8];
        gather_rot_one_d(base, t, at, xb, tA);
#pragma unroll
        for (int q = 0; q < 8; q++) tw0[q] = twist_t[64 * br3(q)];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 16; m++) {
            const uint32_t sg = gather_sign(xb[m]), off_s = P.offset - sg;
            tA[m] = tmp_word(tA[m], sg, off_s, accA[m], msbs);
        }
        wave_sync();  // the gather's reads precede the exchanges' writes into X
        at_next = s_at[i + 1 < n ? i + 1 : i];
        C2 fa[8], fb[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            fa[q] = c2(0.0, 0.0);
            fb[q] = c2(0.0, 0.0);
        }
        uint32_t tbx[16];
#pragma unroll
        for (int rp = 0; rp < L; rp++) {
            C2 d[2][8];
            double2 kpre[4];
            if (rp == 0) {
                pp.mark(1);
                load_digits_pair0_regs<FU>(d, tA, nullptr, L, P.bgbit, tw0);  // rows 0, 1: a's levels 0, 1
            } else {
                if (rp == 1) {  // tB(i) from the loader, packed with a's level 2 (load_digits_pair_tbx)
                    pp.mark(4);
                    spin_short_d(tb_ready + gi, (uint32_t)i + 1u, spin_cap, fail);
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int m = 0; m < 16; m++)
                        tbx[m] = __builtin_amdgcn_ubfe(tA[m], 32 - L * P.bgbit, P.bgbit) |
                                 (T16F ? (uint32_t)T16[t + 64 * m] << 16 : (Y32[1024 + t + 64 * m] & ~((1u << P.bgbit) - 1u)));
                    if (R5 && !T16F) {
                        __builtin_amdgcn_sched_barrier(0);
                        counter_add(tb_read + gi);  // Y is the loader's again (this wave's reads came first)
                    }
                }
                pp.mark(5);
                if (!R5 || rp != 2) load_digits_pair_tbx<FU>(d, tbx, rp, P.bgbit, twist_t);
            }
            if (R5 && rp == 2) {  // row 4 here, row 5's spectrum from the loader
                C2 e[1][8];
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    const int m = br3(q);
                    e[0][q] = twist_in<FU>((double)(int32_t)__builtin_amdgcn_sbfe(tbx[m], 32 - 2 * P.bgbit, P.bgbit),
                                           (double)(int32_t)__builtin_amdgcn_sbfe(tbx[m + 8], 32 - 2 * P.bgbit, P.bgbit),
                                           twist_t[64 * m]);
                }
                fft512<1, false, FU, LdsTw, G4_EX2LDS>(e, X, T, t);
#pragma unroll
                for (int q = 0; q < 8; q++) d[0][q] = e[0][q];
                pp.mark(8);
                spin_short_d(r5_ready + gi, (uint32_t)i + 1u, spin_cap, fail);
                pp.mark(9);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = 0; q < 8; q++) d[1][q] = Y[q * 64 + t];
            } else if (VAR == 1 && rp == 2) {  // knock-out: row 5's transform skipped, its spectrum = row 4's (wrong words)
                C2 e[1][8];
#pragma unroll
                for (int q = 0; q < 8; q++) e[0][q] = d[0][q];
                fft512<1, false, FU>(e, X, T, t);
#pragma unroll
                for (int q = 0; q < 8; q++) d[0][q] = d[1][q] = e[0][q];
            } else {
                if (VAR == 6 || (VAR == 7 && rp == 0) || (VAR == 8 && rp == 2) || (VAR == 9 && rp > 0) ||
                    (VAR == 12 && rp == 1))
                    fft512_x2_ex2r<false, FU>(d, X, T, t);
                else if (VAR == 10)
                    fft512_x2_noex2<false, FU>(d, X, T, t);
                else if (VAR == 13)
                    fft512_x2_half<false, FU>(d, X, T, t);
                else if (VAR == 14)
                    fft512_x2_half<false, FU, LdsTw, true>(d, X, T, t);
                else if (VAR != 11)
                    fft512_x2<false, true, FU>(d, X, T, t);
            }
            const uint32_t k = (uint32_t)(L * i + rp);
            bool early_ok = false;
            if (VAR == 11 && !(R5 && rp == 2)) {
                uint32_t cnt;
                fft512_x2_early<false, FU>(d, X, T, t, s_sync + (k & 1), s_bk + (k & 1) * 2048 + t, cnt, kpre);
                early_ok = __builtin_amdgcn_readfirstlane(cnt) >= 4u * ((k >> 1) + 1u);
            }
            pp.mark(2);
            if (!early_ok) wait_pair_first_group(s_sync, s_bk + (k & 1) * 2048 + t, k, spin_cap, fail, kpre);
            __builtin_amdgcn_sched_barrier(0);
            pp.mark(3);
            mac_pair_lds<FU>(fa, fb, d[0], d[1], s_bk + (k & 1) * 2048, t, kpre);
            __builtin_amdgcn_sched_barrier(0);
            counter_add(s_sync + 2 + (k & 1));
        }
        // hand fb to the loader (it read tB(i) from Y before: this wave's reads came first)
        pp.mark(6);
#pragma unroll
        for (int q = 0; q < 8; q++) Y[q * 64 + t] = fb[q];
        __builtin_amdgcn_sched_barrier(0);
        counter_add(fb_ready + gi);
        pp.mark(7);
        inverse_one_d<FU, false>(fa, X, T, twist_t, t, accA, near);
        wave_sync();
#pragma unroll
        for (int m = 0; m < 16; m++) X32[t + 64 * m] = accA[m];
        wave_sync();
    }
    pp.mark(0);
#ifdef TFHE_PHASE_PROF
    if (t == 0)
        for (int q = 0; q < 10; q++) atomicAdd(&g_phase_cycles[q], (unsigned long long)pp.acc[q]);
#endif
    report_wait_failure(P, fail, DEV_ERR_GATE_WAIT);
    if (FU && VAR != 10 && VAR != 14) near_tie_flag(P, near, g, valid);  // VAR 10/14: garbage values
    if (!valid) return;
    // the a parts of the outputs from the acc_a copy (the loader writes b's)
    if (out_mode == BR_OUT_LV1) {  // sampleExtractIndex(acc, 0): p[0] = a[0], p[j] = -a[N-j]; p[N] = b[0]: loader
        uint32_t *o = out + g * (size_t)1025;
        for (int j = t; j < 1024; j += 64) o[j] = j == 0 ? X32[0] : 0u - X32[1024 - j];
    } else if (out_mode == BR_OUT_LV0_EXTRACT2) {  // sampleExtractIndex2 (trlwe.zig:165-180)
        uint32_t *o = out + g * (size_t)(n + 1);
        for (int j = t; j < n; j += 64) o[j] = j == 0 ? X32[0] : 0u - X32[n - j];
    } else {
        uint32_t *o = out + g * (size_t)2048;
        for (int j = t; j < 1024; j += 64) o[j] = X32[j];
    }
}


hipError_t ab_launch_assist_dev(int var, dim3 grid, dim3 block, hipStream_t s, const KParams &P, const DevTables &T,
                                const uint8_t *ops, const uint32_t *in_a, const uint32_t *in_b, const uint32_t *idx,
                                const uint32_t *testvec, const double2 *bk2, uint32_t *out, int out_mode, size_t B,
                                const char **used) {
    if (P.n > BAD_LDS_AT / 2) return hipErrorInvalidValue;
    switch (var) {
    case 0:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 0>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,0> (A/B copy of the assist form)";
        break;
    case 2:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 2>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,2> (loader also transforms row 5)";
        break;
    case 3:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 3>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,3> (row 5 on the loader, its exchange 2 in registers)";
        break;
    case 4:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 4>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,4> (row 5 on the loader, gate row 4 exchange 2 in LDS)";
        break;
    case 5:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 5>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,5> (row 5 on the loader, tB's top half in its own LDS area)";
        break;
    case 6:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 6>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,6> (forward pairs: exchange 2 in registers)";
        break;
    case 7:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 7>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,7> (exchange 2 in registers: pair 0)";
        break;
    case 8:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 8>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,8> (exchange 2 in registers: pair 2)";
        break;
    case 9:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 9>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,9> (exchange 2 in registers: pairs 1-2)";
        break;
    case 10:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 10>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,10> (knock-out: forward exchange 2 skipped, wrong words)";
        break;
    case 11:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 11>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,11> (slot counter + first BK group read under the last pass)";
        break;
    case 12:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 12>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,12> (row 5 on the loader as VAR 5, pair 1 exchange 2 in registers)";
        break;
    case 13:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 13>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,13> (forward pairs: one exchange 2 in registers, one in LDS)";
        break;
    case 14:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 14>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,14> (knock-out: one exchange 2 per forward pair skipped, wrong words)";
        break;
    case 15:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 15>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,15> (odd gates start ~2 k cycles late)";
        break;
    case 16:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 16>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,16> (odd gates start ~4 k cycles late)";
        break;
    case 1:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 1>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,1> (knock-out: row 5 transform skipped, wrong words)";
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace tfhe
