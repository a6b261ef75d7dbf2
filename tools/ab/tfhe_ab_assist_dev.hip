// tfhe_ab_assist_dev.hip — a development copy of the product's loader-assist whole form
// (csrc/tfhe_kernels_whole.hip, k_blind_rotate_assist) for A/B work in the A/B library only
// (tools/ab_forms.sh).  TFHE_OPT_BR_FORM 9 + VAR:
//   VAR 0  = the product kernel as is (control);
//   VAR 10 = knock-out timing build: the forward pairs skip exchange 2 altogether (wrong words;
//            what that LDS traffic is worth, profiles/r05_ab_ex2_regs.txt);
//   VAR 17 = the half-wave pair layout (round 6) for row pairs 1 and 2: one
//            wave transforms the pair as two 32-lane halves of 16 points each, ONE LDS exchange per
//            pair (half 0 through X, half 1 through Y, which the loader leaves free between the
//            gate's tB read and its fb hand-off), the last radix-2 stage over v_permlane16_swap, and
//            v_permlane32_swap hand-overs into and out of the product's MAC layout (same words);
//   VAR 18 = VAR 17 for row pair 2 only.
// The round-5 variants (row 5 on the loader, exchange 2 in registers, early counter reads,
// phase-shifted gates: VARs 1-9 and 11-16) were removed in round 6; their measurements stay in
// profiles/r05_ab_row5.txt, r05_ab_ex2_regs.txt, r05_ab_phase_shift.txt.
#include "../../zig-tfhe_amd/csrc/tfhe_device.hpp"

namespace tfhe {

constexpr int BAD_LDS_X = 512 * 16;  // per gate
constexpr int BAD_LDS_Y = 512 * 16;  // per gate (its loader's)
constexpr int BAD_LDS_AT = 1024 * 2;
constexpr int BAD_LDS_SYNC = 64;  // pub[2] done[2] fb_ready[4] tb_ready[4]
constexpr int BAD_X_AT = BR_LDS_BK + BR_LDS_TW + BR_LDS_TWIST;
constexpr int BAD_Y_AT = BAD_X_AT + BR_WAVES * BAD_LDS_X;
constexpr int BAD_AT_AT = BAD_Y_AT + BR_WAVES * BAD_LDS_Y;
constexpr int BAD_LDS_TOTAL = BAD_AT_AT + BR_WAVES * BAD_LDS_AT + BAD_LDS_SYNC;
static_assert(BAD_LDS_TOTAL <= 160 * 1024, "assist form LDS");
static_assert(BAD_X_AT % 4096 == 0 && BAD_Y_AT % 4096 == 0 && BAD_LDS_X % 4096 == 0, "gathers need 4 KB-aligned copies");

// Rotation gather of ONE polynomial, as the product's gather_rot_one.
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

// Inverse transform of ONE accumulated spectrum, as the product's inverse_one.
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

DEV void spin_short_d(const uint32_t *p, uint32_t target, uint32_t cap, uint32_t &fail) {
    uint32_t f = 0;
    spin_until_ge<1>(p, target, cap, f);
    fail |= f;
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

// ---- half-wave pair layout (VAR 17 / 18) ----------------------------------------------------
// Row pair (2rp, 2rp+1) as ONE 512-point transform per 32-lane half: half h = lane bit 5 owns row
// 2rp + h, lane j = lane & 31 owns points p = j + 32 mu (mu < 16).  In the reference's DIT
// (bitReverseRadix2 + radix2FFT, fft.zig:582-669) point p sits at position q = bitrev9(p) =
// r + 16 bitrev5(j) with r = bitrev4(mu) the register index, so:
//   pass 1 (stages len 2..16, position bits 0-3) in registers, lane-uniform twiddles;
//   ONE exchange through LDS (half 0's buffer X, half 1's Y): lane j' = c + 16 b8 then holds
//     positions c + 16 s + 256 b8, s < 16 the register;
//   pass 2 (stages len 32..256, bits 4-7) in registers, twiddles W_len[c + 16 (s mod len/32)];
//   stage len 512 (bit 8, lane bit 4): one v_permlane16_swap per dword of each register pair trades
//     bit 8 (lane) for bit 4 (register), then register butterflies with W512[j + 32 (s >> 1)].
// Output Z[j + 32 m] (m < 16).  Every butterfly is the product's (same operands, same recurrence
// twiddles, same fused arithmetic): the same spectrum bits.  The hand-overs from and to the
// product's layout (lane t = j + 32 h holds points / frequencies t + 64 q of BOTH rows) are one
// v_permlane32_swap per dword of 8 complex values each way.
// Slot swizzle of the exchange: slot = q ^ (position bits 6-8 of q), so the writes' 8-lane
// groups (bank = slot mod 8; the lanes of a group differ in position bits 6-8) are conflict-free
// and every lane's 16 write slots are 8 runtime values + compile-time offsets (8 address VGPRs,
// loop-invariant); the reads' 16-lane groups (slot mod 16) see 2-way conflicts (two quads of
// each group differ only in b8), with 4 address VGPRs.  The conflict-free-both swizzle (bit 8 also
// into slot bit 3) needs 16 + 4 address VGPRs, which spilled the kernel.
DEV int hw_slot(int q) { return q ^ ((q >> 6) & 7); }

template <bool FU>
DEV void fft_pair_halfwave(C2 (*d)[8], C2 *hbuf, const C2 *s_tw, const LdsTw &T, int t) {
    const int j = t & 31;
    C2 e[16];
    // product layout -> half-wave: after the swap, d[0][q] = row (2rp + h) at mu = 2 br3(q) and
    // d[1][q] at mu = 2 br3(q) + 1, i.e. registers r = q and r = 8 + q
#pragma unroll
    for (int q = 0; q < 8; q++) {
        swap_lane_reg<2>(d[0][q], d[1][q]);
        e[q] = d[0][q];
        e[8 + q] = d[1][q];
    }
    // pass 1: stages len 2, 4, 8 (passA) in both register halves, then len 16 across them
    passA<false, FU>(e, T.a);
    passA<false, FU>(e + 8, T.a);
    auto tw_at = [&](int idx) {  // read at the stage: an opaque pointer keeps hipcc from hoisting it
        const C2 *p = s_tw;
        asm volatile("" : "+v"(p));
        return p[idx];
    };
    __builtin_amdgcn_sched_barrier(0);
    {
        C2 w16[8];
#pragma unroll
        for (int r = 1; r < 8; r++) w16[r] = tw_at(7 + r);  // lane-uniform (broadcast reads)
        bf1<FU>(e[0], e[8]);
#pragma unroll
        for (int r = 1; r < 8; r++) bf<false, FU>(e[r], e[8 + r], w16[r]);
    }
    // the one exchange
    // hw_slot spelled out so that hipcc sees 8 write and 4 read address values per lane (the
    // rest are immediate offsets): write slot wq + 8 (r >> 3) + ((r & 7) ^ g), g = position bits
    // 6-8 = bitrev5(j) >> 2; read slot 256 b8 + 16 s + (c ^ 4 b8 ^ (s >> 2))
    const int br5 = (int)(__builtin_bitreverse32((uint32_t)j) >> 27), wq = 16 * br5, g = br5 >> 2;
#pragma unroll
    for (int r = 0; r < 16; r++) hbuf[wq + 8 * (r >> 3) + ((r & 7) ^ g)] = e[r];
    wave_sync();
    const int c = j & 15, b8 = j >> 4, x = c ^ (4 * b8);
#pragma unroll
    for (int s = 0; s < 16; s++) e[s] = hbuf[256 * b8 + 16 * s + (x ^ (s >> 2))];
    wave_sync();
    // pass 2: stages len 32, 64, 128, 256 (position bits 4-7 = register bits 0-3).  Each stage's
    // twiddles are read at the stage, behind a scheduling fence: hoisted, the 23 per-lane
    // twiddles of the pass spilled the kernel.
    {
        const C2 w = tw_at(15 + c);
#pragma unroll
        for (int s = 0; s < 16; s += 2) bf<false, FU>(e[s], e[s + 1], w);
    }
    __builtin_amdgcn_sched_barrier(0);
    {
        C2 w[2];
#pragma unroll
        for (int k = 0; k < 2; k++) w[k] = tw_at(31 + c + 16 * k);
#pragma unroll
        for (int s = 0; s < 16; s++)
            if (!(s & 2)) bf<false, FU>(e[s], e[s + 2], w[s & 1]);
    }
    __builtin_amdgcn_sched_barrier(0);
    {
        C2 w[4];
#pragma unroll
        for (int k = 0; k < 4; k++) w[k] = tw_at(63 + c + 16 * k);
#pragma unroll
        for (int s = 0; s < 16; s++)
            if (!(s & 4)) bf<false, FU>(e[s], e[s + 4], w[s & 3]);
    }
    __builtin_amdgcn_sched_barrier(0);
    {
        C2 w[8];
#pragma unroll
        for (int k = 0; k < 8; k++) w[k] = tw_at(127 + c + 16 * k);
#pragma unroll
        for (int s = 0; s < 8; s++) bf<false, FU>(e[s], e[s + 8], w[s]);
    }
    __builtin_amdgcn_sched_barrier(0);
    // stage len 512: position bit 8 (lane bit 4) <-> bit 4 (register bit 0), then in registers
#pragma unroll
    for (int s = 0; s < 16; s += 2) {
        const C2 w = tw_at(255 + j + 32 * (s >> 1));
        swap_lane_reg<1>(e[s], e[s + 1]);
        bf<false, FU>(e[s], e[s + 1], w);
    }
    __builtin_amdgcn_sched_barrier(0);
    // Z[j + 32 m]: m < 8 in e[2m], m >= 8 in e[2 (m - 8) + 1]; back to the product's layout
    // (lane t holds t + 64 q of both rows): m = 2q from half 0's lanes, 2q + 1 from half 1's
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const int m0 = 2 * q, m1 = 2 * q + 1;
        C2 x = m0 < 8 ? e[2 * m0] : e[2 * (m0 - 8) + 1];
        C2 y = m1 < 8 ? e[2 * m1] : e[2 * (m1 - 8) + 1];
        swap_lane_reg<2>(x, y);
        d[0][q] = x;
        d[1][q] = y;
    }
}

template <bool FU, int VAR>
__global__ __launch_bounds__(512, 1) void k_blind_rotate_assist_dev(
    KParams P, DevTables TT, const uint8_t *__restrict__ ops, const uint32_t *__restrict__ in_a,
    const uint32_t *__restrict__ in_b, const uint32_t *__restrict__ idx, const uint32_t *__restrict__ testvec,
    const double2 *__restrict__ bkd, uint32_t *__restrict__ out, int out_mode, size_t B) {
    constexpr int L = 3;
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
    uint32_t *s_sync = reinterpret_cast<uint32_t *>(smem + BAD_LDS_TOTAL - BAD_LDS_SYNC);
    uint32_t *fb_ready = s_sync + 4, *tb_ready = s_sync + 8;
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
        T.init(s_tw);
        const C2 *twist_t = s_twist + t;
        const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lds_void_t *)Y32);  // acc_b copy: Y[0, 4 KB)
        PhaseProf lp;  // tools/phase_prof.hip assist: 0 vmcnt + pub, 1 fb wait, 2 inverse b, 3 gather + tB, 4 refill wait + issue
        lp.start();
        for (uint32_t k = 0; k < pairs; k++) {
            lp.mark(0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of pair k landed
            counter_add(s_sync + (k & 1));
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
                const int at = __builtin_amdgcn_readfirstlane((int)s_at[i]);
                uint32_t v[16], xb[16];
                gather_rot_one_d(base, t, at, xb, v);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int m = 0; m < 16; m++) {
                    const uint32_t sg = gather_sign(xb[m]), off_s = P.offset - sg;
                    Y32[1024 + t + 64 * m] = tmp_word(v[m], sg, off_s, accB[m], msbs);
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
            lp.flush(g_phase_cycles + 16, 8);
#endif
        report_wait_failure(P, fail, DEV_ERR_LOADER_WAIT);
        if (FU && VAR != 10) near_tie_flag(P, near, g, valid);  // VAR 10: garbage values
        if (!valid) return;
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
    if (tid < 12) s_sync[tid] = 0u;
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
    // VAR 17 / 18: the half-wave exchange buffer, half 0 in X and half 1 in Y
    C2 *hbuf = (t & 32) ? Y : X;
    int at_next = s_at[0];
    uint32_t near = NEAR_NONE, fail = 0;
    PhaseProf pp;  // tools/phase_prof.hip assist: 0 gather + tmp, 1 pair 0 fft, 2 pub waits, 3 macs, 4 tB wait, 5 pairs 1-2 fft, 6 fb hand-off, 7 inverse a
    pp.start();
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
                                 (Y32[1024 + t + 64 * m] & ~((1u << P.bgbit) - 1u));
                    if (VAR == 17 || VAR == 18) wave_sync();  // tB read out of Y before the half-wave exchanges
                }
                pp.mark(5);
                load_digits_pair_tbx<FU>(d, tbx, rp, P.bgbit, twist_t);
            }
            if (VAR == 10)
                fft512_x2_noex2<false, FU>(d, X, T, t);
            else if ((VAR == 17 && rp > 0) || (VAR == 18 && rp == 2))
                fft_pair_halfwave<FU>(d, hbuf, s_tw, T, t);
            else
                fft512_x2<false, true, FU>(d, X, T, t);
            const uint32_t k = (uint32_t)(L * i + rp);
            pp.mark(2);
            wait_pair_first_group(s_sync, s_bk + (k & 1) * 2048 + t, k, spin_cap, fail, kpre);
            __builtin_amdgcn_sched_barrier(0);
            pp.mark(3);
            mac_pair_lds<FU>(fa, fb, d[0], d[1], s_bk + (k & 1) * 2048, t, kpre);
            __builtin_amdgcn_sched_barrier(0);
            counter_add(s_sync + 2 + (k & 1));
        }
        // hand fb to the loader (it read tB(i) from Y before: this wave's reads came first)
        pp.mark(6);
        if (VAR == 17 || VAR == 18) wave_sync();  // the half-wave exchange's Y reads precede fb's writes
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
        pp.flush(g_phase_cycles, 8);
#endif
    report_wait_failure(P, fail, DEV_ERR_GATE_WAIT);
    if (FU && VAR != 10) near_tie_flag(P, near, g, valid);  // VAR 10: garbage values
    if (!valid) return;
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
    case 10:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 10>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,10> (knock-out: forward exchange 2 skipped, wrong words)";
        break;
    case 17:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 17>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,17> (half-wave pair layout, row pairs 1-2)";
        break;
    case 18:
        hipLaunchKernelGGL((k_blind_rotate_assist_dev<true, 18>), grid, block, 0, s, P, T, ops, in_a, in_b, idx, testvec,
                           bk2, out, out_mode, B);
        if (used) *used = "k_blind_rotate_assist_dev<true,18> (half-wave pair layout, row pair 2)";
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace tfhe
