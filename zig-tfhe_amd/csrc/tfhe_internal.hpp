// tfhe_internal.hpp — shared declarations between the C-ABI host layer
// (tfhe_gpu.cpp) and the HIP kernels (tfhe_kernels.hip).  Not installed.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace tfhe {

struct C2 {
    double x, y;
};

// Device-side parameter block passed by value to every kernel.
struct KParams {
    int n;          // lv0 dimension
    int N;          // 1024
    int L;          // gadget levels
    int bgbit;      // log2 Bg
    int basebit;    // key-switch base bits
    int iks_t;      // key-switch levels
    uint32_t offset;  // decomposition offset (key.zig:121-131)
    int ks_stride;    // words per device KSK row: n+1 rounded up to 4 (16-B aligned rows)
    // Device error word of the context (sticky, OR of DEV_ERR_* bits; the host
    // reads it at every synchronisation point and fails the call, never
    // returning TFHE_OK over the words of a broken launch).  err[1] counts the
    // items the margin guard's recompute redid (cumulative).
    uint32_t *err;
    uint32_t spin_cap;  // polls before a slot-counter wait gives up (TFHE_OPT_BR_SPIN_CAP; 0 = default)
    // Near-tie flags of the fused arithmetic's margin guard,
    // one byte per item of a blind-rotation launch, all zero between launches:
    // a fused kernel sets tie_flags[g] when item g rounded a value 1/4 or more off
    // its integer (within 1/4 of a tie); the reference-tree recompute launched
    // after it (fallback = 1) redoes the flagged items' workgroups and clears
    // their flags.  Sound while |v_fused - v_reference| < 1/4: measured max 0.094
    // on keygen'd keys, an empirical bound; keys outside that regime are refused
    // the fused arithmetic at load (key admission).
    uint8_t *tie_flags;
    int fallback;
};

// Bits of the device error word.
enum DevErr : uint32_t {
    DEV_ERR_GATE_WAIT = 1u,    // a gate wave's wait for a published BK slot timed out
    DEV_ERR_LOADER_WAIT = 2u,  // a loader wave's wait for a retired BK slot timed out
    DEV_ERR_LDS_LAYOUT = 4u,   // the blind rotation's LDS array is not at address 0 (gather_rot)
};
// Default bound of one slot-counter wait (sleep units).
constexpr uint32_t BR_SPIN_CAP_DEFAULT = 1u << 22;

// Device KSK: the reference's rows [(2^basebit*t*i) + 2^basebit*j + k] of
// n+1 words (key.zig:148-172), each padded to ks_stride words, plus a tail of
// KS_TAIL_WORDS zero words so chunked 16-B loads of the last row stay inside.
constexpr int KS_TAIL_WORDS = 64;
inline int ks_stride_for(int n) { return (n + 1 + 3) & ~3; }

// Output forms of the blind-rotation kernel.
enum BrOut : int {
    BR_OUT_LV1 = 0,    // sampleExtractIndex(acc, 0): TLWELv1, N+1 words per item
    BR_OUT_TRLWE = 1,  // the accumulator itself: TRLWELv1, 2N words per item
    // sampleExtractIndex2(acc, 0) (trlwe.zig:165-180), n+1 words per item: the
    // reference loops i < tlwe_lv0.N, so p[0] = a[0], p[i] = -a[n-i] (0<i<n), p[n] = b[0]
    BR_OUT_LV0_EXTRACT2 = 2,
};

// Device constant tables uploaded once per context (host_tables in tfhe_gpu.cpp).
struct DevTables {
    const C2 *twist;  // N/2 twisting factors exp(i*pi*k/N)        fft.zig:92-106
    const C2 *tw;     // N/2-1 forward stage twiddles (recurrence)  fft.zig:590-616
    C2 twa[4];        // tw[2], tw[4], tw[5], tw[6]: the lane-uniform pass-A twiddles, by value (SGPRs)
};

// Kernel-form choices of one context (tfhe_gpu_set_option, include/tfhe_gpu.h
// TFHE_OPT_*).  The defaults are the measured-fastest forms; the others stay
// for A/B runs and parity tests.  `used` (may be NULL) receives the name of
// the kernel a launcher ran.
struct LaunchOpts {
    int br_form = 0;     // 0 auto, 1 whole, 3 latency (wide), 5 octo (L = 1); 6 duo, 7 wide2 (A/B libraries only)
    int ks_form = 3;     // 0 lanes, 1 select / gather, 2 one-hot GEMM on the matrix cores (basebit 2), 3 auto
    int ks_narrow = 0;   // basebit 2: 1 forces the 32-word x 4-wave blocks
    int ks_groups = 0;   // basebit >= 5: item groups per block (0 auto = 4; 1, 2, 4, 8)
    int ks_sel_items = 8;  // select/gather form: items per block (8, 16, 32)
    int arith_strict = 0;  // 1: the reference's f64 expression trees even where fused multiply-adds round
                           // to the same integers (the L=3 / Bg=2^6 sets); 2: fused even on
                           // a key the admission check refused (margin-guard tests only)
    int key_fused_ok = 1;  // the resident BK passed the fused arithmetic's admission check
};
// The fused arithmetic runs unless the reference's trees are requested, and only on
// an admitted key unless forced (TFHE_OPT_ARITH, LaunchOpts::key_fused_ok).
inline bool fused_allowed(const LaunchOpts &O) {
    return O.arith_strict == 2 || (O.arith_strict == 0 && O.key_fused_ok != 0);
}

// An A/B build (any -D define that changes the kernels or their timing:
// tools/ab_forms.sh, tools/libvar_build.sh, tools/phase_prof.hip, a Makefile
// EXTRA) compiles every unit with TFHE_AB_BUILD; tfhe_gpu_create refuses such a
// library unless TFHE_ALLOW_AB_BUILD=1 is set (tfhe_gpu_build_kind).
#if defined(TFHE_PHASE_PROF) && !defined(TFHE_AB_BUILD)
#define TFHE_AB_BUILD 1
#endif
bool kernels_ab_build();  // tfhe_kernels.hip: this unit was compiled as an A/B build
// The A/B-only blind-rotation forms (TFHE_OPT_BR_FORM 6, 7) are linked in
// (tools/ab/tfhe_ab_forms.hip), i.e. this is an A/B library.
bool ab_forms_linked();

// ---- launchers (tfhe_kernels.hip); all asynchronous on `s` --------------
// idx: NULL, or B pairs (a, b) of ciphertext indices into in_a / in_b (circuit gather)
// The default whole-form kernels (k_blind_rotate<L, true, true, true, true>), built in their
// own unit with the max-memory-clause scheduler (tfhe_kernels_whole.hip).
hipError_t launch_whole_default(int L, dim3 grid, dim3 block, hipStream_t s, const KParams &P, const DevTables &T,
                                const uint8_t *ops, const uint32_t *in_a, const uint32_t *in_b, const uint32_t *idx,
                                const uint32_t *testvec, const double2 *bk2, uint32_t *out, int out_mode, size_t B);
hipError_t launch_blind_rotate(const KParams &P, const DevTables &T, const uint8_t *ops,
                               const uint32_t *in_a, const uint32_t *in_b, const uint32_t *idx,
                               const uint32_t *testvec, const double *bkd, uint32_t *out,
                               int out_mode, size_t B, hipStream_t s, const LaunchOpts &O = LaunchOpts(),
                               const char **used = nullptr);
// CUs of the current device (256 when it cannot be queried) and
// launch_blind_rotate's modelled time for B items on `cus` CUs, in whole-form
// rounds of 4 x cus items (the circuit scheduler's level packing)
size_t device_cus();
double blind_rotate_cost(size_t B, size_t cus, int L = 3);
// dst[k] = (negate ? -1 : 1) * src[idx[k]] for k < count, n+1 words each
// (TLWELv0.neg: gates.zig:132-135)
hipError_t launch_tlwe_gather(const KParams &P, const uint32_t *src, const uint32_t *idx, uint32_t *dst,
                              size_t count, bool negate, hipStream_t s);
// The gemm form's device buffers: the MFMA-layout KSK
// (ks_gemm_bytes) and the K splits' partial sums (ks_gemm_part_bytes(B)).
struct KsGemm {
    const uint32_t *kg = nullptr;
    uint32_t *part = nullptr;
};
// n_in: input coefficients (1024 for the identity key switch, n for a proxy
// re-encryption key); t levels of basebit 2 (t 7..9) or 5 (t 2, 3)
size_t ks_gemm_bytes(const KParams &P, int n_in, int t, int basebit);
size_t ks_gemm_part_bytes(const KParams &P, size_t B, int n_in, int basebit);
bool ks_gemm_supported(const KParams &P);
bool ks_gemm_supported(int t, int basebit);
bool ks_gemm_auto(int t, int basebit);
extern size_t KS_GEMM_MIN_ITEMS;
constexpr size_t KS_GEMM_INPUT_SLACK = 16;  // bytes past the last input row the gemm form may read
hipError_t launch_ksk_to_gemm(const KParams &P, const uint32_t *ksk, uint32_t *kg, int n_in, int t, int basebit,
                              hipStream_t s);
hipError_t launch_key_switch(const KParams &P, const uint32_t *lv1, const uint32_t *ksk,
                             uint32_t *out, size_t B, hipStream_t s, const LaunchOpts &O = LaunchOpts(),
                             const char **used = nullptr, const KsGemm *G = nullptr);
// zero the k = 0 rows (never read by the reference; the kernels subtract them unconditionally)
hipError_t launch_ksk_zero_k0(const KParams &P, uint32_t *ksk, hipStream_t s);
// same for a key-switch-shaped key over n_in input coefficients (proxy re-encryption key)
hipError_t launch_key_zero_k0(const KParams &P, uint32_t *key, int n_in, int t, int basebit, hipStream_t s);
// reencryptTLWELv0 (proxy_reenc.zig:267-306): key-switch-shaped key of n*t*2^basebit
// rows in the padded device layout; in/out B TLWELv0
hipError_t launch_reencrypt(const KParams &P, int t, int basebit, const uint32_t *in, const uint32_t *key,
                            uint32_t *out, size_t B, hipStream_t s, const LaunchOpts &O = LaunchOpts(),
                            const char **used = nullptr, const KsGemm *G = nullptr);
bool reencrypt_supported(int t, int basebit);
hipError_t launch_fft_forward(const DevTables &T, const uint32_t *in, double *out, size_t B,
                              hipStream_t s);
hipError_t launch_fft_inverse(const DevTables &T, const double *in, uint32_t *out, size_t B,
                              hipStream_t s);
// b_stride: words between consecutive b polynomials (0 = one b for all items)
hipError_t launch_poly_mul(const DevTables &T, const uint32_t *a, const uint32_t *b, size_t b_stride,
                           uint32_t *out, size_t B, hipStream_t s);
hipError_t launch_external_product(const KParams &P, const DevTables &T, const double *bkd_row,
                                   const uint32_t *in, uint32_t *out, size_t B, hipStream_t s);
// reference BK layout [n][2L][2][N] -> device layout [n][2L][8][64] x {a_re,a_im,b_re,b_im}
hipError_t launch_bk_permute(const KParams &P, const double *bk_ref, double *bkd, size_t rows,
                             hipStream_t s);
// 64-bit fingerprint of bytes (a multiple of 16) at p into *out (device), async
hipError_t launch_checksum(const void *p, size_t bytes, unsigned long long *out, hipStream_t s);
hipError_t launch_absmax(const double *p, size_t count, unsigned long long *out, hipStream_t s);
// largest spectrum energy of one TRGSW row part (re^2 + im^2 over its N/2 values) over
// `rows` device-layout BK rows (n * 2L), into *out (device, double bits), async
hipError_t launch_row_energy_max(const double *bkd, size_t rows, unsigned long long *out, hipStream_t s);
hipError_t launch_bk_unpermute(const KParams &P, const double *bkd, double *bk_ref, size_t rows,
                               hipStream_t s);

}  // namespace tfhe
