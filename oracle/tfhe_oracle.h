/*
 * tfhe_oracle.h — CPU restatement of zig-tfhe's gate-bootstrap path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: a literal C restatement
 * of the reference's arithmetic (file:line cited per function in tfhe_oracle.c).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it, and only as the checker / CPU baseline — never as the product path.
 *
 * Parity status: the reference is Zig and no Zig toolchain exists in this
 * image, so the reference binary cannot be run here.  The reference ships no
 * bit-level golden vectors for this path.  The oracle is pinned against the
 * reference's own known-answer and semantic tests (polyMulWithXK k=0/1/N,
 * sample-extract b-coefficient, decomposition offset, FFT round-trip/poly_mul
 * tolerance vs the naive product, gate truth tables, 402+304=706), see
 * tests/test_oracle.py.  Bit patterns of the f64 FFT path are therefore pinned
 * to this restatement + glibc 2.35 twiddles, "parity unpinned" vs the Zig
 * binary itself.
 */
#ifndef TFHE_ORACLE_H
#define TFHE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    uint32_t n;        /* TLWE lv0 dimension        params.zig TlweParams.n      */
    uint32_t N;        /* TRLWE polynomial size     params.zig TrgswParams.n     */
    uint32_t nbit;     /* log2(N)                   TrgswParams.nbit             */
    uint32_t L;        /* gadget levels             TrgswParams.l                */
    uint32_t bgbit;    /* log2(Bg)                  TrgswParams.bgbit            */
    uint32_t basebit;  /* key-switch base bits      TrgswParams.basebit          */
    uint32_t iks_t;    /* key-switch levels         TrgswParams.iks_t            */
    uint32_t _pad;
    double alpha_lv0;  /* TLWE lv0 encryption noise tlwe_lv0.alpha               */
    double alpha_lv1;  /* TRLWE/TLWE lv1 noise      trlwe_lv1.alpha              */
    double alpha_ksk;  /* KSK_ALPHA                 params.zig:419-420           */
    double alpha_bsk;  /* BSK_ALPHA                 params.zig:421-422           */
} oracle_params;

/* ---- RNG (restates Zig std.Random.DefaultPrng = Xoshiro256, SplitMix64 seed) */
typedef struct { uint64_t s[4]; } oracle_rng;
void     oracle_rng_init(oracle_rng *r, uint64_t seed);
uint64_t oracle_rng_next(oracle_rng *r);
uint32_t oracle_rng_u32(oracle_rng *r);
int      oracle_rng_bool(oracle_rng *r);
double   oracle_rng_f64(oracle_rng *r);

/* ---- torus utils (utils.zig) */
uint32_t oracle_f64_to_torus(double d);
double   oracle_torus_to_f64(uint32_t t);

/* ---- FFT (fft.zig KlemsaProcessor) */
void oracle_twist_table(uint32_t N, double *re, double *im);               /* N/2 each */
void oracle_stage_twiddles(uint32_t N, int inverse, double *re, double *im);/* N/2-1 each: stage len=2..N/2, w_j j<len/2 */
void oracle_ifft(uint32_t N, const uint32_t *in, double *out);   /* torus -> freq (forward, "ifft") */
void oracle_fft(uint32_t N, const double *in, uint32_t *out);    /* freq -> torus (inverse, "fft")  */
void oracle_poly_mul(uint32_t N, const uint32_t *a, const uint32_t *b, uint32_t *out);
void oracle_poly_mul_naive(uint32_t N, const uint32_t *a, const uint32_t *b, uint32_t *out);

/* ---- TRGSW / TRLWE primitives (trgsw.zig, trlwe.zig) */
uint32_t oracle_decomposition_offset(const oracle_params *p);
void oracle_decomposition(const oracle_params *p, const uint32_t *trlwe /*2N*/, uint32_t offset,
                          uint32_t *dec /*2L*N*/);
void oracle_poly_mul_with_xk(uint32_t N, const uint32_t *a, uint32_t k, uint32_t *out);
void oracle_external_product(const oracle_params *p, const double *trgsw_fft /*2L*2*N*/,
                             const uint32_t *trlwe /*2N*/, uint32_t offset, uint32_t *out /*2N*/);
void oracle_cmux(const oracle_params *p, const uint32_t *in1, const uint32_t *in2,
                 const double *trgsw_fft, uint32_t offset, uint32_t *out);
void oracle_blind_rotate(const oracle_params *p, const uint32_t *tlwe_lv0 /*n+1*/,
                         const uint32_t *testvec /*2N*/, const double *bk, uint32_t offset,
                         uint32_t *out /*2N*/);
void oracle_sample_extract_index(uint32_t N, const uint32_t *trlwe, uint32_t k, uint32_t *out /*N+1*/);
void oracle_sample_extract_index2(uint32_t n, uint32_t N, const uint32_t *trlwe, uint32_t k,
                                  uint32_t *out /*n+1*/);
void oracle_identity_key_switch(const oracle_params *p, const uint32_t *tlwe_lv1 /*N+1*/,
                                const uint32_t *ksk, uint32_t *out /*n+1*/);

/* ---- bootstrap / gates (bootstrap/vanilla.zig, gates.zig) */
void oracle_bootstrap(const oracle_params *p, const uint32_t *in /*n+1*/, const uint32_t *testvec,
                      const double *bk, const uint32_t *ksk, uint32_t offset, uint32_t *out /*n+1*/);
void oracle_bootstrap_without_key_switch(const oracle_params *p, const uint32_t *in /*n+1*/,
                                         const uint32_t *testvec, const double *bk, uint32_t offset,
                                         uint32_t *out /*n+1*/);
/* op codes: see include/tfhe_gpu.h TFHE_GATE_* (same numbering) */
void oracle_gate_combine(const oracle_params *p, int op, const uint32_t *a, const uint32_t *b,
                         uint32_t *out /*n+1*/);
void oracle_gate(const oracle_params *p, int op, const uint32_t *a, const uint32_t *b,
                 const uint32_t *testvec, const double *bk, const uint32_t *ksk, uint32_t offset,
                 uint32_t *out);
/* batch over B items with `threads` std threads (0 = 1); used only as CPU baseline */
void oracle_gate_batch(const oracle_params *p, int threads, size_t B, const uint8_t *ops,
                       const uint32_t *a, const uint32_t *b, const uint32_t *testvec,
                       const double *bk, const uint32_t *ksk, uint32_t offset, uint32_t *out);

/* ---- keys and encryption (key.zig, tlwe.zig, trlwe.zig, trgsw.zig) */
void oracle_secret_key_new(const oracle_params *p, uint64_t seed, uint32_t *key_lv0, uint32_t *key_lv1);
void oracle_testvec(const oracle_params *p, uint32_t *testvec /*2N*/);
/* master RNG seeded with `seed` supplies every getUniqueSeed() of CloudKey.new */
void oracle_cloud_key_new(const oracle_params *p, uint64_t seed, const uint32_t *key_lv0,
                          const uint32_t *key_lv1, uint32_t *ksk, double *bk);
void oracle_tlwe_encrypt_f64(uint32_t n, double mu, double alpha, const uint32_t *key, uint64_t seed,
                             uint32_t *out /*n+1*/);
int  oracle_tlwe_decrypt_bool(uint32_t n, const uint32_t *ct, const uint32_t *key);
uint32_t oracle_tlwe_phase(uint32_t n, const uint32_t *ct, const uint32_t *key);
void oracle_trlwe_encrypt_f64(const oracle_params *p, const double *mu /*N*/, double alpha,
                              const uint32_t *key_lv1, uint64_t seed, uint32_t *out /*2N*/);
void oracle_trlwe_decrypt_bool(const oracle_params *p, const uint32_t *ct, const uint32_t *key_lv1,
                               uint8_t *out /*N*/);
void oracle_trgsw_encrypt_torus_fft(const oracle_params *p, uint32_t mu, double alpha,
                                    const uint32_t *key_lv1, oracle_rng *master, double *out /*2L*2N*/);

/* ---- programmable bootstrap (lut generator/encoder, trgsw.zig:336-400) */
void oracle_lut_generate(uint32_t N, uint32_t message_modulus, const uint32_t *f_table /*m*/,
                         uint32_t *testvec /*2N*/);
void oracle_lut_generate_scaled(uint32_t N, uint32_t m, double scale, const uint32_t *f_table, uint32_t *tv);
void oracle_lut_generate_full(uint32_t N, uint32_t m, const uint32_t *values, uint32_t *tv);
size_t oracle_div_round(size_t a, size_t b);
size_t oracle_lut_mod_switch(uint32_t x, size_t size);
void oracle_tlwe_encrypt_lwe_message(uint32_t n, uint32_t msg, uint32_t m, double alpha,
                                     const uint32_t *key, uint64_t seed, uint32_t *out);
uint32_t oracle_tlwe_decrypt_lwe_message(uint32_t n, const uint32_t *ct, uint32_t m, const uint32_t *key);

/* ---- proxy re-encryption (proxy_reenc.zig) -------------------------- */
/* reencryptTLWELv0 :267-306 — key: n*t*2^basebit rows of n+1 words */
void oracle_reencrypt(uint32_t n, uint32_t basebit, uint32_t t, const uint32_t *ct /*n+1*/,
                      const uint32_t *key, uint32_t *out /*n+1*/);
/* PublicKeyLv0.newWithParams :57-76 — encryption e uses seed seed0+e */
void oracle_public_key_gen(uint32_t n, const uint32_t *key, size_t size, double alpha, uint64_t seed0,
                           uint32_t *pk /*size*(n+1)*/);
/* PublicKeyLv0.encryptF64 :83-113 */
void oracle_public_key_encrypt_f64(uint32_t n, const uint32_t *pk, size_t size, double plaintext, double alpha,
                                   uint64_t seed, uint32_t *out /*n+1*/);
/* ProxyReencryptionKey.new{Symmetric,Asymmetric}WithParams :150-256; pk == NULL selects the
 * symmetric form (key_to used); the c-th encryption in (i, j, k) order uses seed0+c */
void oracle_reenc_key_gen(uint32_t n, const uint32_t *key_from, const uint32_t *key_to, const uint32_t *pk,
                          size_t pk_size, double alpha, uint32_t basebit, uint32_t t, uint64_t seed0,
                          uint32_t *out);

/* cos/sin source of the FFT twiddles: 0 = glibc (default), 1 = the
 * fdlibm/musl kernels Zig's compiler_rt ports. */
void oracle_set_trig_source(int source);
int oracle_get_trig_source(void);
double oracle_trig_cos(double x, int source);
double oracle_trig_sin(double x, int source);
/* 0 = reference expression trees (default); 1 = fused multiply-adds (the
 * MI355X kernels' form at the L=3 / Bg=2^6 sets) */
void oracle_set_fused(int fused);
void oracle_set_regroup(int mode);  /* fused mode: 1 = (rows of a) + (rows of b) (pair/duo forms), 2 = per-row terms summed (latency forms) */
int oracle_get_fused(void);
void oracle_set_fold(int fold);  /* fused mode: forward transforms with the folded twist (evidence only) */
void oracle_folded_twiddles(uint32_t N, double *re, double *im);
/* max |x - round(x)| rounded by oracle_fft on this thread since the last call (then reset) */
double oracle_take_round_error(void);
/* Start capturing the inverse transforms' pre-rounding values into buf (pairs
 * (re_i, im_i) per coefficient i < N/2; NULL stops); returns the count captured
 * by the previous capture. */
size_t oracle_capture_rounded(double *buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif
