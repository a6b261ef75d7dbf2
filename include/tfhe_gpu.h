/*
 * tfhe_gpu.h — C ABI of the MI355X TFHE gate-bootstrap engine.
 *
 * This is the drop-in boundary for zig-tfhe's bootstrap strategy plug point
 * (src/bootstrap.zig:30-47, src/bootstrap/vanilla.zig:38-69, callers
 * src/gates.zig:48-129).  A Zig `bootstrap/hip.zig` strategy would declare
 * these functions `extern fn` and map a negative status to a Zig error
 * (INTEGRATION.md shows the binding).  Plain pointers and sizes only; the
 * library owns all device memory; one context = one HIP device (+ one stream).
 *
 * Layouts are the reference's in-memory layouts:
 *   TLWELv0      = uint32_t[n+1]            (tlwe.zig:11-12, b is the last word)
 *   TLWELv1      = uint32_t[N+1]            (tlwe.zig:243-244)
 *   TRLWELv1     = uint32_t[2][N]  a then b (trlwe.zig:15-17)
 *   BootstrappingKey  = double[n][2L][2][N] (key.zig:31, trgsw.zig:75-77,
 *                        trlwe.zig:104-106: each N = re[N/2] ++ im[N/2])
 *   KeySwitchingKey   = uint32_t[N*t*2^basebit][n+1]  (key.zig:28, :148-172)
 * Status: 0 = OK, negative = error (tfhe_gpu_last_error has the text).
 * Calls on one context are serialised by the caller (as the reference's
 * single-threaded Gates); distinct contexts are independent.
 */
#ifndef TFHE_GPU_H
#define TFHE_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TFHE_GPU_ABI_VERSION 7  /* 7: tfhe_gpu_set_stream(NULL) = the null stream, tfhe_gpu_reset_stream;
                                   6: tfhe_gpu_build_kind, tfhe_lut_generate_scaled / _full; BR forms 6-40
                                   A/B-only, BR_LOADER / BR_SYNC = 1 only;
                                   5: _dev LUT / re-encryption / circuit entries; BR forms 2 and 4 removed */

enum {
    TFHE_OK = 0,
    TFHE_ERR_INVALID = -1,     /* bad argument / unsupported parameter set      */
    TFHE_ERR_HIP = -2,         /* HIP runtime error (no device, launch failure) */
    TFHE_ERR_NO_KEY = -3,      /* bootstrap requested before a cloud key loaded */
    TFHE_ERR_OOM = -4,         /* device allocation failed                      */
    TFHE_ERR_IO = -5,          /* key file cannot be opened, read or written    */
    TFHE_ERR_DEVICE = -6       /* a kernel reported a failure through the context's device
                                  error word (the blind rotation's BK-slot protocol: a wait
                                  timed out); the outputs since the last synchronisation are
                                  invalid; the word is cleared and the context stays usable */
};

/* Gate op codes — gates.zig:48-121 (pre-combination constants SURVEY §8a A2). */
enum {
    TFHE_GATE_NAND = 0, TFHE_GATE_OR = 1, TFHE_GATE_AND = 2, TFHE_GATE_XOR = 3,
    TFHE_GATE_XNOR = 4, TFHE_GATE_NOR = 5, TFHE_GATE_ANDNY = 6, TFHE_GATE_ANDYN = 7,
    TFHE_GATE_ORNY = 8, TFHE_GATE_ORYN = 9,
    TFHE_GATE_NOT = 254,       /* circuits only: negation, no bootstrap (gates.zig:132-135) */
    TFHE_GATE_COPY = 255       /* no pre-combination: bootstrap input a as is */
};

/* Runtime form of params.zig SecurityParams (:36-67).  N must be 1024. */
typedef struct {
    uint32_t n;        /* TLWE lv0 dimension (tlwe_lv0.n)   */
    uint32_t N;        /* polynomial size (trgsw_lv1.n)     */
    uint32_t nbit;     /* log2 N                             */
    uint32_t L;        /* gadget levels                      */
    uint32_t bgbit;    /* log2 Bg                            */
    uint32_t basebit;  /* key-switch base bits               */
    uint32_t iks_t;    /* key-switch levels                  */
    uint32_t _pad;
    double alpha_lv0;  /* tlwe_lv0.alpha                     */
    double alpha_lv1;  /* trlwe_lv1.alpha                    */
    double alpha_ksk;  /* KSK_ALPHA (params.zig:419-420)     */
    double alpha_bsk;  /* BSK_ALPHA (params.zig:421-422)     */
} tfhe_params;

typedef struct tfhe_gpu_ctx tfhe_gpu_ctx;

int         tfhe_gpu_abi_version(void);
/* TFHE_BUILD_PRODUCT for the product library; TFHE_BUILD_AB for a development
 * build (knock-out, timing or losing-form variants: tools/ab_forms.sh,
 * tools/libvar_build.sh, a Makefile EXTRA), which every tfhe_gpu_create*
 * refuses (TFHE_ERR_INVALID) unless the environment sets
 * TFHE_ALLOW_AB_BUILD=1.  (ABI 6) */
enum { TFHE_BUILD_PRODUCT = 0, TFHE_BUILD_AB = 1 };
int         tfhe_gpu_build_kind(void);
/* 16 hex digits of the sha256 of the kernels object this library was linked
 * from (its gfx950 code): measurements (PMC records) are tagged with it. */
const char *tfhe_gpu_build_id(void);
/* Context over HIP devices 0..num_devices-1 of this node:
 * num_devices = 1 is a plain single-device context on device 0, more is the
 * multi-device context of tfhe_gpu_create_multi below.  Replaces the implicit
 * per-thread FFT plan (fft.zig:983-992) and owns the device copy of the
 * CloudKey.  TFHE_ERR_HIP if the node has fewer devices. */
int         tfhe_gpu_create(const tfhe_params *params, int num_devices, tfhe_gpu_ctx **out);
/* Context on the one HIP device `device` (ABI 2's tfhe_gpu_create). */
int         tfhe_gpu_create_on_device(const tfhe_params *params, int device, tfhe_gpu_ctx **out);
void        tfhe_gpu_destroy(tfhe_gpu_ctx *ctx);
/* Text of the context's last failure; with ctx = NULL, the calling thread's
 * last failed tfhe_gpu_create / _create_on_device / _create_multi (ABI 4). */
const char *tfhe_gpu_last_error(const tfhe_gpu_ctx *ctx);
/* Wait for the context's work; TFHE_ERR_DEVICE if a kernel set the device
 * error word since the last synchronisation.  Every host-buffer entry point
 * performs the same check before it returns; after the asynchronous _dev
 * entry points, this (or tfhe_gpu_profile_end) is where a failure surfaces. */
int         tfhe_gpu_sync(tfhe_gpu_ctx *ctx);
/* Run this context's work on a caller-owned hipStream_t of its device; NULL is
 * that device's null stream (torch's default stream has handle 0).  The new
 * stream first waits for everything queued on the old one.  (ABI 7: before,
 * NULL meant the context's own stream, so torch's default stream silently got
 * an unordered non-blocking stream.)  Multi-device context: its first device. */
int         tfhe_gpu_set_stream(tfhe_gpu_ctx *ctx, void *hip_stream);
/* Back to the context's own (non-blocking) stream, ordered after the current one.  (ABI 7) */
int         tfhe_gpu_reset_stream(tfhe_gpu_ctx *ctx);

/* ---- Multi-device context (bootstrap.zig:30-47 strategy over
 * the 8 GPUs of one node) ---------------------------------------------------
 * One context over `num_devices` HIP devices (`devices` = their ids, NULL =
 * 0..num_devices-1).  Key loads (load_cloud_key, keygen, the key file and
 * device-blob imports) land on the first device and are broadcast once to
 * the others with ncclBroadcast over RCCL (xGMI; librccl is loaded at that
 * point); a device listed twice (a test of the sharding on one GPU) gets a
 * device-to-device copy instead.  The host-buffer batch entry points
 * (bootstrap / gate / blind-rotate / LUT / key-switch / re-encryption) split
 * the batch into contiguous slices of ceil(B/num_devices) items, one per
 * device, run them concurrently (one host thread and one stream per device)
 * and copy each slice's results into the caller's buffer; circuit_eval
 * replicates the primary inputs to every device that reads them and places
 * the connected components of the gate DAG (gates joined by gate-to-gate
 * wires) on the devices, largest first onto the least-loaded device, so no
 * gate output crosses a device; when one component dominates it splits every
 * level's gates over the devices instead and all-gathers each level's outputs
 * (peer copies over xGMI) before the next (TFHE_OPT_CIRCUIT_SPLIT).  Device-pointer
 * (_dev) and stage entry points and the profile timers use the first device.
 * Nothing is exchanged between devices after the key broadcast. */
/* Distinct devices must reach each other's memory: create_multi checks
 * hipDeviceCanAccessPeer for every ordered pair and enables peer access (the
 * level split's peer copies then go over xGMI, not through the host); a pair
 * without it fails the create with TFHE_ERR_DEVICE and the pair named in
 * tfhe_gpu_last_error(NULL).  A device id the node does not have fails with
 * TFHE_ERR_HIP. */
int tfhe_gpu_create_multi(const tfhe_params *params, int num_devices, const int *devices, tfhe_gpu_ctx **out);
int tfhe_gpu_num_devices(const tfhe_gpu_ctx *ctx);
/* 64-bit fingerprints of the resident device key (BK and KSK in the device
 * layout; the order-independent k_checksum sum, ~35 us each), the values the
 * multi-device broadcast compares.  Processes that import a broadcast key
 * (tfhe_gpu_import_key_device) compare them across ranks (tfhe_dist.py).
 * TFHE_ERR_NO_KEY without a key.  (ABI 4) */
int tfhe_gpu_key_fingerprint(tfhe_gpu_ctx *ctx, uint64_t *bk, uint64_t *ksk);
/* Blind rotations each device of the context has launched since it was
 * created (counts[d] for device d < max_devices, in create order); returns the
 * number of devices.  Shows where a sharded batch or circuit ran. */
int tfhe_gpu_device_bootstraps(const tfhe_gpu_ctx *ctx, uint64_t *counts, int max_devices);
/* Items whose blind rotation the fused arithmetic's margin guard sent to the
 * reference-tree recompute since the context was created (a value 1/4 or
 * more off its integer), as of the last synchronisation. */
int tfhe_gpu_near_tie_items(const tfhe_gpu_ctx *ctx, uint64_t *count);

/* ---- Options (kernel forms and table sources; default = the measured-
 * fastest forms).  Set on a context before use; a multi-device context
 * passes them to every device.  TFHE_ERR_INVALID for an unknown key or value. */
enum {
    TFHE_OPT_BR_FORM = 1,         /* blind rotation: 0 auto (default), 1 whole, 3 latency, 5 octo (8 items
                                     per workgroup, two gate waves per SIMD; L = 1 only).  2 split and 4
                                     pair were removed in round 4; 6 duo, 7 the split-transform latency
                                     form, 8 round 4's whole form and 9-40 development copies of the L = 3
                                     whole form (all measured slower) exist
                                     only in A/B libraries since round 5 (tools/ab/): TFHE_ERR_INVALID here */
    TFHE_OPT_BR_LOADER = 2,       /* whole form: 1 loader waves issue the BK DMAs (the only value since
                                     round 5; 0, the gate waves issuing them, was removed) */
    TFHE_OPT_KS_FORM = 3,         /* key switch: 3 auto (default: the one-hot GEMM on the matrix
                                     cores for basebit 2 and 5, else lanes), 0 lanes / ring,
                                     1 select / gather, 2 the GEMM at any batch (basebit 2; other
                                     parameter sets fall back to lanes) */
    TFHE_OPT_KS_NARROW = 4,       /* basebit 2: 0 auto (default), 1 32-word x 4-wave blocks */
    TFHE_OPT_KS_ITEM_GROUPS = 5,  /* basebit >= 5: 0 auto (above 64 items the ring form: 4 item groups
                                     share a 4-deep DMA ring), 1, 2, 4, 8 forces the lane form with
                                     that many item groups per block */
    TFHE_OPT_KS_SEL_ITEMS = 6,    /* select / gather form: items per block, 8 (default), 16, 32 */
    TFHE_OPT_CIRCUIT_PACK = 7,    /* circuit_eval round packing: 1 (default), 0 off */
    TFHE_OPT_TWIDDLES = 8,        /* cos/sin source of the FFT tables: TFHE_TWIDDLES_* (set before a key
                                     is generated: keygen transforms the key with these tables) */
    TFHE_OPT_ARITH = 9,           /* blind-rotation f64 arithmetic: TFHE_ARITH_* */
    TFHE_OPT_BR_SYNC = 10,        /* whole form: 1 per-slot LDS counters (gate waves wait for their data,
                                     not for each other; the only value since round 5: 0, a workgroup
                                     barrier per BK row pair, was removed) */
    TFHE_OPT_BR_SPIN_CAP = 11,    /* polls before one slot-counter wait gives up and sets the device
                                     error word (0 = default, 2^22 sleep units; fault-injection tests
                                     set a few polls to see TFHE_ERR_DEVICE come back) */
    TFHE_OPT_HOST_PIPELINE = 12,  /* host-buffer bootstrap / gate / LUT batches of >= 4 x #CUs items:
                                     0 (default) one H2D -> kernels -> D2H sequence, 1 chunked through
                                     pinned staging on 4 streams (measured slower on the MI355X box,
                                     whose pageable copies run at ~50 GB/s: DESIGN.md §2.1) */
    TFHE_OPT_CIRCUIT_SPLIT = 13,  /* multi-device circuit_eval: 0 auto (default: connected components
                                     on devices, or by levels when one component dominates), 1
                                     components, 2 levels (each level's gates split over the devices,
                                     outputs all-gathered by peer copies before the next level) */
    TFHE_OPT_FUSED_ADMITTED = 14, /* read-only (get_option): 1 if the resident cloud key passed the fused
                                     arithmetic's admission check at load (largest BK spectrum component
                                     <= 2^39 and every TRGSW row's RMS <= 0.65 x 2^31), 0
                                     if it was refused and TFHE_ARITH_AUTO runs the reference's expression
                                     trees for it */
    TFHE_OPT_LEVEL_ISSUE_US = 15, /* read-only: host microseconds the last level-split circuit_eval spent
                                     issuing its per-level launches, peer copies and event waits (one
                                     host thread for all devices) */
    TFHE_OPT_KEY_ROW_RMS_PPM = 16, /* read-only: the resident key's largest TRGSW row RMS / 2^31, in
                                     millionths (the admission's row-energy rule admits <= 650000;
                                     keygen'd keys ~600000; ABI 6) */
    TFHE_OPT_HOST_STAGING = 17    /* host-buffer copies: 0 pageable hipMemcpyAsync from / to the caller's buffers
                                     (default), 1 through per-device pinned staging (host memcpy + DMA).  Same
                                     words either way.  Measured: 8 concurrent shards'
                                     pageable copies 52.9 GB/s in total against 47.2 staged, and the one-card
                                     8-shard step 54.5 vs 56.6 ms, so staging is for hosts whose pageable
                                     copies serialise */
};
enum { TFHE_STAGING_PAGEABLE = 0, TFHE_STAGING_PINNED = 1 };  /* TFHE_OPT_HOST_STAGING */
/* TFHE_ARITH_AUTO (default): at the L=3 / Bg=2^6 sets the blind rotation
 * runs fused multiply-adds in the reference's operation order, with a margin
 * guard: every value it rounds must lie within 1/4 of an integer; an item
 * that rounded anything further off is recomputed in the reference's
 * expression trees in the same stream (tfhe_gpu_near_tie_items counts them).
 * Both round to the same integers while the fused and the reference's values
 * differ by less than 1/4: an EMPIRICAL bound (measured max 0.094 on keygen'd
 * keys), so a key is admitted to the fused arithmetic only
 * when its BK lies in the measured regime (TFHE_OPT_FUSED_ADMITTED); other
 * keys run the reference's trees.  UINT4: the reference's trees.
 * TFHE_ARITH_REFERENCE: the reference's expression trees everywhere.
 * TFHE_ARITH_FUSED_FORCED: fused (with the guard) even on a refused key —
 * for tests of the margin guard only. */
enum { TFHE_ARITH_AUTO = 0, TFHE_ARITH_REFERENCE = 1, TFHE_ARITH_FUSED_FORCED = 2 };
/* The two libm candidates a Zig build of the reference can bind @cos/@sin to
 * (fft.zig:98-106, :591-593): glibc (linkLibC on Linux) or Zig's compiler_rt
 * port of the fdlibm/musl kernels.  DESIGN.md §6 lists the entries where the
 * two tables differ. */
enum { TFHE_TWIDDLES_GLIBC = 0, TFHE_TWIDDLES_FDLIBM = 1 };
int tfhe_gpu_set_option(tfhe_gpu_ctx *ctx, int key, int64_t value);
int tfhe_gpu_get_option(const tfhe_gpu_ctx *ctx, int key, int64_t *value);
/* Names of the kernels the last bootstrap launch of this context ran
 * ("<blind rotation> + <key switch>"; first device of a multi-device context). */
const char *tfhe_gpu_last_kernels(tfhe_gpu_ctx *ctx);
/* The FFT constant tables for N (twist N/2 entries, forward stage twiddles
 * N/2-1 entries, fft.zig:92-106 and :590-616) from `source`; host only. */
int tfhe_fft_tables(uint32_t N, int source, double *twist_re, double *twist_im, double *stage_re,
                    double *stage_im);

/* ---- Cloud key (key.zig:61-118) -------------------------------------- */
/* Upload a CloudKey held in host memory in the reference layout
 * (CloudKey.decomposition_offset, .blind_rotate_testvec, .bootstrapping_key
 * .items, .key_switching_key.items).  bsk_len / ksk_len are element counts. */
int tfhe_gpu_load_cloud_key(tfhe_gpu_ctx *ctx, uint32_t decomposition_offset,
                            const uint32_t *testvec_a, const uint32_t *testvec_b,
                            const double *bsk, size_t bsk_len,
                            const uint32_t *ksk, size_t ksk_len);
/* Generate SecretKey.new (key.zig:41-57) + CloudKey.new (key.zig:70-77) with
 * a seeded RNG (Zig DefaultPrng restated; `seed` replaces getUniqueSeed()),
 * FFTs on the device, and load it.  key_lv0/key_lv1 receive the secret key
 * (n / N words); bsk_out / ksk_out (may be NULL) receive the host copy in the
 * reference layout. */
int tfhe_gpu_keygen(tfhe_gpu_ctx *ctx, uint64_t secret_seed, uint64_t cloud_seed,
                    uint32_t *key_lv0, uint32_t *key_lv1, double *bsk_out, uint32_t *ksk_out);
/* Device-resident key blob, for the one-time RCCL broadcast across ranks:
 * export copies the context's device key into caller device buffers of the
 * reported sizes; import loads a blob another context exported. */
int tfhe_gpu_key_blob_bytes(const tfhe_gpu_ctx *ctx, size_t *bsk_bytes, size_t *ksk_bytes);
int tfhe_gpu_export_key_device(tfhe_gpu_ctx *ctx, void *bsk_dev, void *ksk_dev,
                               uint32_t *decomposition_offset, uint32_t *testvec /*2N host*/);
int tfhe_gpu_import_key_device(tfhe_gpu_ctx *ctx, const void *bsk_dev, const void *ksk_dev,
                               uint32_t decomposition_offset, const uint32_t *testvec /*2N host*/);
/* The loaded CloudKey back in the reference's host layout (the inverse of
 * tfhe_gpu_load_cloud_key; bsk: n*2L*2*N doubles, ksk: N*t*2^basebit*(n+1)
 * words, the never-read k = 0 slots as zeros).  NULL outputs are skipped. */
int tfhe_gpu_export_cloud_key(tfhe_gpu_ctx *ctx, uint32_t *decomposition_offset, uint32_t *testvec_a,
                              uint32_t *testvec_b, double *bsk, uint32_t *ksk);

/* ---- Cloud-key files (SURVEY §5 checkpoint row, §8f N3) -----------------
 * The reference has no key serialization: every process regenerates its
 * CloudKey (key.zig:70-77, ~30 s on a CPU).  A key file is a 64-byte header
 * {char magic[8] = "ZTFHECK1"; u32 version = 1, n, N, L, bgbit, basebit,
 * iks_t, decomposition_offset; u64 bsk_len, ksk_len, checksum} followed by
 * testvec a (N u32), testvec b (N u32), the BootstrappingKey (bsk_len f64)
 * and the KeySwitchingKey (ksk_len u32), all little-endian in the layouts
 * above.  checksum = FNV-1a-64 over the four sections in 8-byte words.
 * Reading checks the magic, the parameter set against `params` and the
 * checksum (TFHE_ERR_INVALID); TFHE_ERR_IO: cannot open, short read/write. */
int tfhe_cloud_key_write(const char *path, const tfhe_params *params, uint32_t decomposition_offset,
                         const uint32_t *testvec_a, const uint32_t *testvec_b, const double *bsk, size_t bsk_len,
                         const uint32_t *ksk, size_t ksk_len);
int tfhe_cloud_key_read(const char *path, const tfhe_params *params, uint32_t *decomposition_offset,
                        uint32_t *testvec_a, uint32_t *testvec_b, double *bsk, size_t bsk_len, uint32_t *ksk,
                        size_t ksk_len);
/* Export + write, and read + load, for a context (host memory for one key). */
int tfhe_gpu_save_cloud_key(tfhe_gpu_ctx *ctx, const char *path);
int tfhe_gpu_load_cloud_key_file(tfhe_gpu_ctx *ctx, const char *path);

/* ---- Bootstrap / gates (host buffers, synchronous) ---------------------- */
/* VanillaBootstrap.bootstrap (vanilla.zig:38-52) over B TLWELv0. */
int tfhe_gpu_bootstrap_batch(tfhe_gpu_ctx *ctx, const uint32_t *in, uint32_t *out, size_t B);
/* VanillaBootstrap.bootstrapWithoutKeySwitch (vanilla.zig:58-69): blind
 * rotation + sampleExtractIndex2(acc, 0) (trlwe.zig:165-180), n+1 words per
 * item in the reference's hybrid form (p[0]=a[0], p[i]=-a[n-i], p[n]=b[0]). */
int tfhe_gpu_bootstrap_without_key_switch_batch(tfhe_gpu_ctx *ctx, const uint32_t *in, uint32_t *out,
                                                size_t B);
/* Gates.*Gate (gates.zig:48-121): per-item op + pre-combination + bootstrap. */
int tfhe_gpu_gate_batch(tfhe_gpu_ctx *ctx, const uint8_t *ops, const uint32_t *a,
                        const uint32_t *b, uint32_t *out, size_t B);
/* trgsw.blindRotate (trgsw.zig:290-333) / blindRotateWithTestvec (:336-400):
 * testvec = NULL uses the cloud key's; out = B TRLWELv1. */
int tfhe_gpu_blind_rotate_batch(tfhe_gpu_ctx *ctx, const uint32_t *in, const uint32_t *testvec,
                                uint32_t *trlwe_out, size_t B);
/* Programmable bootstrap: blindRotateWithTestvec + sampleExtractIndex(0) +
 * identityKeySwitching with a LUT test vector (lut/generator.zig:85-135). */
int tfhe_gpu_bootstrap_lut_batch(tfhe_gpu_ctx *ctx, const uint32_t *in, const uint32_t *testvec,
                                 uint32_t *out, size_t B);

/* ---- Circuits: level-scheduled gate DAG ----------------
 * Replaces gate-by-gate evaluation of a circuit (examples/add_two_numbers.zig:
 * 24-73, Gates.muxNaive gates.zig:124-129).  Wires 0..n_inputs-1 are the
 * inputs (TLWELv0 each); gate g drives wire n_inputs+g from wires in_a[g],
 * in_b[g] (both < n_inputs+g; in_b ignored for NOT/COPY).  ops: TFHE_GATE_*
 * (bootstrapped) or TFHE_GATE_NOT (free).  Each dependency level is one
 * batched bootstrap launch; every wire stays in HBM.  Gates with slack may
 * run one level later than their earliest level when that avoids a ragged
 * partial round (depth unchanged; TFHE_OPT_CIRCUIT_PACK = 0 disables it).
 * outputs receives the n_outputs wires out_wires[]; *levels (may be NULL)
 * the bootstrap depth. */
int tfhe_gpu_circuit_eval(tfhe_gpu_ctx *ctx, size_t n_inputs, const uint32_t *inputs, size_t n_gates,
                          const uint8_t *ops, const uint32_t *in_a, const uint32_t *in_b, size_t n_outputs,
                          const uint32_t *out_wires, uint32_t *outputs, uint32_t *levels);
/* The same with the inputs and outputs in HBM (the circuit itself, ops / in_a /
 * in_b / out_wires, stays a host description), single-device contexts, async on
 * the context stream (tfhe_gpu_sync reports device errors). */
int tfhe_gpu_circuit_eval_dev(tfhe_gpu_ctx *ctx, size_t n_inputs, const uint32_t *inputs_dev, size_t n_gates,
                              const uint8_t *ops, const uint32_t *in_a, const uint32_t *in_b, size_t n_outputs,
                              const uint32_t *out_wires, uint32_t *outputs_dev, uint32_t *levels);

/* The schedule tfhe_gpu_circuit_eval runs, host only (no device): levels[g]
 * = the level gate g runs at (NOT: the level of its input), *depth (may be
 * NULL) = the bootstrap depth, for a device with `cus` compute units (256 on
 * the MI355X), with round packing when pack != 0. */
int tfhe_circuit_schedule(size_t n_inputs, size_t n_gates, const uint8_t *ops, const uint32_t *in_a,
                          const uint32_t *in_b, uint32_t cus, int pack, uint32_t *levels, uint32_t *depth);

/* The device placement a multi-device tfhe_gpu_circuit_eval uses, host only:
 * device_of_gate[g] < num_devices.  Gates joined by gate-to-gate wires share a
 * device; primary inputs are replicated and join nothing. */
int tfhe_circuit_partition(size_t n_inputs, size_t n_gates, const uint8_t *ops, const uint32_t *in_a,
                           const uint32_t *in_b, int num_devices, uint32_t *device_of_gate);

/* ---- Proxy re-encryption (proxy_reenc.zig) -------------
 * reencryptTLWELv0 is the identity key switch over a TLWELv0 input (n
 * coefficients instead of N), so it runs on the same lane-per-item kernel.
 * The key is ProxyReencryptionKey.key_encryptions: n*t*2^basebit TLWELv0 at
 * index (2^basebit*t*i) + (2^basebit*j) + k (proxy_reenc.zig:150-196). */
typedef struct tfhe_gpu_reenc_key tfhe_gpu_reenc_key;
int  tfhe_gpu_reenc_key_load(tfhe_gpu_ctx *ctx, const uint32_t *key_encryptions, size_t len /* words */,
                             uint32_t basebit, uint32_t t, tfhe_gpu_reenc_key **out);
void tfhe_gpu_reenc_key_destroy(tfhe_gpu_reenc_key *key);
int  tfhe_gpu_reencrypt_batch(tfhe_gpu_ctx *ctx, const tfhe_gpu_reenc_key *key, const uint32_t *in,
                              uint32_t *out, size_t B);

/* ---- Same, on device-resident buffers (async on the context stream) ---- */
int tfhe_gpu_gate_batch_dev(tfhe_gpu_ctx *ctx, const uint8_t *ops_dev, const uint32_t *a_dev,
                            const uint32_t *b_dev, uint32_t *out_dev, size_t B);
int tfhe_gpu_bootstrap_batch_dev(tfhe_gpu_ctx *ctx, const uint32_t *in_dev, uint32_t *out_dev,
                                 size_t B);
/* tfhe_gpu_bootstrap_lut_batch on device buffers (the test vector too: 2N
 * words of a TRLWE), single-device contexts (TFHE_ERR_INVALID on a multi-device one). */
int tfhe_gpu_bootstrap_lut_batch_dev(tfhe_gpu_ctx *ctx, const uint32_t *in_dev, const uint32_t *testvec_dev,
                                     uint32_t *out_dev, size_t B);
/* tfhe_gpu_reencrypt_batch on device buffers (B TLWELv0 of n + 1 words each),
 * single-device contexts; replaces the same reencryptTLWELv0 loop
 * (proxy_reenc.zig:267-306) without the PCIe copies. */
int tfhe_gpu_reencrypt_batch_dev(tfhe_gpu_ctx *ctx, const tfhe_gpu_reenc_key *key, const uint32_t *in_dev,
                                 uint32_t *out_dev, size_t B);

/* ---- Device timing (HIP events on the context stream, around each kernel) */
/* Between begin and end every bootstrap launch records events around its
 * blind-rotation and key-switch kernels; end synchronises and returns the
 * summed kernel milliseconds and the number of bootstrap launches. */
int tfhe_gpu_profile_begin(tfhe_gpu_ctx *ctx);
int tfhe_gpu_profile_end(tfhe_gpu_ctx *ctx, double *blind_rotate_ms, double *key_switch_ms,
                         int *launches);

/* ---- Stage entry points (parity tests; same kernels as the path) ------- */
/* KlemsaProcessor.ifft1024 (fft.zig:293-366): B×N u32 -> B×N f64. */
int tfhe_gpu_fft_forward_batch(tfhe_gpu_ctx *ctx, const uint32_t *in, double *out, size_t B);
/* KlemsaProcessor.fft1024 (fft.zig:370-443): B×N f64 -> B×N u32. */
int tfhe_gpu_fft_inverse_batch(tfhe_gpu_ctx *ctx, const double *in, uint32_t *out, size_t B);
/* KlemsaProcessor.poly_mul (fft.zig:458-492): B pairs. */
int tfhe_gpu_poly_mul_batch(tfhe_gpu_ctx *ctx, const uint32_t *a, const uint32_t *b,
                            uint32_t *out, size_t B);
/* trgsw.externalProductWithFft (trgsw.zig:111-154) against BK row `bk_index`
 * of the loaded key (or `trgsw_fft` = one TRGSWLv1FFT, 2L*2*N doubles, if non-NULL). */
int tfhe_gpu_external_product_batch(tfhe_gpu_ctx *ctx, const double *trgsw_fft, uint32_t bk_index,
                                    const uint32_t *trlwe_in, uint32_t *trlwe_out, size_t B);
/* trgsw.identityKeySwitching (trgsw.zig:471-502): B TLWELv1 -> B TLWELv0. */
int tfhe_gpu_key_switch_batch(tfhe_gpu_ctx *ctx, const uint32_t *in_lv1, uint32_t *out_lv0, size_t B);

/* ---- Host-side TLWELv0 helpers (no device needed) ---------------------- */
/* SecretKey.new (key.zig:41-57) from DefaultPrng(seed): n lv0 bits, then N lv1 bits. */
int tfhe_secret_key_new(const tfhe_params *params, uint64_t seed, uint32_t *key_lv0, uint32_t *key_lv1);
/* TLWELv0.encryptBool (tlwe.zig:52-55 -> encryptF64 :34-49); item i uses
 * DefaultPrng(seed0 + i) in place of getUniqueSeed(). */
int tfhe_encrypt_bool_batch(const tfhe_params *params, const uint32_t *key_lv0, const uint8_t *bits,
                            uint64_t seed0, uint32_t *out, size_t B);
/* TLWELv0.decryptBool (tlwe.zig:58-68). */
int tfhe_decrypt_bool_batch(const tfhe_params *params, const uint32_t *key_lv0, const uint32_t *ct,
                            uint8_t *bits, size_t B);
/* encryptLweMessage / decryptLweMessage (tlwe.zig:74-117), message modulus m. */
int tfhe_encrypt_lwe_message_batch(const tfhe_params *params, const uint32_t *key_lv0,
                                   const uint32_t *msgs, uint32_t m, uint64_t seed0, uint32_t *out,
                                   size_t B);
int tfhe_decrypt_lwe_message_batch(const tfhe_params *params, const uint32_t *key_lv0,
                                   const uint32_t *ct, uint32_t m, uint32_t *msgs, size_t B);
/* Proxy re-encryption key material (host, seeded; the reference's
 * getUniqueSeed() for the k-th encryptF64 call of a routine becomes seed0 + k).
 * PublicKeyLv0.newWithParams (proxy_reenc.zig:57-76): `size` encryptions of 0. */
int tfhe_public_key_gen(const tfhe_params *params, const uint32_t *key_lv0, size_t size, double alpha,
                        uint64_t seed0, uint32_t *pk /* size*(n+1) */);
/* PublicKeyLv0.encryptBool (proxy_reenc.zig:83-120), one DefaultPrng(seed0 + i) per item. */
int tfhe_public_key_encrypt_bool_batch(const tfhe_params *params, const uint32_t *pk, size_t pk_size,
                                       const uint8_t *bits, double alpha, uint64_t seed0, uint32_t *out,
                                       size_t B);
/* ProxyReencryptionKey.newSymmetricWithParams (:214-256) / newAsymmetricWithParams
 * (:150-196); out: n*t*2^basebit*(n+1) words, k = 0 entries zero. */
int tfhe_reenc_key_gen_symmetric(const tfhe_params *params, const uint32_t *key_from, const uint32_t *key_to,
                                 double alpha, uint32_t basebit, uint32_t t, uint64_t seed0, uint32_t *out);
int tfhe_reenc_key_gen_asymmetric(const tfhe_params *params, const uint32_t *key_from, const uint32_t *pk,
                                  size_t pk_size, double alpha, uint32_t basebit, uint32_t t, uint64_t seed0,
                                  uint32_t *out);
/* Generator.generateLookupTableAssign (lut/generator.zig:85-135): testvec
 * (2N words, a = 0) for f given as a table f_table[x], x < m, encoded by
 * Encoder.new(m) (scale 1/(2m), encoder.zig:29-42).  1 <= m <= TFHE_LUT_MAX_M
 * (TFHE_ERR_INVALID outside; m > N leaves some messages' ranges empty, as the
 * reference's divRound ranges do).  testvec must hold 2N words. */
#define TFHE_LUT_MAX_M (1u << 24)
int tfhe_lut_generate(const tfhe_params *params, uint32_t m, const uint32_t *f_table,
                      uint32_t *testvec);
/* The same with Encoder.withScale(m, scale) (Generator.withScale, generateLookupTableCustom;
 * generator.zig:47-56, :202-213).  (ABI 6) */
int tfhe_lut_generate_scaled(const tfhe_params *params, uint32_t m, double scale, const uint32_t *f_table,
                             uint32_t *testvec);
/* generateLookupTableFull (generator.zig:144-191): values[x] is message x's Torus value as is.  (ABI 6) */
int tfhe_lut_generate_full(const tfhe_params *params, uint32_t m, const uint32_t *values, uint32_t *testvec);

#ifdef __cplusplus
}
#endif
#endif /* TFHE_GPU_H */
