// tfhe_gpu.cpp — C-ABI implementation (include/tfhe_gpu.h): contexts, device
// key residency, batch entry points and seeded key generation.  Host code;
// all bootstrap arithmetic runs in tfhe_kernels.hip.
#include "tfhe_gpu.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types and prototypes only: librccl is dlopen'ed on first multi-device key load

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <new>
#include <vector>

#include "host_math.hpp"
#include "tfhe_internal.hpp"

using namespace tfhe;

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
};

// Persistent host workers of one context (the host-buffer pipeline's staging
// copies and its per-stream enqueueing): run(n, f) calls
// f(0..n-1) on n workers (n <= size) and returns when all are done.
class WorkerPool {
  public:
    explicit WorkerPool(int n) {
        for (int i = 0; i < n; i++) th_.emplace_back([this, i] { loop(i); });
    }
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (std::thread &t : th_) t.join();
    }
    int size() const { return (int)th_.size(); }
    void run(int n, const std::function<void(int)> &f) {
        std::unique_lock<std::mutex> g(m_);
        job_ = &f;
        active_ = n;
        pending_ = n;
        gen_++;
        cv_.notify_all();
        done_.wait(g, [this] { return pending_ == 0; });
        job_ = nullptr;
    }

  private:
    void loop(int i) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)> *f = nullptr;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return stop_ || (gen_ != seen && i < active_); });
                if (stop_) return;
                seen = gen_;
                f = job_;
            }
            (*f)(i);
            std::lock_guard<std::mutex> g(m_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)> *job_ = nullptr;
    int active_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

constexpr int PIPE_STREAMS = 4;  // concurrent chunks of the host-buffer pipeline (HIP's 4 hardware queues)

struct tfhe_gpu_ctx {
    tfhe_params P{};
    KParams K{};
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    hipEvent_t stream_ev = nullptr;  // tfhe_gpu_set_stream: the old stream's work, waited for by the new one
    std::string err;
    // device error word (KParams::err; DEV_ERR_* bits) and its pinned host copy,
    // read at every synchronisation point (sync_check); words 2-3 of both hold
    // a key fingerprint (key_fingerprint)
    uint32_t *d_err = nullptr;
    uint32_t *h_err = nullptr;
    // constant tables
    C2 *d_twist = nullptr, *d_tw = nullptr;
    C2 twa[4] = {};  // host copy of the pass-A twiddles (DevTables::twa)
    // cloud key
    bool has_key = false;
    uint32_t offset = 0;
    std::vector<uint32_t> testvec;  // host copy, 2N
    uint32_t *d_testvec = nullptr;  // cloud testvec (2N)
    double *d_bk = nullptr;         // device layout, n*2L*512 double4
    uint32_t *d_ksk = nullptr;      // reference rows padded to K.ks_stride words (ksk_dev_bytes)
    size_t bk_bytes = 0, ksk_bytes = 0;
    // scratch, grown on demand
    DevBuf s_a, s_b, s_out, s_lv1, s_ops, s_tv, s_tmp;
    DevBuf s_wires, s_cidx, s_cops;  // circuit evaluator: wire table, gather indices, op codes
    DevBuf s_ties;                   // near-tie flags (KParams::tie_flags), one byte per item, zero between launches
    DevBuf s_kspart;                 // gemm key switch: the K splits' partial sums
    uint32_t *d_ksk_gemm = nullptr;  // gemm key switch: the MFMA-layout KSK (ks_gemm_bytes), built from d_ksk
    bool ksk_gemm_ok = false;        // d_ksk_gemm matches d_ksk
    // device timing (tfhe_gpu_profile_begin/end): 3 events per bootstrap launch
    bool profiling = false;
    std::vector<hipEvent_t> events;
    size_t ev_used = 0;
    // kernel-form options (tfhe_gpu_set_option) and what the last launch ran
    LaunchOpts opts{};
    int64_t circuit_pack = 1;
    int64_t circuit_split = 0;  // TFHE_OPT_CIRCUIT_SPLIT
    int64_t twiddle_source = TFHE_TWIDDLES_GLIBC;
    bool key_from_keygen = false;  // the resident BK was transformed with this context's tables
    double bk_absmax = 0.0;        // largest |BK spectrum component| of the resident key, reference scale
    double bk_row_rms = 0.0;       // largest TRGSW row RMS / 2^31 of the resident key (by Parseval)
    int64_t level_issue_us = 0;    // host time the last level-split circuit spent issuing (TFHE_OPT_LEVEL_ISSUE_US)
    uint64_t near_tie_items = 0;   // items the margin guard recomputed (device err[1], read by sync_check)
    const char *last_br = "", *last_ks = "";
    std::string last_kernels;
    // multi-device context (tfhe_gpu_create_multi): shards[0] is this context
    // (device devices[0]); shards[k > 0] are owned single-device contexts.
    // Empty for a single-device context.
    std::vector<tfhe_gpu_ctx *> shards;
    bool distinct_devices = true;    // RCCL needs each device once; else D2D copies
    // blind rotations launched on this device since creation (tfhe_gpu_device_bootstraps)
    uint64_t bootstraps = 0;
    // host-buffer pipeline (pipelined_bootstrap): streams, pinned staging, workers
    hipStream_t pipe[PIPE_STREAMS] = {};
    hipEvent_t pipe_ev = nullptr;
    char *pin_in = nullptr, *pin_out = nullptr;
    size_t pin_in_bytes = 0, pin_out_bytes = 0;
    std::unique_ptr<WorkerPool> workers;
    int64_t pipeline = 0;  // TFHE_OPT_HOST_PIPELINE (off by default: measured slower)
    // host-buffer copies through pinned staging (TFHE_OPT_HOST_STAGING; h2d / d2h_sync): the
    // arena's bytes in use since the last synchronisation of this context's stream
    int64_t host_staging = TFHE_STAGING_PAGEABLE;
    char *stage_in = nullptr, *stage_out = nullptr;
    size_t stage_in_bytes = 0, stage_out_bytes = 0, stage_used = 0;
    std::vector<ncclComm_t> comms;   // one communicator per shard, created on the first key broadcast
};

namespace {

int fail(tfhe_gpu_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    return code;
}

// the calling thread's last failed create (tfhe_gpu_last_error(NULL))
thread_local std::string g_create_error;
static int create_fail(int code, const std::string &msg) {
    g_create_error = msg;
    return code;
}

int hip_fail(tfhe_gpu_ctx *c, hipError_t e, const char *where) {
    return fail(c, TFHE_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

#define HIPCHK(c, expr)                                         \
    do {                                                        \
        hipError_t _e = (expr);                                 \
        if (_e != hipSuccess) return hip_fail((c), _e, #expr);  \
    } while (0)

bool params_ok(const tfhe_params *p, std::string &why) {
    if (!p) { why = "params is NULL"; return false; }
    if (p->N != 1024 || p->nbit != 10) { why = "only N=1024 (nbit=10) is supported"; return false; }
    if (p->n == 0 || p->n > 1024) { why = "n must be in [1, 1024]"; return false; }
    if (p->L < 1 || p->L > 3) { why = "L must be 1, 2 or 3"; return false; }
    if (p->bgbit < 1 || p->bgbit * p->L > 32) { why = "bgbit*L must be <= 32"; return false; }
    // key-switch kernels are instantiated for basebit 2 with t in [7, 9]
    // (128/80-bit) and basebit 3..8 with t in [2, 4] (Uint sets)
    const bool ks_sel = p->basebit == 2 && p->iks_t >= 7 && p->iks_t <= 9;
    const bool ks_gather = p->basebit >= 3 && p->basebit <= 8 && p->iks_t >= 2 && p->iks_t <= 4;
    if (!(ks_sel || ks_gather) || p->basebit * p->iks_t >= 31) {
        why = "unsupported key-switch base/levels";
        return false;
    }
    return true;
}

int ensure(tfhe_gpu_ctx *c, DevBuf &b, size_t bytes) {
    if (b.bytes >= bytes) return TFHE_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    size_t want = std::max<size_t>(bytes, 4096);
    hipError_t e = hipMalloc(&b.p, want);
    if (e != hipSuccess) return fail(c, TFHE_ERR_OOM, std::string("hipMalloc: ") + hipGetErrorString(e));
    b.bytes = want;
    return TFHE_OK;
}

DevTables tables(const tfhe_gpu_ctx *c) {
    return DevTables{c->d_twist, c->d_tw, {c->twa[0], c->twa[1], c->twa[2], c->twa[3]}};
}

size_t tlwe0_words(const tfhe_gpu_ctx *c) { return (size_t)c->P.n + 1; }
size_t bk_rows(const tfhe_params &p) { return (size_t)p.n * 2 * p.L; }
size_t ksk_rows(const tfhe_params &p) { return (size_t)p.N * p.iks_t * (1u << p.basebit); }
size_t ksk_words(const tfhe_params &p) { return ksk_rows(p) * (p.n + 1); }
// device KSK: padded rows + zero tail (tfhe_internal.hpp)
size_t ksk_dev_bytes(const tfhe_params &p) {
    return (ksk_rows(p) * ks_stride_for((int)p.n) + KS_TAIL_WORDS) * sizeof(uint32_t);
}

// host KSK (reference layout) -> device KSK (padded rows), async on the ctx stream
int upload_ksk(tfhe_gpu_ctx *c, const uint32_t *ksk) {
    const size_t w = c->P.n + 1, stride = c->K.ks_stride;
    c->ksk_gemm_ok = false;
    HIPCHK(c, hipMemsetAsync(c->d_ksk, 0, c->ksk_bytes, c->stream));
    HIPCHK(c, hipMemcpy2DAsync(c->d_ksk, stride * 4, ksk, w * 4, w * 4, ksk_rows(c->P), hipMemcpyHostToDevice,
                               c->stream));
    return TFHE_OK;
}

int set_key_common(tfhe_gpu_ctx *c, uint32_t offset, const uint32_t *tv_a, const uint32_t *tv_b) {
    const uint32_t N = c->P.N;
    c->offset = offset;
    c->K.offset = offset;
    c->testvec.assign(tv_a, tv_a + N);
    c->testvec.insert(c->testvec.end(), tv_b, tv_b + N);
    if (!c->d_testvec) HIPCHK(c, hipMalloc((void **)&c->d_testvec, sizeof(uint32_t) * 2 * N));
    HIPCHK(c, hipMemcpyAsync(c->d_testvec, c->testvec.data(), sizeof(uint32_t) * 2 * N, hipMemcpyHostToDevice,
                             c->stream));
    if (!c->d_bk) {
        c->bk_bytes = bk_rows(c->P) * 2048 * sizeof(double);
        c->ksk_bytes = ksk_dev_bytes(c->P);
        hipError_t e = hipMalloc((void **)&c->d_bk, c->bk_bytes);
        if (e != hipSuccess) return fail(c, TFHE_ERR_OOM, "hipMalloc(bk)");
        e = hipMalloc((void **)&c->d_ksk, c->ksk_bytes);
        if (e != hipSuccess) return fail(c, TFHE_ERR_OOM, "hipMalloc(ksk)");
    }
    return TFHE_OK;
}

// What a blind-rotation launch hands back.
enum RunKind : int {
    RUN_BOOTSTRAP = 0,     // sample extract + key switch: TLWELv0 (vanilla.zig:38-52)
    RUN_TRLWE = 1,         // the accumulator: TRLWELv1 (trgsw.zig:290-333)
    RUN_NO_KEYSWITCH = 2,  // sampleExtractIndex2, n+1 words (vanilla.zig:58-69)
};

// The gemm key switch's buffers for a batch of B (TFHE_OPT_KS_FORM = 2, or 3 from
// KS_GEMM_MIN_ITEMS items): the
// MFMA-layout KSK, rebuilt on the stream after a key change, and the partial
// sums.  G stays empty for the other forms (launch_key_switch ignores it).
int ks_gemm_args(tfhe_gpu_ctx *c, size_t B, KsGemm &G) {
    G = KsGemm();
    const bool want = c->opts.ks_form == 2 ||
                      (c->opts.ks_form == 3 && B >= KS_GEMM_MIN_ITEMS && ks_gemm_auto(c->K.iks_t, c->K.basebit));
    if (!want || !ks_gemm_supported(c->K)) return TFHE_OK;
    if (!c->d_ksk_gemm) {
        hipError_t e = hipMalloc((void **)&c->d_ksk_gemm, ks_gemm_bytes(c->K, 1024, c->K.iks_t, c->K.basebit));
        if (e != hipSuccess) return fail(c, TFHE_ERR_OOM, "hipMalloc(ksk gemm layout)");
    }
    if (!c->ksk_gemm_ok) {
        HIPCHK(c, launch_ksk_to_gemm(c->K, c->d_ksk, c->d_ksk_gemm, 1024, c->K.iks_t, c->K.basebit, c->stream));
        c->ksk_gemm_ok = true;
    }
    int rc = ensure(c, c->s_kspart, ks_gemm_part_bytes(c->K, B, 1024, c->K.basebit));
    if (rc) return rc;
    G.kg = c->d_ksk_gemm;
    G.part = (uint32_t *)c->s_kspart.p;
    return TFHE_OK;
}

// Blind rotation (+ key switch for RUN_BOOTSTRAP) over device buffers, async.
int run_bootstrap_dev(tfhe_gpu_ctx *c, const uint8_t *ops, const uint32_t *a, const uint32_t *b,
                      const uint32_t *testvec_dev, uint32_t *out, size_t B, int kind,
                      const uint32_t *idx = nullptr) {
    const bool key_switch = kind == RUN_BOOTSTRAP;
    const int out_mode = kind == RUN_BOOTSTRAP ? BR_OUT_LV1 : kind == RUN_TRLWE ? BR_OUT_TRLWE : BR_OUT_LV0_EXTRACT2;
    if (!c->has_key) return fail(c, TFHE_ERR_NO_KEY, "no cloud key loaded");
    if (B == 0) return TFHE_OK;
    int rc = ensure(c, c->s_lv1, B * 1025 * sizeof(uint32_t));
    if (rc) return rc;
    if (c->s_ties.bytes < B) {  // the flags are all zero between launches: a new buffer starts zeroed
        rc = ensure(c, c->s_ties, B);
        if (rc) return rc;
        HIPCHK(c, hipMemsetAsync(c->s_ties.p, 0, c->s_ties.bytes, c->stream));
    }
    KParams K = c->K;
    K.tie_flags = (uint8_t *)c->s_ties.p;
    uint32_t *lv1 = key_switch ? (uint32_t *)c->s_lv1.p : out;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    if (c->profiling) {
        while (c->events.size() < c->ev_used + 3) {
            hipEvent_t e;
            HIPCHK(c, hipEventCreate(&e));
            c->events.push_back(e);
        }
        for (int i = 0; i < 3; i++) ev[i] = c->events[c->ev_used + i];
        c->ev_used += 3;
        HIPCHK(c, hipEventRecord(ev[0], c->stream));
    }
    HIPCHK(c, launch_blind_rotate(K, tables(c), ops, a, b, idx, testvec_dev ? testvec_dev : c->d_testvec, c->d_bk,
                                  lv1, out_mode, B, c->stream, c->opts, &c->last_br));
    c->bootstraps += B;
    if (ev[1]) HIPCHK(c, hipEventRecord(ev[1], c->stream));
    c->last_ks = "";
    if (key_switch) {
        KsGemm G;
        if ((rc = ks_gemm_args(c, B, G))) return rc;
        HIPCHK(c, launch_key_switch(c->K, lv1, c->d_ksk, out, B, c->stream, c->opts, &c->last_ks, &G));
    }
    if (ev[2]) HIPCHK(c, hipEventRecord(ev[2], c->stream));
    return TFHE_OK;
}

bool staged(const tfhe_gpu_ctx *c) { return c->host_staging == TFHE_STAGING_PINNED; }

// Pinned host buffer of at least `bytes` (grown by doubling; nothing may be in flight from it).
int ensure_stage(tfhe_gpu_ctx *c, char *&p, size_t &have, size_t bytes) {
    if (have >= bytes) return TFHE_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    have = 0;
    const size_t want = std::max(bytes, (size_t)1 << 20);
    HIPCHK(c, hipHostMalloc((void **)&p, want, hipHostMallocDefault));
    have = want;
    return TFHE_OK;
}

// Host -> device into `buf`.  Pageable: one hipMemcpyAsync from the caller's buffer.  Staged
// (TFHE_OPT_HOST_STAGING): a host memcpy into this context's pinned arena, then the DMA from
// there, so concurrent shards' copies do not go through the runtime's pageable staging
// (for hosts where those serialise across host threads; on the MI355X box they do not and
// pageable copies are faster).  The arena is reused from
// offset 0 after every synchronisation of the stream (d2h_sync); when it is full the stream
// is synchronised first, so no copy in flight ever reads overwritten bytes.
int h2d(tfhe_gpu_ctx *c, DevBuf &buf, const void *src, size_t bytes) {
    int rc = ensure(c, buf, bytes);
    if (rc) return rc;
    if (!staged(c) || !bytes) {
        HIPCHK(c, hipMemcpyAsync(buf.p, src, bytes, hipMemcpyHostToDevice, c->stream));
        return TFHE_OK;
    }
    const size_t need = (bytes + 255) & ~(size_t)255;
    if (c->stage_used + need > c->stage_in_bytes) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        c->stage_used = 0;
        if (need > c->stage_in_bytes) {  // grow (doubling) only when one copy does not fit the empty arena
            rc = ensure_stage(c, c->stage_in, c->stage_in_bytes, std::max(need, 2 * c->stage_in_bytes));
            if (rc) return rc;
        }
    }
    char *p = c->stage_in + c->stage_used;
    std::memcpy(p, src, bytes);
    HIPCHK(c, hipMemcpyAsync(buf.p, p, bytes, hipMemcpyHostToDevice, c->stream));
    c->stage_used += need;
    return TFHE_OK;
}

// Synchronise the context stream and fail the call if a kernel on it set the
// device error word (a slot-counter wait of the blind rotation gave up: its
// words are not the reference's).  The word is copied into pinned host memory
// on the stream, so the one synchronisation covers both; a reported error is
// cleared, and the context stays usable.
// Queue the copy of the device error word (and the recompute counter) into
// pinned host memory on the context stream.
static int queue_err_copy(tfhe_gpu_ctx *c) {
    HIPCHK(c, hipMemcpyAsync(c->h_err, c->d_err, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    return TFHE_OK;
}

// After a synchronisation that covered queue_err_copy: fail the call if a
// kernel set the error word (clearing it; the context stays usable).
static int check_err_word(tfhe_gpu_ctx *c) {
    c->near_tie_items = c->h_err[1];
    const uint32_t e = *c->h_err;
    if (!e) return TFHE_OK;
    *c->h_err = 0;
    HIPCHK(c, hipMemsetAsync(c->d_err, 0, sizeof(uint32_t), c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::string what;
    if (e & DEV_ERR_GATE_WAIT) what += "slot-counter protocol failure: a gate wave's wait for a BK slot timed out";
    if (e & DEV_ERR_LOADER_WAIT)
        what += std::string(what.empty() ? "slot-counter protocol failure:" : " and") +
                " a loader wave's wait for a free BK slot timed out";
    if (e & DEV_ERR_LDS_LAYOUT) what += std::string(what.empty() ? "" : "; ") + "LDS array not at address 0, nothing computed";
    return fail(c, TFHE_ERR_DEVICE,
                "blind rotation: " + what + " (device error word 0x" +
                    [&] { char b[16]; std::snprintf(b, sizeof b, "%x", e); return std::string(b); }() +
                    "); the outputs of the work since the last synchronisation are invalid");
}

int sync_check(tfhe_gpu_ctx *c) {
    int rc = queue_err_copy(c);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return check_err_word(c);
}

// 64-bit fingerprints of this context's device BK and KSK (k_checksum), synchronous.
int key_fingerprint(tfhe_gpu_ctx *c, uint64_t &bk, uint64_t &ksk) {
    auto *d = reinterpret_cast<unsigned long long *>(c->d_err + 2);
    auto *h = reinterpret_cast<volatile unsigned long long *>(c->h_err + 2);
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, launch_checksum(c->d_bk, c->bk_bytes, d, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->h_err + 2, d, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    bk = *h;
    HIPCHK(c, launch_checksum(c->d_ksk, c->ksk_bytes, d, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->h_err + 2, d, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    ksk = *h;
    return TFHE_OK;
}

// Key admission of the fused arithmetic.  Its margin guard gives
// the reference's words while the fused and the reference's pre-rounding values
// differ by less than 1/4 — measured, not proven.  Two rules, both on the device
// key at load:
//  - spectrum: the largest BK spectrum component (reference scale) <= 2^39 (round
//    4: concentrated spectra, 2^40.4-2^41.3, reached gaps of 0.19-0.31);
//  - row energy (round 5): every TRGSW row's RMS <= 0.65 x 2^31.  By Parseval the
//    spectrum energy of a row is 2048 x its coefficient energy, so this bounds
//    every row's L1 norm by 1024 x 0.65 x 2^31 and with it every pre-rounding value
//    of the external product, |sum_i digit . row_i| <= 6 x 32 x 1024 x 0.65 x 2^31
//    < 2^48 at the 128-bit set: below 2^48 an f64 ulp is at most 2^-5, half what it
//    is above.  A hill-climbing search for the worst admitted key
//    (tools/admission_search.py, profiles/r05_admission_search.json) finds gaps of
//    at most 0.1875 under the spectrum rule alone (rows of +-(2^31 - 1), RMS 1) and
//    0.125 under both.  Keygen'd rows have RMS 0.545-0.605 (8,400 rows of the
//    seeded 128-bit key); exceeding 0.65 needs a 9.6-sigma row mean of a square.
// A key outside either rule runs the reference's expression trees
// (TFHE_OPT_FUSED_ADMITTED reads the outcome, TFHE_OPT_KEY_ROW_RMS_PPM the RMS).
constexpr double FUSED_BK_SPECTRUM_MAX = 549755813888.0;  // 2^39
constexpr double FUSED_BK_ROW_RMS_MAX = 0.65;             // x 2^31
int key_admission(tfhe_gpu_ctx *c) {
    // refused until measured: a failure below (absmax launch, copy, sync) must not
    // leave the previous key's admission in place
    c->opts.key_fused_ok = 0;
    auto *d = reinterpret_cast<unsigned long long *>(c->d_err + 2);
    auto *h = reinterpret_cast<volatile unsigned long long *>(c->h_err + 2);
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, launch_absmax(c->d_bk, c->bk_bytes / sizeof(double), d, c->stream));
    HIPCHK(c, launch_row_energy_max(c->d_bk, (size_t)c->P.n * 2 * c->P.L, d + 1, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->h_err + 2, d, 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const unsigned long long bits = h[0], ebits = h[1];
    double m, e;
    std::memcpy(&m, (const void *)&bits, 8);
    std::memcpy(&e, (const void *)&ebits, 8);
    c->bk_absmax = std::ldexp(m, 10);  // the device BK is the reference's spectrum x 2^-10 (k_bk_permute)
    // row energy: device spectrum energy x 2^20 = reference spectrum energy = 2048 x N x RMS^2
    c->bk_row_rms = std::sqrt(std::ldexp(e, 20) / (2048.0 * c->P.N)) / 2147483648.0;
    c->opts.key_fused_ok =
        c->bk_absmax <= FUSED_BK_SPECTRUM_MAX && c->bk_row_rms <= FUSED_BK_ROW_RMS_MAX ? 1 : 0;  // NaN fails
    return TFHE_OK;
}

// The outputs and the error word in one synchronisation: the word's copy is
// queued first, so it has landed when the outputs have (one round trip fewer
// than copying it after them: DESIGN.md §2.1).
int d2h_sync(tfhe_gpu_ctx *c, void *dst, const void *src, size_t bytes) {
    int rc = queue_err_copy(c);
    if (rc) return rc;
    if (staged(c) && bytes) {  // DMA into the pinned arena, one synchronisation, then a host memcpy
        rc = ensure_stage(c, c->stage_out, c->stage_out_bytes, bytes);
        if (rc) return rc;
        HIPCHK(c, hipMemcpyAsync(c->stage_out, src, bytes, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        c->stage_used = 0;  // every staged H2D of the call has landed
        std::memcpy(dst, c->stage_out, bytes);
        return check_err_word(c);
    }
    HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    // a pageable destination makes the copy synchronous: the stream is idle by
    // now and hipStreamQuery says so at once, where hipStreamSynchronize on an
    // idle stream still took ~19 us (profiles/r03_host_path_trace.txt)
    const hipError_t q = hipStreamQuery(c->stream);
    if (q == hipErrorNotReady) HIPCHK(c, hipStreamSynchronize(c->stream));
    else HIPCHK(c, q);
    return check_err_word(c);
}

// TLWELv0.encryptF64 (tlwe.zig:34-49) with DefaultPrng(seed).
void tlwe_encrypt(uint32_t n, double mu, double alpha, const uint32_t *key, uint64_t seed, uint32_t *out) {
    host::Rng r(seed);
    uint32_t inner = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t x = r.u32();
        inner += key[i] * x;
        out[i] = x;
    }
    host::NormalDist nd(0.0, alpha);
    uint32_t mu_t = host::f64_to_torus(mu);
    out[n] = inner + host::gaussian_torus(mu_t, nd, r);
}

uint32_t tlwe_phase(uint32_t n, const uint32_t *ct, const uint32_t *key) {
    uint32_t inner = 0;
    for (uint32_t i = 0; i < n; i++) inner += ct[i] * key[i];
    return ct[n] - inner;
}

// PublicKeyLv0.encryptF64 (proxy_reenc.zig:83-113): plaintext on b, each
// encryption of zero kept with probability 1/2 and added or subtracted with
// probability 1/2 (two booleans, the second only when kept), then fresh noise.
void pk_encrypt(uint32_t n, const uint32_t *pk, size_t pk_size, double plaintext, double alpha, uint64_t seed,
                uint32_t *out) {
    host::Rng r(seed);
    std::fill(out, out + n + 1, 0u);
    out[n] = host::f64_to_torus(plaintext);
    for (size_t e = 0; e < pk_size; e++) {
        if (!r.boolean()) continue;
        const uint32_t *enc = pk + e * (n + 1);
        if (r.boolean())
            for (uint32_t x = 0; x <= n; x++) out[x] += enc[x];
        else
            for (uint32_t x = 0; x <= n; x++) out[x] -= enc[x];
    }
    host::NormalDist nd(0.0, alpha);
    out[n] += host::gaussian_torus(0u, nd, r);
}

// ProxyReencryptionKey.new{Symmetric,Asymmetric}WithParams (proxy_reenc.zig:
// 150-256): entry (i, j, k != 0) encrypts k * key_from[i] / 2^((j+1)*basebit)
// under the target; the c-th encryption in (i, j, k) order uses seed0 + c.
template <class Enc>
void reenc_key_gen(uint32_t n, const uint32_t *key_from, uint32_t basebit, uint32_t t, uint64_t seed0,
                   uint32_t *out, Enc enc) {
    const uint32_t base = 1u << basebit;
    std::fill(out, out + (size_t)n * t * base * (n + 1), 0u);
    uint64_t c = 0;
    for (uint32_t i = 0; i < n; i++)
        for (uint32_t j = 0; j < t; j++)
            for (uint32_t k = 1; k < base; k++) {
                const double p = ((double)k * (double)key_from[i]) / (double)(1u << ((j + 1) * basebit));
                enc(p, seed0 + c++, out + ((size_t)base * t * i + (size_t)base * j + k) * (n + 1));
            }
}

int broadcast_key(tfhe_gpu_ctx *c);    // multi-device key broadcast (end of file)
bool is_multi(const tfhe_gpu_ctx *c);  // a context over more than one device (end of file)
void destroy_shards(tfhe_gpu_ctx *c);  // sub-contexts and RCCL communicators (end of file)

// FFT constant tables (fft.zig:92-106 twists, :590-616 recurrence) from the
// chosen cos/sin source (host_math.hpp), uploaded to the context's device.
int build_tables(tfhe_gpu_ctx *c, int source) {
    std::vector<double> tre, tim, fre, fim, ire, iim;
    host::twist_table(c->P.N, tre, tim, source);
    host::stage_twiddles(c->P.N, false, fre, fim, source);
    host::stage_twiddles(c->P.N, true, ire, iim, source);
    // the inverse kernels use conj(forward): that must equal the inverse
    // recurrence bit for bit (both sources have an odd sin and an even cos)
    for (size_t i = 0; i < fre.size(); i++)
        if (std::memcmp(&fre[i], &ire[i], 8) != 0 || -fim[i] != iim[i])
            return fail(c, TFHE_ERR_INVALID, "inverse twiddle table is not the conjugate of the forward one");
    std::vector<C2> tw2(tre.size()), st2(fre.size());
    for (size_t i = 0; i < tre.size(); i++) tw2[i] = C2{tre[i], tim[i]};
    for (size_t i = 0; i < fre.size(); i++) st2[i] = C2{fre[i], fim[i]};
    // passA's bf_m1 (tfhe_kernels.hip) relies on W4[1].im == W8[2].im == -1.0 exactly
    if (st2[2].y != -1.0 || st2[5].y != -1.0)
        return fail(c, TFHE_ERR_INVALID, "twiddle table: W4[1] / W8[2] imaginary part is not exactly -1");
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->d_twist) HIPCHK(c, hipMalloc((void **)&c->d_twist, sizeof(C2) * tw2.size()));
    if (!c->d_tw) HIPCHK(c, hipMalloc((void **)&c->d_tw, sizeof(C2) * st2.size()));
    HIPCHK(c, hipStreamSynchronize(c->stream));  // no launch may still read the old tables
    HIPCHK(c, hipMemcpy(c->d_twist, tw2.data(), sizeof(C2) * tw2.size(), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_tw, st2.data(), sizeof(C2) * st2.size(), hipMemcpyHostToDevice));
    c->twa[0] = st2[2];
    c->twa[1] = st2[4];
    c->twa[2] = st2[5];
    c->twa[3] = st2[6];
    c->twiddle_source = source;
    return TFHE_OK;
}

}  // namespace

extern "C" {

int tfhe_gpu_abi_version(void) { return TFHE_GPU_ABI_VERSION; }

static const char *AB_REFUSAL =
    "tfhe_gpu_create: this library is an A/B build (tfhe_gpu_build_kind), not the product; set "
    "TFHE_ALLOW_AB_BUILD=1 to use it for A/B runs";
static bool ab_build_refused() {  // knock-out / timing / losing-form builds need the opt-in
    if (tfhe_gpu_build_kind() == TFHE_BUILD_PRODUCT) return false;
    const char *allow = std::getenv("TFHE_ALLOW_AB_BUILD");
    return !allow || std::strcmp(allow, "1") != 0;
}

int tfhe_gpu_build_kind(void) {
#ifdef TFHE_AB_BUILD
    return TFHE_BUILD_AB;
#else
    return kernels_ab_build() || ab_forms_linked() ? TFHE_BUILD_AB : TFHE_BUILD_PRODUCT;
#endif
}

int tfhe_gpu_create_on_device(const tfhe_params *params, int device, tfhe_gpu_ctx **out) {
    if (!out) return TFHE_ERR_INVALID;
    *out = nullptr;
    std::string why;
    if (!params_ok(params, why)) return create_fail(TFHE_ERR_INVALID, "tfhe_gpu_create: " + why);
    if (ab_build_refused()) return create_fail(TFHE_ERR_INVALID, AB_REFUSAL);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return create_fail(TFHE_ERR_HIP, "device " + std::to_string(device) + " does not exist (" +
                                             std::to_string(ndev) + " HIP device(s) visible)");
    auto *c = new tfhe_gpu_ctx();
    c->P = *params;
    c->device = device;
    c->K = KParams{(int)params->n, (int)params->N, (int)params->L, (int)params->bgbit, (int)params->basebit,
                   (int)params->iks_t, 0, ks_stride_for((int)params->n), nullptr, 0u, nullptr, 0};
    int rc = TFHE_OK;
    do {
        hipError_t e = hipSetDevice(device);
        if (e != hipSuccess) { rc = hip_fail(c, e, "hipSetDevice"); break; }
        e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
        if (e != hipSuccess) { rc = hip_fail(c, e, "hipStreamCreate"); break; }
        c->stream = c->own_stream;
        e = hipMalloc((void **)&c->d_err, 64);
        if (e == hipSuccess) e = hipMemset(c->d_err, 0, 64);
        if (e == hipSuccess) e = hipHostMalloc((void **)&c->h_err, 64, hipHostMallocDefault);
        if (e != hipSuccess) { rc = hip_fail(c, e, "device error word"); break; }
        std::memset(c->h_err, 0, 64);
        c->K.err = c->d_err;
        rc = build_tables(c, TFHE_TWIDDLES_GLIBC);
    } while (0);
    if (rc != TFHE_OK) {
        const std::string msg = "tfhe_gpu_create: " + c->err;
        tfhe_gpu_destroy(c);
        return create_fail(rc, msg);
    }
    *out = c;
    return TFHE_OK;
}

void tfhe_gpu_destroy(tfhe_gpu_ctx *c) {
    if (!c) return;
    destroy_shards(c);
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);  // NULL is a valid stream here (the device's null stream)
    for (void *p : {(void *)c->d_err, (void *)c->d_twist, (void *)c->d_tw, (void *)c->d_testvec, (void *)c->d_bk, (void *)c->d_ksk,
                    c->s_a.p, c->s_b.p, c->s_out.p, c->s_lv1.p, c->s_ops.p, c->s_tv.p, c->s_tmp.p, c->s_ties.p,
                    c->s_wires.p, c->s_cidx.p, c->s_cops.p, c->s_kspart.p, (void *)c->d_ksk_gemm})
        if (p) (void)hipFree(p);
    for (hipEvent_t e : c->events) (void)hipEventDestroy(e);
    if (c->h_err) (void)hipHostFree(c->h_err);
    c->workers.reset();
    for (hipStream_t &p : c->pipe)
        if (p) (void)hipStreamDestroy(p);
    if (c->pipe_ev) (void)hipEventDestroy(c->pipe_ev);
    if (c->pin_in) (void)hipHostFree(c->pin_in);
    if (c->pin_out) (void)hipHostFree(c->pin_out);
    if (c->stage_in) (void)hipHostFree(c->stage_in);
    if (c->stage_out) (void)hipHostFree(c->stage_out);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    if (c->stream_ev) (void)hipEventDestroy(c->stream_ev);
    delete c;
}

const char *tfhe_gpu_last_error(const tfhe_gpu_ctx *c) {
    if (c) return c->err.c_str();
    return g_create_error.empty() ? "null context" : g_create_error.c_str();
}

int tfhe_gpu_key_fingerprint(tfhe_gpu_ctx *c, uint64_t *bk, uint64_t *ksk) {
    if (!c || !bk || !ksk) return fail(c, TFHE_ERR_INVALID, "null argument");
    if (!c->has_key) return fail(c, TFHE_ERR_NO_KEY, "no cloud key loaded");
    uint64_t b = 0, k = 0;
    const int rc = key_fingerprint(c, b, k);
    if (rc) return rc;
    *bk = b;
    *ksk = k;
    return TFHE_OK;
}

int tfhe_gpu_sync(tfhe_gpu_ctx *c) {
    if (!c) return TFHE_ERR_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    return sync_check(c);
}

// The context queues its own work on its stream too (the MFMA-layout KSK build,
// the near-tie flag and error-word clears): the new stream waits for everything
// queued on the old one, so a _dev call on the new stream never overtakes it.
static int switch_stream(tfhe_gpu_ctx *c, hipStream_t ns) {
    if (ns == c->stream) return TFHE_OK;
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->stream_ev) HIPCHK(c, hipEventCreateWithFlags(&c->stream_ev, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(c->stream_ev, c->stream));
    HIPCHK(c, hipStreamWaitEvent(ns, c->stream_ev, 0));
    c->stream = ns;
    return TFHE_OK;
}

// ABI 7: NULL is the device's null stream (torch's default stream has handle 0),
// no longer "back to the context's own stream", which is tfhe_gpu_reset_stream.
// Up to ABI 6 a caller passing torch's default stream got the context's own
// non-blocking stream, unordered with torch's work.
int tfhe_gpu_set_stream(tfhe_gpu_ctx *c, void *s) {
    if (!c) return TFHE_ERR_INVALID;
    return switch_stream(c, (hipStream_t)s);
}

int tfhe_gpu_reset_stream(tfhe_gpu_ctx *c) {
    if (!c) return TFHE_ERR_INVALID;
    return switch_stream(c, c->own_stream);
}

int tfhe_gpu_load_cloud_key(tfhe_gpu_ctx *c, uint32_t offset, const uint32_t *tv_a, const uint32_t *tv_b,
                            const double *bsk, size_t bsk_len, const uint32_t *ksk, size_t ksk_len) {
    if (!c || !tv_a || !tv_b || !bsk || !ksk) return fail(c, TFHE_ERR_INVALID, "null argument");
    const size_t rows = bk_rows(c->P);
    if (bsk_len != rows * 2 * c->P.N) return fail(c, TFHE_ERR_INVALID, "bsk_len != n*2L*2*N");
    if (ksk_len != ksk_words(c->P)) return fail(c, TFHE_ERR_INVALID, "ksk_len != N*t*2^basebit*(n+1)");
    HIPCHK(c, hipSetDevice(c->device));
    int rc = set_key_common(c, offset, tv_a, tv_b);
    if (rc) return rc;
    rc = h2d(c, c->s_tmp, bsk, bsk_len * sizeof(double));
    if (rc) return rc;
    HIPCHK(c, launch_bk_permute(c->K, (const double *)c->s_tmp.p, c->d_bk, rows, c->stream));
    rc = upload_ksk(c, ksk);
    if (rc) return rc;
    HIPCHK(c, launch_ksk_zero_k0(c->K, c->d_ksk, c->stream));  // reference leaves k=0 rows undefined
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->has_key = true;
    c->key_from_keygen = false;
    return broadcast_key(c);
}

int tfhe_gpu_key_blob_bytes(const tfhe_gpu_ctx *c, size_t *bsk_bytes, size_t *ksk_bytes) {
    if (!c || !bsk_bytes || !ksk_bytes) return TFHE_ERR_INVALID;
    *bsk_bytes = bk_rows(c->P) * 2048 * sizeof(double);
    *ksk_bytes = ksk_dev_bytes(c->P);  // device layout (padded rows), not the reference's
    return TFHE_OK;
}

int tfhe_gpu_export_key_device(tfhe_gpu_ctx *c, void *bsk_dev, void *ksk_dev, uint32_t *offset,
                               uint32_t *testvec) {
    if (!c || !bsk_dev || !ksk_dev) return fail(c, TFHE_ERR_INVALID, "null argument");
    if (!c->has_key) return fail(c, TFHE_ERR_NO_KEY, "no cloud key loaded");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(bsk_dev, c->d_bk, c->bk_bytes, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(ksk_dev, c->d_ksk, c->ksk_bytes, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (offset) *offset = c->offset;
    if (testvec) std::memcpy(testvec, c->testvec.data(), sizeof(uint32_t) * 2 * c->P.N);
    return TFHE_OK;
}

int tfhe_gpu_import_key_device(tfhe_gpu_ctx *c, const void *bsk_dev, const void *ksk_dev, uint32_t offset,
                               const uint32_t *testvec) {
    if (!c || !bsk_dev || !ksk_dev || !testvec) return fail(c, TFHE_ERR_INVALID, "null argument");
    HIPCHK(c, hipSetDevice(c->device));
    int rc = set_key_common(c, offset, testvec, testvec + c->P.N);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(c->d_bk, bsk_dev, c->bk_bytes, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_ksk, ksk_dev, c->ksk_bytes, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, launch_ksk_zero_k0(c->K, c->d_ksk, c->stream));
    c->ksk_gemm_ok = false;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->has_key = true;
    c->key_from_keygen = false;
    return broadcast_key(c);
}

// Device key -> reference host layout: BK un-permuted (and un-scaled) by
// k_bk_permute's inverse, KSK rows un-padded.
int tfhe_gpu_export_cloud_key(tfhe_gpu_ctx *c, uint32_t *offset, uint32_t *tv_a, uint32_t *tv_b, double *bsk,
                              uint32_t *ksk) {
    if (!c) return TFHE_ERR_INVALID;
    if (!c->has_key) return fail(c, TFHE_ERR_NO_KEY, "no cloud key loaded");
    HIPCHK(c, hipSetDevice(c->device));
    const size_t N = c->P.N;
    if (offset) *offset = c->offset;
    if (tv_a) std::memcpy(tv_a, c->testvec.data(), N * sizeof(uint32_t));
    if (tv_b) std::memcpy(tv_b, c->testvec.data() + N, N * sizeof(uint32_t));
    if (bsk) {
        const size_t rows = bk_rows(c->P), bytes = rows * 2 * N * sizeof(double);
        int rc = ensure(c, c->s_tmp, bytes);
        if (rc) return rc;
        HIPCHK(c, launch_bk_unpermute(c->K, c->d_bk, (double *)c->s_tmp.p, rows, c->stream));
        HIPCHK(c, hipMemcpyAsync(bsk, c->s_tmp.p, bytes, hipMemcpyDeviceToHost, c->stream));
    }
    if (ksk) {
        const size_t w = c->P.n + 1;
        HIPCHK(c, hipMemcpy2DAsync(ksk, w * 4, c->d_ksk, (size_t)c->K.ks_stride * 4, w * 4, ksk_rows(c->P),
                                   hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TFHE_OK;
}

}  // extern "C"

// ---- Cloud-key files (include/tfhe_gpu.h) ---------------
namespace {

struct KeyFileHeader {
    char magic[8];
    uint32_t version, n, N, L, bgbit, basebit, iks_t, offset;
    uint64_t bsk_len, ksk_len, checksum;
};
static_assert(sizeof(KeyFileHeader) == 64, "key file header is 64 bytes");
constexpr char KEY_MAGIC[8] = {'Z', 'T', 'F', 'H', 'E', 'C', 'K', '1'};

// FNV-1a-64 over 8-byte little-endian words; a section's last < 8 bytes one by one
struct Fnv64 {
    uint64_t h = 0xcbf29ce484222325ull;
    void add(const void *p, size_t bytes) {
        const unsigned char *b = static_cast<const unsigned char *>(p);
        size_t k = 0;
        for (; k + 8 <= bytes; k += 8) {
            uint64_t w;
            std::memcpy(&w, b + k, 8);
            h = (h ^ w) * 0x100000001b3ull;
        }
        for (; k < bytes; k++) h = (h ^ b[k]) * 0x100000001b3ull;
    }
};

uint64_t key_checksum(const tfhe_params *p, const uint32_t *tv_a, const uint32_t *tv_b, const double *bsk,
                      size_t bsk_len, const uint32_t *ksk, size_t ksk_len) {
    Fnv64 f;
    f.add(tv_a, p->N * sizeof(uint32_t));
    f.add(tv_b, p->N * sizeof(uint32_t));
    f.add(bsk, bsk_len * sizeof(double));
    f.add(ksk, ksk_len * sizeof(uint32_t));
    return f.h;
}

bool key_shape_ok(const tfhe_params *p, size_t bsk_len, size_t ksk_len) {
    std::string why;
    return params_ok(p, why) && bsk_len == bk_rows(*p) * 2 * p->N && ksk_len == ksk_words(*p);
}

}  // namespace

extern "C" {

int tfhe_cloud_key_write(const char *path, const tfhe_params *p, uint32_t offset, const uint32_t *tv_a,
                         const uint32_t *tv_b, const double *bsk, size_t bsk_len, const uint32_t *ksk,
                         size_t ksk_len) {
    if (!path || !tv_a || !tv_b || !bsk || !ksk || !key_shape_ok(p, bsk_len, ksk_len)) return TFHE_ERR_INVALID;
    KeyFileHeader h{};
    std::memcpy(h.magic, KEY_MAGIC, 8);
    h.version = 1;
    h.n = p->n, h.N = p->N, h.L = p->L, h.bgbit = p->bgbit, h.basebit = p->basebit, h.iks_t = p->iks_t;
    h.offset = offset;
    h.bsk_len = bsk_len;
    h.ksk_len = ksk_len;
    h.checksum = key_checksum(p, tv_a, tv_b, bsk, bsk_len, ksk, ksk_len);
    FILE *fp = std::fopen(path, "wb");
    if (!fp) return TFHE_ERR_IO;
    bool ok = std::fwrite(&h, sizeof h, 1, fp) == 1 && std::fwrite(tv_a, 4, p->N, fp) == p->N &&
              std::fwrite(tv_b, 4, p->N, fp) == p->N && std::fwrite(bsk, 8, bsk_len, fp) == bsk_len &&
              std::fwrite(ksk, 4, ksk_len, fp) == ksk_len;
    ok = std::fclose(fp) == 0 && ok;
    return ok ? TFHE_OK : TFHE_ERR_IO;
}

int tfhe_cloud_key_read(const char *path, const tfhe_params *p, uint32_t *offset, uint32_t *tv_a, uint32_t *tv_b,
                        double *bsk, size_t bsk_len, uint32_t *ksk, size_t ksk_len) {
    if (!path || !offset || !tv_a || !tv_b || !bsk || !ksk || !key_shape_ok(p, bsk_len, ksk_len))
        return TFHE_ERR_INVALID;
    FILE *fp = std::fopen(path, "rb");
    if (!fp) return TFHE_ERR_IO;
    KeyFileHeader h{};
    int rc = TFHE_OK;
    if (std::fread(&h, sizeof h, 1, fp) != 1)
        rc = TFHE_ERR_IO;
    else if (std::memcmp(h.magic, KEY_MAGIC, 8) != 0 || h.version != 1)
        rc = TFHE_ERR_INVALID;  // not a key file of this format
    else if (h.n != p->n || h.N != p->N || h.L != p->L || h.bgbit != p->bgbit || h.basebit != p->basebit ||
             h.iks_t != p->iks_t || h.bsk_len != bsk_len || h.ksk_len != ksk_len)
        rc = TFHE_ERR_INVALID;  // another parameter set
    else if (std::fread(tv_a, 4, p->N, fp) != p->N || std::fread(tv_b, 4, p->N, fp) != p->N ||
             std::fread(bsk, 8, bsk_len, fp) != bsk_len || std::fread(ksk, 4, ksk_len, fp) != ksk_len)
        rc = TFHE_ERR_IO;  // truncated
    std::fclose(fp);
    if (rc) return rc;
    if (key_checksum(p, tv_a, tv_b, bsk, bsk_len, ksk, ksk_len) != h.checksum) return TFHE_ERR_INVALID;
    *offset = h.offset;
    return TFHE_OK;
}

int tfhe_gpu_save_cloud_key(tfhe_gpu_ctx *c, const char *path) {
    if (!c || !path) return fail(c, TFHE_ERR_INVALID, "null argument");
    const size_t N = c->P.N, bl = bk_rows(c->P) * 2 * N, kl = ksk_words(c->P);
    std::vector<uint32_t> ta(N), tb(N), ksk(kl);
    std::vector<double> bsk(bl);
    uint32_t off = 0;
    int rc = tfhe_gpu_export_cloud_key(c, &off, ta.data(), tb.data(), bsk.data(), ksk.data());
    if (rc) return rc;
    rc = tfhe_cloud_key_write(path, &c->P, off, ta.data(), tb.data(), bsk.data(), bl, ksk.data(), kl);
    if (rc) return fail(c, rc, std::string("cannot write key file ") + path);
    return TFHE_OK;
}

int tfhe_gpu_load_cloud_key_file(tfhe_gpu_ctx *c, const char *path) {
    if (!c || !path) return fail(c, TFHE_ERR_INVALID, "null argument");
    const size_t N = c->P.N, bl = bk_rows(c->P) * 2 * N, kl = ksk_words(c->P);
    std::vector<uint32_t> ta(N), tb(N), ksk(kl);
    std::vector<double> bsk(bl);
    uint32_t off = 0;
    int rc = tfhe_cloud_key_read(path, &c->P, &off, ta.data(), tb.data(), bsk.data(), bl, ksk.data(), kl);
    if (rc == TFHE_ERR_IO) return fail(c, rc, std::string("cannot read key file ") + path);
    if (rc) return fail(c, rc, std::string(path) + ": not a key file of this parameter set, or checksum mismatch");
    return tfhe_gpu_load_cloud_key(c, off, ta.data(), tb.data(), bsk.data(), bl, ksk.data(), kl);
}

// SecretKey.new + CloudKey.new, seeded.  Host: every RNG draw in reference
// order; device: the FFT-based poly_mul of each TRLWE encryption
// (trlwe.zig:56-61) and the TRGSWLv1FFT forward transforms (trgsw.zig:81-91).
int tfhe_gpu_keygen(tfhe_gpu_ctx *c, uint64_t secret_seed, uint64_t cloud_seed, uint32_t *key_lv0,
                    uint32_t *key_lv1, double *bsk_out, uint32_t *ksk_out) {
    if (!c || !key_lv0 || !key_lv1) return fail(c, TFHE_ERR_INVALID, "null argument");
    const tfhe_params &p = c->P;
    const uint32_t N = p.N, n = p.n, L = p.L, T = p.iks_t, base = 1u << p.basebit;
    HIPCHK(c, hipSetDevice(c->device));
    tfhe_secret_key_new(&p, secret_seed, key_lv0, key_lv1);
    host::Rng master(cloud_seed);
    // genKeySwitchingKey (key.zig:148-172): k = 0 rows are zeroed
    std::vector<uint32_t> ksk(ksk_words(p), 0u);
    for (uint32_t i = 0; i < N; i++)
        for (uint32_t j = 0; j < T; j++)
            for (uint32_t k = 1; k < base; k++) {
                size_t idx = (size_t)base * T * i + (size_t)base * j + k;
                uint32_t shift = (j + 1) * p.basebit;
                double pv = ((double)k * (double)key_lv1[i]) / (double)(1u << shift);
                tlwe_encrypt(n, pv, p.alpha_ksk, key_lv0, master.next(), ksk.data() + idx * (n + 1));
            }
    // genBootstrappingKey (key.zig:175-212): per i, TRGSW encryptTorus of
    // key_lv0[i]: 2L TRLWE encryptions of zero (trlwe.zig:30-64), gadget on
    // a[0] of row l / b[0] of row L+l.
    const size_t R = bk_rows(p);  // n*2L TRLWE rows
    std::vector<uint32_t> rows(R * 2 * N);
    std::vector<uint32_t> noise(R * N);
    for (size_t row = 0; row < R; row++) {
        host::Rng r(master.next());
        uint32_t *a = rows.data() + row * 2 * N;
        for (uint32_t x = 0; x < N; x++) a[x] = r.u32();
        host::NormalDist nd(0.0, p.alpha_bsk);
        for (uint32_t x = 0; x < N; x++) noise[row * N + x] = host::gaussian_torus(0u, nd, r);
    }
    int rc = h2d(c, c->s_b, key_lv1, N * sizeof(uint32_t));
    if (rc) return rc;
    rc = ensure(c, c->s_out, R * N * sizeof(uint32_t));
    if (rc) return rc;
    // a*s for all rows: a_i lives at stride 2N inside `rows`
    std::vector<uint32_t> a_only(R * N);
    for (size_t row = 0; row < R; row++)
        std::memcpy(a_only.data() + row * N, rows.data() + row * 2 * N, N * sizeof(uint32_t));
    rc = h2d(c, c->s_a, a_only.data(), a_only.size() * sizeof(uint32_t));
    if (rc) return rc;
    HIPCHK(c, launch_poly_mul(tables(c), (const uint32_t *)c->s_a.p, (const uint32_t *)c->s_b.p, 0,
                              (uint32_t *)c->s_out.p, R, c->stream));
    std::vector<uint32_t> as(R * N);
    rc = d2h_sync(c, as.data(), c->s_out.p, as.size() * sizeof(uint32_t));
    if (rc) return rc;
    for (size_t row = 0; row < R; row++) {
        uint32_t *b = rows.data() + row * 2 * N + N;
        for (uint32_t x = 0; x < N; x++) b[x] = noise[row * N + x] + as[row * N + x];
    }
    for (uint32_t i = 0; i < n; i++) {
        uint32_t mu = key_lv0[i];
        for (uint32_t l = 0; l < L; l++) {
            uint32_t h = host::f64_to_torus(std::ldexp(1.0, -(int)((l + 1) * p.bgbit)));
            rows[((size_t)i * 2 * L + l) * 2 * N] += mu * h;              // trlwe[l].a[0]
            rows[((size_t)i * 2 * L + L + l) * 2 * N + N] += mu * h;      // trlwe[L+l].b[0]
        }
    }
    // TRGSWLv1FFT.new: ifft of every a and b polynomial -> reference BK layout
    rc = h2d(c, c->s_a, rows.data(), rows.size() * sizeof(uint32_t));
    if (rc) return rc;
    rc = ensure(c, c->s_tmp, R * 2 * N * sizeof(double));
    if (rc) return rc;
    HIPCHK(c, launch_fft_forward(tables(c), (const uint32_t *)c->s_a.p, (double *)c->s_tmp.p, R * 2, c->stream));
    std::vector<uint32_t> tv(2 * N);
    for (uint32_t x = 0; x < N; x++) {  // genTestvec (key.zig:134-145)
        tv[x] = 0;
        tv[N + x] = host::f64_to_torus(0.125);
    }
    uint32_t offset = 0;  // genDecompositionOffset (key.zig:121-131)
    for (uint32_t l = 0; l < L; l++) offset += ((1u << p.bgbit) / 2) * (1u << (32 - (l + 1) * p.bgbit));
    rc = set_key_common(c, offset, tv.data(), tv.data() + N);
    if (rc) return rc;
    HIPCHK(c, launch_bk_permute(c->K, (const double *)c->s_tmp.p, c->d_bk, R, c->stream));
    rc = upload_ksk(c, ksk.data());
    if (rc) return rc;
    if (bsk_out)
        HIPCHK(c, hipMemcpyAsync(bsk_out, c->s_tmp.p, R * 2 * N * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (ksk_out) std::memcpy(ksk_out, ksk.data(), ksk.size() * sizeof(uint32_t));
    c->has_key = true;
    c->key_from_keygen = true;
    return broadcast_key(c);
}

}  // extern "C"

namespace {

int ensure_pinned(tfhe_gpu_ctx *c, char *&p, size_t &have, size_t bytes) {
    if (have >= bytes) return TFHE_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    have = 0;
    HIPCHK(c, hipHostMalloc((void **)&p, bytes, hipHostMallocDefault));
    have = bytes;
    return TFHE_OK;
}

// Host-buffer bootstrap of B >= one whole-form round, pipelined (DESIGN.md
// §2.1): the batch is cut into chunks of #CUs items (a quarter round: #CUs/4
// workgroups of the whole form).  Worker s owns stream s and chunks s, s+S, ...;
// per chunk it copies the caller's inputs into pinned staging, then enqueues
// H2D -> blind rotation (whole form; the guard's recompute) -> key switch ->
// D2H on its stream, so chunk k+1's copies run while chunks <= k compute and
// the S streams' kernels share the CUs.  Each worker then waits for its stream
// and copies its chunks' outputs to the caller.  ops / b / tv_dev may be NULL.
int pipelined_bootstrap(tfhe_gpu_ctx *c, const uint8_t *ops, const uint32_t *a, const uint32_t *b,
                        const uint32_t *tv_dev, uint32_t *out, size_t B) {
    const size_t w = tlwe0_words(c), wb = w * 4, chunk = device_cus();
    const size_t nch = (B + chunk - 1) / chunk;
    const int S = (int)std::min<size_t>(PIPE_STREAMS, nch);
    // staging layout per item: op byte region, then a, then b (all chunks contiguous)
    const size_t ops_bytes = ops ? (B + 15) / 16 * 16 : 0, a_bytes = B * wb, b_bytes = b ? B * wb : 0;
    int rc = ensure_pinned(c, c->pin_in, c->pin_in_bytes, ops_bytes + a_bytes + b_bytes);
    if (!rc) rc = ensure_pinned(c, c->pin_out, c->pin_out_bytes, B * wb);
    if (!rc && ops) rc = ensure(c, c->s_ops, B);
    if (!rc) rc = ensure(c, c->s_a, B * wb);
    if (!rc && b) rc = ensure(c, c->s_b, B * wb);
    if (!rc) rc = ensure(c, c->s_out, B * wb);
    if (!rc) rc = ensure(c, c->s_lv1, B * 1025 * sizeof(uint32_t));
    if (rc) return rc;
    if (c->s_ties.bytes < B) {
        rc = ensure(c, c->s_ties, B);
        if (rc) return rc;
        HIPCHK(c, hipMemsetAsync(c->s_ties.p, 0, c->s_ties.bytes, c->stream));
    }
    if (!c->pipe_ev) HIPCHK(c, hipEventCreateWithFlags(&c->pipe_ev, hipEventDisableTiming));
    for (hipStream_t &p : c->pipe)
        if (!p) HIPCHK(c, hipStreamCreateWithFlags(&p, hipStreamNonBlocking));
    if (!c->workers) c->workers.reset(new WorkerPool(PIPE_STREAMS));
    // the GEMM key switch per chunk (the default form where it applies): its MFMA-layout
    // key is built once on the context stream, and each stream gets its own
    // partial-sum buffer, so every chunk runs the same key-switch form as the
    // unpipelined path (last_kernels names it)
    KsGemm G;
    rc = ks_gemm_args(c, chunk, G);
    if (rc) return rc;
    std::vector<KsGemm> Gs(S, G);
    if (G.kg) {
        const size_t pb = ks_gemm_part_bytes(c->K, chunk, 1024, c->K.basebit);
        rc = ensure(c, c->s_kspart, pb * S);
        if (rc) return rc;
        for (int s = 0; s < S; s++) Gs[s].part = (uint32_t *)((char *)c->s_kspart.p + (size_t)s * pb);
    }
    // everything enqueued on the context stream (key loads, the flags' memset) first
    HIPCHK(c, hipEventRecord(c->pipe_ev, c->stream));
    LaunchOpts o = c->opts;
    if (!o.br_form) o.br_form = 1;  // whole form for every chunk (a chunk is a quarter round)
    char *pin_ops = c->pin_in, *pin_a = c->pin_in + ops_bytes, *pin_b = pin_a + a_bytes;
    uint8_t *d_ops = (uint8_t *)c->s_ops.p;
    uint32_t *d_a = (uint32_t *)c->s_a.p, *d_b = (uint32_t *)c->s_b.p, *d_out = (uint32_t *)c->s_out.p;
    uint32_t *d_lv1 = (uint32_t *)c->s_lv1.p;
    std::vector<hipError_t> err(S, hipSuccess);
    std::vector<const char *> where(S, "");
    c->workers->run(S, [&](int s) {
        hipStream_t st = c->pipe[s];
        auto chk = [&](hipError_t e, const char *what) {
            if (e != hipSuccess && err[s] == hipSuccess) {
                err[s] = e;
                where[s] = what;
            }
            return e == hipSuccess;
        };
        if (!chk(hipSetDevice(c->device), "hipSetDevice") || !chk(hipStreamWaitEvent(st, c->pipe_ev, 0), "hipStreamWaitEvent"))
            return;
        for (size_t k = (size_t)s; k < nch; k += (size_t)S) {
            const size_t k0 = k * chunk, n = std::min(B, k0 + chunk) - k0;
            if (ops) std::memcpy(pin_ops + k0, ops + k0, n);
            std::memcpy(pin_a + k0 * wb, a + k0 * w, n * wb);
            if (b) std::memcpy(pin_b + k0 * wb, b + k0 * w, n * wb);
            if (ops && !chk(hipMemcpyAsync(d_ops + k0, pin_ops + k0, n, hipMemcpyHostToDevice, st), "H2D ops")) return;
            if (!chk(hipMemcpyAsync(d_a + k0 * w, pin_a + k0 * wb, n * wb, hipMemcpyHostToDevice, st), "H2D a")) return;
            if (b && !chk(hipMemcpyAsync(d_b + k0 * w, pin_b + k0 * wb, n * wb, hipMemcpyHostToDevice, st), "H2D b"))
                return;
            KParams K = c->K;
            K.tie_flags = (uint8_t *)c->s_ties.p + k0;
            if (!chk(launch_blind_rotate(K, tables(c), ops ? d_ops + k0 : nullptr, d_a + k0 * w, b ? d_b + k0 * w : nullptr,
                                         nullptr, tv_dev ? tv_dev : c->d_testvec, c->d_bk, d_lv1 + k0 * 1025, BR_OUT_LV1,
                                         n, st, o, s == 0 && k == 0 ? &c->last_br : nullptr),
                     "blind rotation") ||
                !chk(launch_key_switch(c->K, d_lv1 + k0 * 1025, c->d_ksk, d_out + k0 * w, n, st, c->opts,
                                       s == 0 && k == 0 ? &c->last_ks : nullptr, &Gs[s]),
                     "key switch") ||
                !chk(hipMemcpyAsync(c->pin_out + k0 * wb, d_out + k0 * w, n * wb, hipMemcpyDeviceToHost, st), "D2H"))
                return;
        }
        if (!chk(hipStreamSynchronize(st), "hipStreamSynchronize")) return;
        for (size_t k = (size_t)s; k < nch; k += (size_t)S) {
            const size_t k0 = k * chunk, n = std::min(B, k0 + chunk) - k0;
            std::memcpy(out + k0 * w, c->pin_out + k0 * wb, n * wb);
        }
    });
    for (int s = 0; s < S; s++)
        if (err[s] != hipSuccess) {
            for (int t = 0; t < S; t++) (void)hipStreamSynchronize(c->pipe[t]);
            return hip_fail(c, err[s], where[s]);
        }
    c->bootstraps += B;
    return sync_check(c);  // the device error word (and the recompute counter) after all streams
}

// The pipeline serves host-buffer bootstraps of at least one whole-form round
// (4 x #CUs items) unless TFHE_OPT_HOST_PIPELINE = 0 or device timing is on
// (its events bracket single launches on the context stream).
bool use_pipeline(const tfhe_gpu_ctx *c, size_t B) {
    return c->pipeline && !c->profiling && B >= 4 * device_cus();
}

}  // namespace

extern "C" {

static int bootstrap_batch_one(tfhe_gpu_ctx *c, const uint32_t *in, uint32_t *out, size_t B) {
    if (!c || (B && (!in || !out))) return fail(c, TFHE_ERR_INVALID, "null argument");
    if (B == 0) return TFHE_OK;
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->has_key) return fail(c, TFHE_ERR_NO_KEY, "no cloud key loaded");
    if (use_pipeline(c, B)) return pipelined_bootstrap(c, nullptr, in, nullptr, nullptr, out, B);
    const size_t w = tlwe0_words(c);
    int rc = h2d(c, c->s_a, in, B * w * 4);
    if (!rc) rc = ensure(c, c->s_out, B * w * 4);
    if (!rc) rc = run_bootstrap_dev(c, nullptr, (const uint32_t *)c->s_a.p, nullptr, nullptr, (uint32_t *)c->s_out.p, B, RUN_BOOTSTRAP);
    if (!rc) rc = d2h_sync(c, out, c->s_out.p, B * w * 4);
    return rc;
}

static int bootstrap_without_key_switch_batch_one(tfhe_gpu_ctx *c, const uint32_t *in, uint32_t *out, size_t B) {
    if (!c || (B && (!in || !out))) return fail(c, TFHE_ERR_INVALID, "null argument");
    if (B == 0) return TFHE_OK;
    HIPCHK(c, hipSetDevice(c->device));
    const size_t w = tlwe0_words(c);
    int rc = h2d(c, c->s_a, in, B * w * 4);
    if (!rc) rc = ensure(c, c->s_out, B * w * 4);
    if (!rc) rc = run_bootstrap_dev(c, nullptr, (const uint32_t *)c->s_a.p, nullptr, nullptr, (uint32_t *)c->s_out.p, B, RUN_NO_KEYSWITCH);
    if (!rc) rc = d2h_sync(c, out, c->s_out.p, B * w * 4);
    return rc;
}

static int gate_batch_one(tfhe_gpu_ctx *c, const uint8_t *ops, const uint32_t *a, const uint32_t *b, uint32_t *out,
                        size_t B) {
    if (!c || (B && (!ops || !a || !b || !out))) return fail(c, TFHE_ERR_INVALID, "null argument");
    if (B == 0) return TFHE_OK;
    for (size_t i = 0; i < B; i++)
        if (ops[i] > TFHE_GATE_ORYN && ops[i] != TFHE_GATE_COPY) return fail(c, TFHE_ERR_INVALID, "bad gate op");
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->has_key) return fail(c, TFHE_ERR_NO_KEY, "no cloud key loaded");
    if (use_pipeline(c, B)) return pipelined_bootstrap(c, ops, a, b, nullptr, out, B);
    const size_t w = tlwe0_words(c);
    int rc = h2d(c, c->s_ops, ops, B);
    if (!rc) rc = h2d(c, c->s_a, a, B * w * 4);
    if (!rc) rc = h2d(c, c->s_b, b, B * w * 4);
    if (!rc) rc = ensure(c, c->s_out, B * w * 4);
    if (!rc)
        rc = run_bootstrap_dev(c, (const uint8_t *)c->s_ops.p, (const uint32_t *)c->s_a.p, (const uint32_t *)c->s_b.p,
                               nullptr, (uint32_t *)c->s_out.p, B, RUN_BOOTSTRAP);
    if (!rc) rc = d2h_sync(c, out, c->s_out.p, B * w * 4);
    return rc;
}

static int blind_rotate_batch_one(tfhe_gpu_ctx *c, const uint32_t *in, const uint32_t *testvec, uint32_t *trlwe_out,
                                size_t B) {
    if (!c || (B && (!in || !trlwe_out))) return fail(c, TFHE_ERR_INVALID, "null argument");
    if (B == 0) return TFHE_OK;
    HIPCHK(c, hipSetDevice(c->device));
    const size_t w = tlwe0_words(c);
    int rc = h2d(c, c->s_a, in, B * w * 4);
    const uint32_t *tv = nullptr;
    if (!rc && testvec) {
        rc = h2d(c, c->s_tv, testvec, 2 * c->P.N * 4);
        tv = (const uint32_t *)c->s_tv.p;
    }
    if (!rc) rc = ensure(c, c->s_out, B * 2 * c->P.N * 4);
    if (!rc) rc = run_bootstrap_dev(c, nullptr, (const uint32_t *)c->s_a.p, nullptr, tv, (uint32_t *)c->s_out.p, B, RUN_TRLWE);
    if (!rc) rc = d2h_sync(c, trlwe_out, c->s_out.p, B * 2 * c->P.N * 4);
    return rc;
}

static int bootstrap_lut_batch_one(tfhe_gpu_ctx *c, const uint32_t *in, const uint32_t *testvec, uint32_t *out,
                                 size_t B) {
    if (!c || !testvec || (B && (!in || !out))) return fail(c, TFHE_ERR_INVALID, "null argument");
    if (B == 0) return TFHE_OK;
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->has_key) return fail(c, TFHE_ERR_NO_KEY, "no cloud key loaded");
    const size_t w = tlwe0_words(c);
    int rc = h2d(c, c->s_tv, testvec, 2 * c->P.N * 4);
    if (rc) return rc;
    if (use_pipeline(c, B)) return pipelined_bootstrap(c, nullptr, in, nullptr, (const uint32_t *)c->s_tv.p, out, B);
    rc = h2d(c, c->s_a, in, B * w * 4);
    if (!rc) rc = ensure(c, c->s_out, B * w * 4);
    if (!rc)
        rc = run_bootstrap_dev(c, nullptr, (const uint32_t *)c->s_a.p, nullptr, (const uint32_t *)c->s_tv.p,
                               (uint32_t *)c->s_out.p, B, RUN_BOOTSTRAP);
    if (!rc) rc = d2h_sync(c, out, c->s_out.p, B * w * 4);
    return rc;
}

// ---- Proxy re-encryption ------------------------------------
}  // extern "C"

struct tfhe_gpu_reenc_key {
    int device = 0;
    uint32_t basebit = 0, t = 0;
    uint32_t *d_key = nullptr;  // padded rows like the KSK (K.ks_stride words) + zero tail
    uint32_t *d_key_gemm = nullptr;  // the gemm key switch's layout of d_key (basebit 2, t 7..9), or NULL
    std::vector<tfhe_gpu_reenc_key *> peers;  // multi-device context: the copy on shard k is peers[k - 1]
};

extern "C" {

static int reenc_key_load_one(tfhe_gpu_ctx *c, const uint32_t *key_encryptions, size_t len, uint32_t basebit,
                            uint32_t t, tfhe_gpu_reenc_key **out) {
    if (!c || !key_encryptions || !out) return fail(c, TFHE_ERR_INVALID, "null argument");
    const size_t n = c->P.n, rows = n * t * ((size_t)1 << basebit);
    if (basebit < 1 || basebit > 8 || t < 1 || basebit * t >= 31 || !reencrypt_supported((int)t, (int)basebit))
        return fail(c, TFHE_ERR_INVALID, "unsupported re-encryption base/levels");
    if (len != rows * (n + 1)) return fail(c, TFHE_ERR_INVALID, "len != n*t*2^basebit*(n+1)");
    HIPCHK(c, hipSetDevice(c->device));
    auto *k = new tfhe_gpu_reenc_key;
    k->device = c->device;
    k->basebit = basebit;
    k->t = t;
    const size_t stride = c->K.ks_stride, bytes = (rows * stride + KS_TAIL_WORDS) * sizeof(uint32_t);
    hipError_t e = hipMalloc((void **)&k->d_key, bytes);
    if (e != hipSuccess) {
        delete k;
        return fail(c, TFHE_ERR_OOM, "hipMalloc(reencryption key)");
    }
    e = hipMemsetAsync(k->d_key, 0, bytes, c->stream);
    if (e == hipSuccess)
        e = hipMemcpy2DAsync(k->d_key, stride * 4, key_encryptions, (n + 1) * 4, (n + 1) * 4, rows,
                             hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = launch_key_zero_k0(c->K, k->d_key, (int)n, (int)t, (int)basebit, c->stream);
    if (e == hipSuccess && ks_gemm_supported((int)t, (int)basebit)) {  // §4.4b layout for the gemm form
        e = hipMalloc((void **)&k->d_key_gemm, ks_gemm_bytes(c->K, (int)n, (int)t, (int)basebit));
        if (e == hipSuccess) e = launch_ksk_to_gemm(c->K, k->d_key, k->d_key_gemm, (int)n, (int)t, (int)basebit, c->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
        (void)hipFree(k->d_key);
        if (k->d_key_gemm) (void)hipFree(k->d_key_gemm);
        delete k;
        return hip_fail(c, e, "upload reencryption key");
    }
    *out = k;
    return TFHE_OK;
}

void tfhe_gpu_reenc_key_destroy(tfhe_gpu_reenc_key *k) {
    if (!k) return;
    for (tfhe_gpu_reenc_key *p : k->peers) tfhe_gpu_reenc_key_destroy(p);
    (void)hipSetDevice(k->device);
    (void)hipFree(k->d_key);
    if (k->d_key_gemm) (void)hipFree(k->d_key_gemm);
    delete k;
}

static int reencrypt_batch_one(tfhe_gpu_ctx *c, const tfhe_gpu_reenc_key *k, const uint32_t *in, uint32_t *out,
                             size_t B) {
    if (!c || !k || (B && (!in || !out))) return fail(c, TFHE_ERR_INVALID, "null argument");
    if (k->device != c->device) return fail(c, TFHE_ERR_INVALID, "key belongs to another device");
    if (B == 0) return TFHE_OK;
    HIPCHK(c, hipSetDevice(c->device));
    const size_t w = tlwe0_words(c);
    int rc = ensure(c, c->s_a, B * w * 4 + KS_GEMM_INPUT_SLACK);  // the gemm form reads whole blocks of 8
    if (!rc) rc = h2d(c, c->s_a, in, B * w * 4);
    if (!rc) rc = ensure(c, c->s_out, B * w * 4);
    if (rc) return rc;
    KsGemm G;
    if (k->d_key_gemm) {
        rc = ensure(c, c->s_kspart, ks_gemm_part_bytes(c->K, B, (int)c->P.n, (int)k->basebit));
        if (rc) return rc;
        G.kg = k->d_key_gemm;
        G.part = (uint32_t *)c->s_kspart.p;
    }
    HIPCHK(c, launch_reencrypt(c->K, (int)k->t, (int)k->basebit, (const uint32_t *)c->s_a.p, k->d_key,
                               (uint32_t *)c->s_out.p, B, c->stream, c->opts, &c->last_ks, &G));
    return d2h_sync(c, out, c->s_out.p, B * w * 4);
}

// Device-resident re-encryption (async on the context stream, like the other
// _dev entry points): the input is copied device-to-device into the staging
// buffer, whose slack the GEMM form's whole-block reads need; the kernel writes
// out_dev directly.
static int reencrypt_batch_dev_one(tfhe_gpu_ctx *c, const tfhe_gpu_reenc_key *k, const uint32_t *in_dev,
                                   uint32_t *out_dev, size_t B) {
    if (!c || !k || (B && (!in_dev || !out_dev))) return fail(c, TFHE_ERR_INVALID, "null argument");
    if (k->device != c->device) return fail(c, TFHE_ERR_INVALID, "key belongs to another device");
    if (B == 0) return TFHE_OK;
    HIPCHK(c, hipSetDevice(c->device));
    const size_t w = tlwe0_words(c);
    int rc = ensure(c, c->s_a, B * w * 4 + KS_GEMM_INPUT_SLACK);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(c->s_a.p, in_dev, B * w * 4, hipMemcpyDeviceToDevice, c->stream));
    KsGemm G;
    if (k->d_key_gemm) {
        rc = ensure(c, c->s_kspart, ks_gemm_part_bytes(c->K, B, (int)c->P.n, (int)k->basebit));
        if (rc) return rc;
        G.kg = k->d_key_gemm;
        G.part = (uint32_t *)c->s_kspart.p;
    }
    HIPCHK(c, launch_reencrypt(c->K, (int)k->t, (int)k->basebit, (const uint32_t *)c->s_a.p, k->d_key, out_dev, B,
                               c->stream, c->opts, &c->last_ks, &G));
    return TFHE_OK;
}

int tfhe_secret_key_new(const tfhe_params *p, uint64_t seed, uint32_t *key_lv0, uint32_t *key_lv1) {
    if (!p || !key_lv0 || !key_lv1) return TFHE_ERR_INVALID;
    host::Rng r(seed);  // SecretKey.new (key.zig:41-57)
    for (uint32_t i = 0; i < p->n; i++) key_lv0[i] = r.boolean() ? 1u : 0u;
    for (uint32_t i = 0; i < p->N; i++) key_lv1[i] = r.boolean() ? 1u : 0u;
    return TFHE_OK;
}

int tfhe_public_key_gen(const tfhe_params *p, const uint32_t *key, size_t size, double alpha, uint64_t seed0,
                        uint32_t *pk) {
    if (!p || !key || (size && !pk)) return TFHE_ERR_INVALID;
    for (size_t e = 0; e < size; e++) tlwe_encrypt(p->n, 0.0, alpha, key, seed0 + e, pk + e * (p->n + 1));
    return TFHE_OK;
}

int tfhe_public_key_encrypt_bool_batch(const tfhe_params *p, const uint32_t *pk, size_t pk_size, const uint8_t *bits,
                                       double alpha, uint64_t seed0, uint32_t *out, size_t B) {
    if (!p || (pk_size && !pk) || (B && (!bits || !out))) return TFHE_ERR_INVALID;
    for (size_t i = 0; i < B; i++)
        pk_encrypt(p->n, pk, pk_size, bits[i] ? 0.125 : -0.125, alpha, seed0 + i, out + i * (p->n + 1));
    return TFHE_OK;
}

int tfhe_reenc_key_gen_symmetric(const tfhe_params *p, const uint32_t *key_from, const uint32_t *key_to, double alpha,
                                 uint32_t basebit, uint32_t t, uint64_t seed0, uint32_t *out) {
    if (!p || !key_from || !key_to || !out || basebit < 1 || basebit > 8 || t < 1) return TFHE_ERR_INVALID;
    reenc_key_gen(p->n, key_from, basebit, t, seed0, out, [&](double v, uint64_t seed, uint32_t *o) {
        tlwe_encrypt(p->n, v, alpha, key_to, seed, o);
    });
    return TFHE_OK;
}

int tfhe_reenc_key_gen_asymmetric(const tfhe_params *p, const uint32_t *key_from, const uint32_t *pk, size_t pk_size,
                                  double alpha, uint32_t basebit, uint32_t t, uint64_t seed0, uint32_t *out) {
    if (!p || !key_from || !out || (pk_size && !pk) || basebit < 1 || basebit > 8 || t < 1) return TFHE_ERR_INVALID;
    reenc_key_gen(p->n, key_from, basebit, t, seed0, out, [&](double v, uint64_t seed, uint32_t *o) {
        pk_encrypt(p->n, pk, pk_size, v, alpha, seed, o);
    });
    return TFHE_OK;
}

// ---- Circuit evaluation with a level scheduler -------------
// Round packing.  A bootstrapped gate whose consumers all sit at least two
// levels later, and that feeds no NOT, can run one level later without
// changing the depth.  Levels are visited in ascending order; each moves to
// the next level the number of such gates that minimises the modelled
// blind-rotation time of the two levels (blind_rotate_cost: whole rounds of
// 4 x #CUs gates, a ragged tail in the latency form).  Example: a level of
// 10,256 gates hands 16 of them to the next level instead of running a
// 16-gate tail.  Moved gates may move again from their new level.
// TFHE_OPT_CIRCUIT_PACK = 0 turns packing off (A/B runs and tests).
static void pack_levels(size_t n_inputs, size_t n_gates, const uint8_t *ops, const uint32_t *in_a,
                        const uint32_t *in_b, size_t cus, std::vector<uint32_t> &level,
                        std::vector<std::vector<uint32_t>> &bs) {
    const size_t W = n_inputs + n_gates;
    const uint32_t max_level = (uint32_t)bs.size() - 1;
    // earliest level among each wire's bootstrapped consumers; NOT consumers pin it
    constexpr uint32_t PINNED = 0, FREE = 0xFFFFFFFFu;
    // (kept from the ASAP levels: moving a gate later only raises its inputs'
    // true first use, so the values stay safe)
    std::vector<uint32_t> first_use(W, FREE);
    for (size_t g = 0; g < n_gates; g++) {
        const bool two = ops[g] <= TFHE_GATE_ORYN;
        for (int k = 0; k < (two ? 2 : 1); k++) {
            const uint32_t src = k ? in_b[g] : in_a[g];
            if (ops[g] == TFHE_GATE_NOT) first_use[src] = PINNED;
            else if (first_use[src] != PINNED) first_use[src] = std::min(first_use[src], level[n_inputs + g]);
        }
    }
    const size_t R = 4 * cus;
    const size_t J = (512 + cus - 1) / cus + 1;  // tail breakpoints per round (multiples of #CUs)
    auto cost = [&](size_t b) { return blind_rotate_cost(b, cus); };
    std::vector<uint32_t> cand;
    for (uint32_t lv = 1; lv < max_level; lv++) {
        cand.clear();
        for (uint32_t g : bs[lv]) {
            const uint32_t u = first_use[n_inputs + g];
            if (u != PINNED && (u == FREE || u >= lv + 2)) cand.push_back(g);
        }
        if (cand.empty()) continue;
        const size_t c0 = bs[lv].size(), c1 = bs[lv + 1].size(), k = cand.size();
        // blind_rotate_cost(c0 - d) only drops where c0 - d reaches a breakpoint
        // m*R + j*#CUs, so those d (and d = 0) are the only candidates
        size_t best_d = 0;
        double best = cost(c0) + cost(c1);
        for (size_t m = (c0 - k) / R; m <= c0 / R; m++)
            for (size_t j = 0; j <= J; j++) {
                const size_t bp = m * R + j * cus;
                if (bp > c0 || bp + k < c0) continue;
                const size_t d = c0 - bp;
                const double cd = cost(bp) + cost(c1 + d);
                if (cd < best - 1e-9 || (cd < best + 1e-9 && d < best_d)) {
                    best = cd;
                    best_d = d;
                }
            }
        if (best_d == 0) continue;
        // move the last best_d candidates (those of the latest gates); their
        // consumers are at lv + 2 or later, their inputs only gain slack
        for (size_t x = k - best_d; x < k; x++) {
            level[n_inputs + cand[x]] = lv + 1;
            bs[lv + 1].push_back(cand[x]);
        }
        std::vector<uint32_t> keep;
        keep.reserve(c0 - best_d);
        for (uint32_t g : bs[lv])
            if (level[n_inputs + g] == lv) keep.push_back(g);
        bs[lv].swap(keep);
    }
}

// Wire w < n_inputs is input w; gate g drives wire n_inputs + g.  A
// bootstrapped gate is ready one level after the later of its inputs; a NOT
// (negation) is ready with its input.  Fills level[] (per wire), the depth and
// the bootstrapped / NOT gates of every level (packed unless `pack` is false);
// returns nullptr, or the reason the graph is invalid.
static const char *schedule_levels(size_t n_inputs, size_t n_gates, const uint8_t *ops, const uint32_t *in_a,
                                   const uint32_t *in_b, bool pack, size_t cus, std::vector<uint32_t> &level,
                                   uint32_t &max_level, std::vector<std::vector<uint32_t>> &bs,
                                   std::vector<std::vector<uint32_t>> &nots) {
    level.assign(n_inputs + n_gates, 0);
    max_level = 0;
    for (size_t g = 0; g < n_gates; g++) {
        const size_t w = n_inputs + g;
        const int op = ops[g];
        const bool bootstrapped = op <= TFHE_GATE_ORYN || op == TFHE_GATE_COPY;
        if (!bootstrapped && op != TFHE_GATE_NOT) return "unknown gate op";
        if (in_a[g] >= w) return "gate input a is not an earlier wire";
        const bool two = op <= TFHE_GATE_ORYN;
        if (two && in_b[g] >= w) return "gate input b is not an earlier wire";
        uint32_t r = level[in_a[g]];
        if (two) r = std::max(r, level[in_b[g]]);
        level[w] = bootstrapped ? r + 1 : r;
        max_level = std::max(max_level, level[w]);
    }
    // groups in evaluation order: NOT(0), BS(1), NOT(1), ..., BS(max), NOT(max)
    bs.assign(max_level + 1, {});
    nots.assign(max_level + 1, {});
    for (size_t g = 0; g < n_gates; g++) {
        const uint32_t lv = level[n_inputs + g];
        (ops[g] == TFHE_GATE_NOT ? nots[lv] : bs[lv]).push_back((uint32_t)g);
    }
    if (pack && max_level > 1) pack_levels(n_inputs, n_gates, ops, in_a, in_b, cus, level, bs);
    return nullptr;
}

int tfhe_circuit_schedule(size_t n_inputs, size_t n_gates, const uint8_t *ops, const uint32_t *in_a,
                          const uint32_t *in_b, uint32_t cus, int pack, uint32_t *levels, uint32_t *depth) {
    if ((n_gates && (!ops || !in_a || !in_b || !levels)) || cus == 0) return TFHE_ERR_INVALID;
    if (n_inputs + n_gates > 0xFFFFFFFFull) return TFHE_ERR_INVALID;
    std::vector<uint32_t> level;
    std::vector<std::vector<uint32_t>> bs, nots;
    uint32_t max_level = 0;
    if (schedule_levels(n_inputs, n_gates, ops, in_a, in_b, pack != 0, cus, level, max_level, bs, nots))
        return TFHE_ERR_INVALID;
    for (size_t g = 0; g < n_gates; g++) levels[g] = level[n_inputs + g];
    if (depth) *depth = max_level;
    return TFHE_OK;
}

}  // extern "C"

namespace {

// A circuit's evaluation plan: the level schedule and the device wire table
// laid out in evaluation order — inputs | NOTs of level 0 | gates of level 1 |
// NOTs of level 1 | ... — so each level's batch writes one contiguous run of
// slots; its inputs are gathered by index inside the blind-rotation prologue.
// idx / cops: per-group gather indices and op codes, concatenated in
// evaluation order, then the output wires' slots.
struct CircuitPlan {
    std::vector<std::vector<uint32_t>> bs, nots;
    uint32_t max_level = 0;
    std::vector<uint32_t> idx;
    std::vector<uint8_t> cops;
};

const char *plan_circuit(size_t n_inputs, size_t n_gates, const uint8_t *ops, const uint32_t *in_a,
                         const uint32_t *in_b, size_t n_outputs, const uint32_t *out_wires, bool pack, size_t cus,
                         CircuitPlan &pl) {
    const size_t W = n_inputs + n_gates;
    if (W > 0xFFFFFFFFull) return "too many wires";
    std::vector<uint32_t> ready;
    if (const char *why = schedule_levels(n_inputs, n_gates, ops, in_a, in_b, pack, cus, ready, pl.max_level, pl.bs,
                                          pl.nots))
        return why;
    for (size_t o = 0; o < n_outputs; o++)
        if (out_wires[o] >= W) return "output wire out of range";
    std::vector<uint32_t> slot(W);
    for (size_t w = 0; w < n_inputs; w++) slot[w] = (uint32_t)w;
    uint32_t next = (uint32_t)n_inputs;
    for (uint32_t lv = 0; lv <= pl.max_level; lv++) {
        for (uint32_t g : pl.bs[lv]) slot[n_inputs + g] = next++;
        for (uint32_t g : pl.nots[lv]) slot[n_inputs + g] = next++;
    }
    pl.idx.clear();
    pl.cops.clear();
    pl.idx.reserve(2 * n_gates + n_outputs);
    for (uint32_t lv = 0; lv <= pl.max_level; lv++) {
        for (uint32_t g : pl.bs[lv]) {
            const bool two = ops[g] <= TFHE_GATE_ORYN;
            pl.idx.push_back(slot[in_a[g]]);
            pl.idx.push_back(two ? slot[in_b[g]] : slot[in_a[g]]);
            pl.cops.push_back(ops[g]);
        }
        for (uint32_t g : pl.nots[lv]) pl.idx.push_back(slot[in_a[g]]);
    }
    for (size_t o = 0; o < n_outputs; o++) pl.idx.push_back(slot[out_wires[o]]);
    return nullptr;
}

// Device side of a plan on one context: wire table with the inputs, the gather
// indices and op codes, uploaded on its stream.
int upload_plan(tfhe_gpu_ctx *c, const CircuitPlan &pl, size_t W, size_t n_inputs, const uint32_t *inputs,
                size_t n_outputs, bool inputs_on_device = false) {
    const size_t w1 = tlwe0_words(c);
    HIPCHK(c, hipSetDevice(c->device));
    int rc = ensure(c, c->s_wires, std::max<size_t>(W, 1) * w1 * 4);
    if (!rc) rc = ensure(c, c->s_cidx, std::max<size_t>(pl.idx.size(), 1) * 4);
    if (!rc) rc = ensure(c, c->s_cops, std::max<size_t>(pl.cops.size(), 1));
    if (!rc) rc = ensure(c, c->s_out, std::max<size_t>(n_outputs, 1) * w1 * 4);
    if (rc) return rc;
    if (n_inputs)
        HIPCHK(c, hipMemcpyAsync(c->s_wires.p, inputs, n_inputs * w1 * 4,
                                 inputs_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream));
    // the plan vectors are pageable: hipMemcpyAsync stages them before it returns, so the caller
    // may drop `pl` while the copies are still in flight (the _dev circuit call does not sync)
    if (!pl.idx.empty())
        HIPCHK(c, hipMemcpyAsync(c->s_cidx.p, pl.idx.data(), pl.idx.size() * 4, hipMemcpyHostToDevice, c->stream));
    if (!pl.cops.empty())
        HIPCHK(c, hipMemcpyAsync(c->s_cops.p, pl.cops.data(), pl.cops.size(), hipMemcpyHostToDevice, c->stream));
    return TFHE_OK;
}

}  // namespace

extern "C" {

// dev: inputs and outputs are device pointers (tfhe_gpu_circuit_eval_dev): the inputs are copied
// device-to-device into the wire table, the outputs gathered straight into `outputs`, and the call
// returns without waiting (async on the context stream, like the other _dev entries)
static int circuit_eval_one(tfhe_gpu_ctx *c, size_t n_inputs, const uint32_t *inputs, size_t n_gates,
                          const uint8_t *ops, const uint32_t *in_a, const uint32_t *in_b, size_t n_outputs,
                          const uint32_t *out_wires, uint32_t *outputs, uint32_t *levels_out, bool dev = false) {
    if (!c || (n_inputs && !inputs) || (n_gates && (!ops || !in_a || !in_b)) || (n_outputs && (!out_wires || !outputs)))
        return fail(c, TFHE_ERR_INVALID, "null argument");
    if (!c->has_key) return fail(c, TFHE_ERR_NO_KEY, "no cloud key loaded");
    const size_t W = n_inputs + n_gates, w1 = tlwe0_words(c);
    HIPCHK(c, hipSetDevice(c->device));
    CircuitPlan pl;
    if (const char *why = plan_circuit(n_inputs, n_gates, ops, in_a, in_b, n_outputs, out_wires, c->circuit_pack != 0,
                                       device_cus(), pl))
        return fail(c, TFHE_ERR_INVALID, why);
    int rc = upload_plan(c, pl, W, n_inputs, inputs, n_outputs, dev);
    if (rc) return rc;
    const auto &bs = pl.bs;
    const auto &nots = pl.nots;
    const uint32_t max_level = pl.max_level;
    uint32_t *wires = (uint32_t *)c->s_wires.p;
    const uint32_t *d_idx = (const uint32_t *)c->s_cidx.p;
    const uint8_t *d_ops = (const uint8_t *)c->s_cops.p;
    size_t ip = 0, op_pos = 0, sp = n_inputs;
    for (uint32_t lv = 0; lv <= max_level; lv++) {
        const size_t nb = bs[lv].size(), nn = nots[lv].size();
        if (nb) {
            rc = run_bootstrap_dev(c, d_ops + op_pos, wires, wires, nullptr, wires + sp * w1, nb, RUN_BOOTSTRAP,
                                   d_idx + ip);
            if (rc) return rc;
            ip += 2 * nb;
            op_pos += nb;
            sp += nb;
        }
        if (nn) {
            HIPCHK(c, launch_tlwe_gather(c->K, wires, d_idx + ip, wires + sp * w1, nn, true, c->stream));
            ip += nn;
            sp += nn;
        }
    }
    if (n_outputs && dev) {
        HIPCHK(c, launch_tlwe_gather(c->K, wires, d_idx + ip, outputs, n_outputs, false, c->stream));
    } else if (n_outputs) {
        HIPCHK(c, launch_tlwe_gather(c->K, wires, d_idx + ip, (uint32_t *)c->s_out.p, n_outputs, false, c->stream));
        rc = d2h_sync(c, outputs, c->s_out.p, n_outputs * w1 * 4);
        if (rc) return rc;
    } else if (dev) {
    } else {
        rc = sync_check(c);
        if (rc) return rc;
    }
    if (levels_out) *levels_out = max_level;
    return TFHE_OK;
}

int tfhe_gpu_gate_batch_dev(tfhe_gpu_ctx *c, const uint8_t *ops_dev, const uint32_t *a_dev, const uint32_t *b_dev,
                            uint32_t *out_dev, size_t B) {
    if (!c || (B && (!ops_dev || !a_dev || !b_dev || !out_dev))) return fail(c, TFHE_ERR_INVALID, "null argument");
    HIPCHK(c, hipSetDevice(c->device));
    return run_bootstrap_dev(c, ops_dev, a_dev, b_dev, nullptr, out_dev, B, RUN_BOOTSTRAP);
}

int tfhe_gpu_bootstrap_batch_dev(tfhe_gpu_ctx *c, const uint32_t *in_dev, uint32_t *out_dev, size_t B) {
    if (!c || (B && (!in_dev || !out_dev))) return fail(c, TFHE_ERR_INVALID, "null argument");
    HIPCHK(c, hipSetDevice(c->device));
    return run_bootstrap_dev(c, nullptr, in_dev, nullptr, nullptr, out_dev, B, RUN_BOOTSTRAP);
}

int tfhe_gpu_bootstrap_lut_batch_dev(tfhe_gpu_ctx *c, const uint32_t *in_dev, const uint32_t *testvec_dev,
                                     uint32_t *out_dev, size_t B) {
    if (!c || !testvec_dev || (B && (!in_dev || !out_dev))) return fail(c, TFHE_ERR_INVALID, "null argument");
    if (is_multi(c)) return fail(c, TFHE_ERR_INVALID, "device-resident calls take a single-device context");
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->has_key) return fail(c, TFHE_ERR_NO_KEY, "no cloud key loaded");
    return run_bootstrap_dev(c, nullptr, in_dev, nullptr, testvec_dev, out_dev, B, RUN_BOOTSTRAP);
}

int tfhe_gpu_profile_begin(tfhe_gpu_ctx *c) {
    if (!c) return TFHE_ERR_INVALID;
    c->profiling = true;
    c->ev_used = 0;
    return TFHE_OK;
}

int tfhe_gpu_profile_end(tfhe_gpu_ctx *c, double *br_ms, double *ks_ms, int *launches) {
    if (!c) return TFHE_ERR_INVALID;
    c->profiling = false;
    const int rc = sync_check(c);
    if (rc) {
        c->ev_used = 0;
        return rc;
    }
    double br = 0.0, ks = 0.0;
    for (size_t i = 0; i + 3 <= c->ev_used; i += 3) {
        float a = 0.f, b = 0.f;
        HIPCHK(c, hipEventElapsedTime(&a, c->events[i], c->events[i + 1]));
        HIPCHK(c, hipEventElapsedTime(&b, c->events[i + 1], c->events[i + 2]));
        br += a;
        ks += b;
    }
    if (br_ms) *br_ms = br;
    if (ks_ms) *ks_ms = ks;
    if (launches) *launches = (int)(c->ev_used / 3);
    c->ev_used = 0;
    return TFHE_OK;
}

int tfhe_gpu_fft_forward_batch(tfhe_gpu_ctx *c, const uint32_t *in, double *out, size_t B) {
    if (!c || (B && (!in || !out))) return fail(c, TFHE_ERR_INVALID, "null argument");
    if (B == 0) return TFHE_OK;
    HIPCHK(c, hipSetDevice(c->device));
    int rc = h2d(c, c->s_a, in, B * 1024 * 4);
    if (!rc) rc = ensure(c, c->s_tmp, B * 1024 * 8);
    if (rc) return rc;
    HIPCHK(c, launch_fft_forward(tables(c), (const uint32_t *)c->s_a.p, (double *)c->s_tmp.p, B, c->stream));
    return d2h_sync(c, out, c->s_tmp.p, B * 1024 * 8);
}

int tfhe_gpu_fft_inverse_batch(tfhe_gpu_ctx *c, const double *in, uint32_t *out, size_t B) {
    if (!c || (B && (!in || !out))) return fail(c, TFHE_ERR_INVALID, "null argument");
    if (B == 0) return TFHE_OK;
    HIPCHK(c, hipSetDevice(c->device));
    int rc = h2d(c, c->s_tmp, in, B * 1024 * 8);
    if (!rc) rc = ensure(c, c->s_out, B * 1024 * 4);
    if (rc) return rc;
    HIPCHK(c, launch_fft_inverse(tables(c), (const double *)c->s_tmp.p, (uint32_t *)c->s_out.p, B, c->stream));
    return d2h_sync(c, out, c->s_out.p, B * 1024 * 4);
}

int tfhe_gpu_poly_mul_batch(tfhe_gpu_ctx *c, const uint32_t *a, const uint32_t *b, uint32_t *out, size_t B) {
    if (!c || (B && (!a || !b || !out))) return fail(c, TFHE_ERR_INVALID, "null argument");
    if (B == 0) return TFHE_OK;
    HIPCHK(c, hipSetDevice(c->device));
    int rc = h2d(c, c->s_a, a, B * 1024 * 4);
    if (!rc) rc = h2d(c, c->s_b, b, B * 1024 * 4);
    if (!rc) rc = ensure(c, c->s_out, B * 1024 * 4);
    if (rc) return rc;
    HIPCHK(c, launch_poly_mul(tables(c), (const uint32_t *)c->s_a.p, (const uint32_t *)c->s_b.p, 1024,
                              (uint32_t *)c->s_out.p, B, c->stream));
    return d2h_sync(c, out, c->s_out.p, B * 1024 * 4);
}

int tfhe_gpu_external_product_batch(tfhe_gpu_ctx *c, const double *trgsw_fft, uint32_t bk_index,
                                    const uint32_t *in, uint32_t *out, size_t B) {
    if (!c || (B && (!in || !out))) return fail(c, TFHE_ERR_INVALID, "null argument");
    if (B == 0) return TFHE_OK;
    HIPCHK(c, hipSetDevice(c->device));
    const size_t row_d = (size_t)2 * c->P.L * 2048;  // doubles per TRGSW
    const double *row = nullptr;
    int rc = TFHE_OK;
    if (trgsw_fft) {
        rc = h2d(c, c->s_tmp, trgsw_fft, row_d * 8);
        if (!rc) rc = ensure(c, c->s_tv, row_d * 8);
        if (rc) return rc;
        HIPCHK(c, launch_bk_permute(c->K, (const double *)c->s_tmp.p, (double *)c->s_tv.p, 2 * c->P.L, c->stream));
        row = (const double *)c->s_tv.p;
        if (c->K.offset == 0) {  // no key loaded yet: use the parameter set's offset
            uint32_t off = 0;
            for (uint32_t l = 0; l < c->P.L; l++)
                off += ((1u << c->P.bgbit) / 2) * (1u << (32 - (l + 1) * c->P.bgbit));
            c->K.offset = off;
        }
    } else {
        if (!c->has_key) return fail(c, TFHE_ERR_NO_KEY, "no cloud key loaded");
        if (bk_index >= c->P.n) return fail(c, TFHE_ERR_INVALID, "bk_index >= n");
        row = c->d_bk + (size_t)bk_index * row_d;
    }
    rc = h2d(c, c->s_a, in, B * 2048 * 4);
    if (!rc) rc = ensure(c, c->s_out, B * 2048 * 4);
    if (rc) return rc;
    HIPCHK(c, launch_external_product(c->K, tables(c), row, (const uint32_t *)c->s_a.p, (uint32_t *)c->s_out.p, B,
                                      c->stream));
    return d2h_sync(c, out, c->s_out.p, B * 2048 * 4);
}

static int key_switch_batch_one(tfhe_gpu_ctx *c, const uint32_t *in_lv1, uint32_t *out_lv0, size_t B) {
    if (!c || (B && (!in_lv1 || !out_lv0))) return fail(c, TFHE_ERR_INVALID, "null argument");
    if (!c->has_key) return fail(c, TFHE_ERR_NO_KEY, "no cloud key loaded");
    if (B == 0) return TFHE_OK;
    HIPCHK(c, hipSetDevice(c->device));
    const size_t w = tlwe0_words(c);
    int rc = h2d(c, c->s_lv1, in_lv1, B * 1025 * 4);
    if (!rc) rc = ensure(c, c->s_out, B * w * 4);
    if (rc) return rc;
    KsGemm G;
    if ((rc = ks_gemm_args(c, B, G))) return rc;
    HIPCHK(c, launch_key_switch(c->K, (const uint32_t *)c->s_lv1.p, c->d_ksk, (uint32_t *)c->s_out.p, B, c->stream,
                                c->opts, &c->last_ks, &G));
    return d2h_sync(c, out_lv0, c->s_out.p, B * w * 4);
}

// ---- host-side TLWELv0 helpers ------------------------------------------
int tfhe_encrypt_bool_batch(const tfhe_params *p, const uint32_t *key, const uint8_t *bits, uint64_t seed0,
                            uint32_t *out, size_t B) {
    if (!p || !key || (B && (!bits || !out))) return TFHE_ERR_INVALID;
    for (size_t i = 0; i < B; i++)
        tlwe_encrypt(p->n, bits[i] ? 0.125 : -0.125, p->alpha_lv0, key, seed0 + i, out + i * (p->n + 1));
    return TFHE_OK;
}

int tfhe_decrypt_bool_batch(const tfhe_params *p, const uint32_t *key, const uint32_t *ct, uint8_t *bits, size_t B) {
    if (!p || !key || (B && (!bits || !ct))) return TFHE_ERR_INVALID;
    for (size_t i = 0; i < B; i++) bits[i] = (int32_t)tlwe_phase(p->n, ct + i * (p->n + 1), key) >= 0;
    return TFHE_OK;
}

int tfhe_encrypt_lwe_message_batch(const tfhe_params *p, const uint32_t *key, const uint32_t *msgs, uint32_t m,
                                   uint64_t seed0, uint32_t *out, size_t B) {
    if (!p || !key || m == 0 || (B && (!msgs || !out))) return TFHE_ERR_INVALID;
    const double scale = 1.0 / (2.0 * (double)m);
    for (size_t i = 0; i < B; i++)
        tlwe_encrypt(p->n, (double)(msgs[i] % m) * scale, p->alpha_lv0, key, seed0 + i, out + i * (p->n + 1));
    return TFHE_OK;
}

int tfhe_decrypt_lwe_message_batch(const tfhe_params *p, const uint32_t *key, const uint32_t *ct, uint32_t m,
                                   uint32_t *msgs, size_t B) {
    if (!p || !key || m == 0 || (B && (!msgs || !ct))) return TFHE_ERR_INVALID;
    const double scale = 1.0 / (2.0 * (double)m);
    for (size_t i = 0; i < B; i++) {
        double f = (double)tlwe_phase(p->n, ct + i * (p->n + 1), key) / 4294967296.0;
        msgs[i] = (uint32_t)((uint64_t)(f / scale + 0.5) % m);
    }
    return TFHE_OK;
}

// generateLookupTableFullAssign (lut/generator.zig:155-191): message x's range
// [divRound(xN, m), divRound((x+1)N, m)) of the raw table holds values[x]; the
// table is rotated by divRound(N, 2m), its last divRound(N, 2m) entries negated,
// and stored as the b polynomial (a = 0).  divRound(a, b) = (a + b/2) / b
// (generator.zig:253-255).  Any m >= 1, as the reference (m > N leaves ranges empty).
static void lut_from_values(size_t N, size_t m, const uint32_t *values, uint32_t *tv) {
    std::vector<uint32_t> raw(N, 0u);
    auto div_round = [](size_t a, size_t b) { return (a + b / 2) / b; };
    for (size_t x = 0; x < m; x++) {
        const size_t s = div_round(x * N, m), e = div_round((x + 1) * N, m);
        for (size_t i = s; i < e; i++) raw[i] = values[x];
    }
    const size_t off = div_round(N, 2 * m);
    for (size_t i = 0; i < N; i++) tv[N + i] = raw[(i + off) % N];
    for (size_t i = N - off; i < N; i++) tv[N + i] = ~tv[N + i] + 1u;
    for (size_t i = 0; i < N; i++) tv[i] = 0;
}

int tfhe_lut_generate_scaled(const tfhe_params *p, uint32_t m, double scale, const uint32_t *f_table, uint32_t *tv) {
    if (!p || !f_table || !tv || m == 0 || m > TFHE_LUT_MAX_M) return TFHE_ERR_INVALID;
    try {
        std::vector<uint32_t> enc(m);
        for (uint32_t x = 0; x < m; x++)  // Encoder.encode (encoder.zig:66-74): (f(x) mod m) * scale -> torus
            enc[x] = host::f64_to_torus((double)(f_table[x] % m) * scale);
        lut_from_values(p->N, m, enc.data(), tv);
    } catch (const std::bad_alloc &) {  // never through the C ABI (std::terminate)
        return TFHE_ERR_OOM;
    }
    return TFHE_OK;
}

int tfhe_lut_generate(const tfhe_params *p, uint32_t m, const uint32_t *f_table, uint32_t *tv) {
    if (!p || m == 0 || m > TFHE_LUT_MAX_M) return TFHE_ERR_INVALID;
    return tfhe_lut_generate_scaled(p, m, 1.0 / (2.0 * (double)m), f_table, tv);  // Encoder.new (encoder.zig:29-42)
}

int tfhe_lut_generate_full(const tfhe_params *p, uint32_t m, const uint32_t *values, uint32_t *tv) {
    if (!p || !values || !tv || m == 0 || m > TFHE_LUT_MAX_M) return TFHE_ERR_INVALID;
    try {
        lut_from_values(p->N, m, values, tv);
    } catch (const std::bad_alloc &) {
        return TFHE_ERR_OOM;
    }
    return TFHE_OK;
}

}  // extern "C"

// ---- Options ------------------------------------------------------------------
extern "C" {

}  // extern "C"

namespace {

// Range check of one option value, before anything is applied to any device.
bool option_ok(const tfhe_gpu_ctx *c, int key, int64_t v, std::string &why) {
    bool ok = false;
    switch (key) {
    case TFHE_OPT_BR_FORM:
        // 2 split, 4 pair: removed in round 4; 6 duo, 7 split-transform latency
        // form, 8 the whole form without loader assist: A/B libraries only (tools/ab/); 5 octo: L = 1 only
        ok = v == 0 || v == 1 || v == 3 || (v == 5 && c->P.L == 1) || (v >= 6 && v <= 40 && ab_forms_linked());
        if (!ok && v == 5) why = "TFHE_OPT_BR_FORM 5 (octo form) exists at L = 1 only";
        if (!ok && v >= 6 && v <= 8) why = "TFHE_OPT_BR_FORM " + std::to_string(v) + ": an A/B-only form, not in the product library (tools/ab/)";
        break;
    case TFHE_OPT_KS_FORM: ok = v >= 0 && v <= 3; break;
    case TFHE_OPT_BR_LOADER:  // the whole form always runs loader waves with slot counters (the
    case TFHE_OPT_BR_SYNC:    // gate-wave DMA and per-pair barrier variants were removed in round 5)
        ok = v == 1;
        if (!ok) why = "option " + std::to_string(key) + ": only 1 (the variant with value 0 was removed in round 5)";
        break;
    case TFHE_OPT_KS_NARROW:
    case TFHE_OPT_CIRCUIT_PACK: ok = v == 0 || v == 1; break;
    case TFHE_OPT_KS_ITEM_GROUPS: ok = v == 0 || v == 1 || v == 2 || v == 4 || v == 8; break;
    case TFHE_OPT_KS_SEL_ITEMS: ok = v == 8 || v == 16 || v == 32; break;
    case TFHE_OPT_ARITH: ok = v == TFHE_ARITH_AUTO || v == TFHE_ARITH_REFERENCE || v == TFHE_ARITH_FUSED_FORCED; break;
    case TFHE_OPT_BR_SPIN_CAP: ok = v >= 0 && v <= 0xFFFFFFFFll; break;
    case TFHE_OPT_HOST_PIPELINE: ok = v == 0 || v == 1; break;
    case TFHE_OPT_CIRCUIT_SPLIT: ok = v >= 0 && v <= 2; break;
    case TFHE_OPT_HOST_STAGING: ok = v == TFHE_STAGING_PAGEABLE || v == TFHE_STAGING_PINNED; break;
    case TFHE_OPT_TWIDDLES:
        ok = v == TFHE_TWIDDLES_GLIBC || v == TFHE_TWIDDLES_FDLIBM;
        // tfhe_gpu_keygen transformed the resident BK with the current tables:
        // other tables would no longer match it (a loaded reference key is data
        // and may be paired with either table)
        if (ok && c->key_from_keygen && v != c->twiddle_source) {
            why = "TFHE_OPT_TWIDDLES: the resident key was generated (tfhe_gpu_keygen) with the current FFT tables; "
                  "set the twiddle source before keygen";
            return false;
        }
        break;
    default: why = "unknown option key " + std::to_string(key); return false;
    }
    if (!ok && why.empty()) why = "bad value " + std::to_string(v) + " for option " + std::to_string(key);
    return ok;
}

// Apply a checked option to one device's context.
int apply_option(tfhe_gpu_ctx *c, int key, int64_t v) {
    LaunchOpts &o = c->opts;
    switch (key) {
    case TFHE_OPT_BR_FORM: o.br_form = (int)v; break;
    case TFHE_OPT_BR_LOADER: break;
    case TFHE_OPT_KS_FORM: o.ks_form = (int)v; break;
    case TFHE_OPT_KS_NARROW: o.ks_narrow = (int)v; break;
    case TFHE_OPT_KS_ITEM_GROUPS: o.ks_groups = (int)v; break;
    case TFHE_OPT_KS_SEL_ITEMS: o.ks_sel_items = (int)v; break;
    case TFHE_OPT_CIRCUIT_PACK: c->circuit_pack = v; break;
    case TFHE_OPT_TWIDDLES: return v == c->twiddle_source ? TFHE_OK : build_tables(c, (int)v);
    case TFHE_OPT_BR_SYNC: break;
    case TFHE_OPT_ARITH: o.arith_strict = v == TFHE_ARITH_REFERENCE ? 1 : v == TFHE_ARITH_FUSED_FORCED ? 2 : 0; break;
    case TFHE_OPT_BR_SPIN_CAP: c->K.spin_cap = (uint32_t)v; break;
    case TFHE_OPT_HOST_PIPELINE: c->pipeline = v; break;
    case TFHE_OPT_CIRCUIT_SPLIT: c->circuit_split = v; break;
    case TFHE_OPT_HOST_STAGING:
        if (c->stage_used) HIPCHK(c, hipStreamSynchronize(c->stream));  // nothing in flight from the arena
        c->stage_used = 0;
        c->host_staging = v;
        break;
    default: return TFHE_ERR_INVALID;
    }
    return TFHE_OK;
}

}  // namespace

extern "C" {

// Validated once, then applied to every device (shards 1.., then the root).
int tfhe_gpu_set_option(tfhe_gpu_ctx *c, int key, int64_t v) {
    if (!c) return TFHE_ERR_INVALID;
    std::string why;
    if (!option_ok(c, key, v, why)) return fail(c, TFHE_ERR_INVALID, why);
    for (size_t d = 1; d < c->shards.size(); d++) {
        const int rc = apply_option(c->shards[d], key, v);
        if (rc) return fail(c, rc, c->shards[d]->err);
    }
    return apply_option(c, key, v);
}

int tfhe_gpu_get_option(const tfhe_gpu_ctx *c, int key, int64_t *v) {
    if (!c || !v) return TFHE_ERR_INVALID;
    const LaunchOpts &o = c->opts;
    switch (key) {
    case TFHE_OPT_BR_FORM: *v = o.br_form; break;
    case TFHE_OPT_BR_LOADER: *v = 1; break;
    case TFHE_OPT_KS_FORM: *v = o.ks_form; break;
    case TFHE_OPT_KS_NARROW: *v = o.ks_narrow; break;
    case TFHE_OPT_KS_ITEM_GROUPS: *v = o.ks_groups; break;
    case TFHE_OPT_KS_SEL_ITEMS: *v = o.ks_sel_items; break;
    case TFHE_OPT_CIRCUIT_PACK: *v = c->circuit_pack; break;
    case TFHE_OPT_TWIDDLES: *v = c->twiddle_source; break;
    case TFHE_OPT_ARITH: *v = o.arith_strict == 1 ? TFHE_ARITH_REFERENCE : o.arith_strict == 2 ? TFHE_ARITH_FUSED_FORCED : TFHE_ARITH_AUTO; break;
    case TFHE_OPT_FUSED_ADMITTED: *v = o.key_fused_ok; break;
    case TFHE_OPT_LEVEL_ISSUE_US: *v = c->level_issue_us; break;
    case TFHE_OPT_KEY_ROW_RMS_PPM: *v = (int64_t)std::llround(c->bk_row_rms * 1e6); break;
    case TFHE_OPT_BR_SYNC: *v = 1; break;
    case TFHE_OPT_BR_SPIN_CAP: *v = c->K.spin_cap; break;
    case TFHE_OPT_HOST_PIPELINE: *v = c->pipeline; break;
    case TFHE_OPT_CIRCUIT_SPLIT: *v = c->circuit_split; break;
    case TFHE_OPT_HOST_STAGING: *v = c->host_staging; break;
    default: return TFHE_ERR_INVALID;
    }
    return TFHE_OK;
}

const char *tfhe_gpu_last_kernels(tfhe_gpu_ctx *c) {
    if (!c) return "";
    c->last_kernels = c->last_br;
    if (c->last_ks && c->last_ks[0]) c->last_kernels += std::string(" + ") + c->last_ks;
    return c->last_kernels.c_str();
}

int tfhe_fft_tables(uint32_t N, int source, double *twist_re, double *twist_im, double *stage_re, double *stage_im) {
    if (N < 4 || (N & (N - 1)) || (source != TFHE_TWIDDLES_GLIBC && source != TFHE_TWIDDLES_FDLIBM))
        return TFHE_ERR_INVALID;
    std::vector<double> a, b;
    host::twist_table(N, a, b, source);
    if (twist_re) std::memcpy(twist_re, a.data(), a.size() * 8);
    if (twist_im) std::memcpy(twist_im, b.data(), b.size() * 8);
    host::stage_twiddles(N, false, a, b, source);
    if (stage_re) std::memcpy(stage_re, a.data(), a.size() * 8);
    if (stage_im) std::memcpy(stage_im, b.data(), b.size() * 8);
    return TFHE_OK;
}

}  // extern "C"

// ---- Multi-device context ----------------------------------
namespace {

// librccl, loaded on the first multi-device key broadcast.  dlopen keeps the
// library loadable where RCCL is absent and, under PyTorch, reuses the RCCL
// that torch has already mapped (same SONAME) instead of a second copy.
struct RcclApi {
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclBroadcast) broadcast = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

const RcclApi *rccl_api(std::string &why) {
    static std::once_flag once;
    static RcclApi api;
    static std::string load_error;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
        if (!h) {
            load_error = std::string("cannot load librccl.so.1: ") + dlerror();
            return;
        }
        api.comm_init_all = (decltype(api.comm_init_all))dlsym(h, "ncclCommInitAll");
        api.comm_destroy = (decltype(api.comm_destroy))dlsym(h, "ncclCommDestroy");
        api.broadcast = (decltype(api.broadcast))dlsym(h, "ncclBroadcast");
        api.group_start = (decltype(api.group_start))dlsym(h, "ncclGroupStart");
        api.group_end = (decltype(api.group_end))dlsym(h, "ncclGroupEnd");
        api.error_string = (decltype(api.error_string))dlsym(h, "ncclGetErrorString");
        if (!api.comm_init_all || !api.comm_destroy || !api.broadcast || !api.group_start || !api.group_end ||
            !api.error_string)
            load_error = "librccl.so.1 lacks an nccl* entry point";
    });
    why = load_error;
    return load_error.empty() ? &api : nullptr;
}

bool is_multi(const tfhe_gpu_ctx *c) { return c && c->shards.size() > 1; }

void destroy_shards(tfhe_gpu_ctx *c) {
    if (!c->comms.empty()) {
        std::string why;
        if (const RcclApi *r = rccl_api(why))
            for (ncclComm_t m : c->comms)
                if (m) r->comm_destroy(m);
        c->comms.clear();
    }
    for (size_t d = 1; d < c->shards.size(); d++) tfhe_gpu_destroy(c->shards[d]);
    c->shards.clear();
}

// The key just loaded on shard 0 -> every other shard: one ncclBroadcast of
// the device BK and KSK (RCCL over xGMI), or a device-to-device copy when a
// device appears twice.  The test vector / offset are host state (8 KB).
int broadcast_key(tfhe_gpu_ctx *c) {
    int rc0 = key_admission(c);  // every key load ends here: admit the fused arithmetic or not
    if (rc0) {  // an unmeasured key is not a loaded key
        c->has_key = false;
        return rc0;
    }
    if (c->shards.empty()) return TFHE_OK;
    const size_t D = c->shards.size();
    for (size_t d = 1; d < D; d++) {
        tfhe_gpu_ctx *s = c->shards[d];
        s->has_key = false;
        HIPCHK(c, hipSetDevice(s->device));
        int rc = set_key_common(s, c->offset, c->testvec.data(), c->testvec.data() + c->P.N);
        if (rc) return fail(c, rc, s->err);
        HIPCHK(c, hipStreamSynchronize(s->stream));
    }
    if (c->distinct_devices) {
        std::string why;
        const RcclApi *r = rccl_api(why);
        if (!r) return fail(c, TFHE_ERR_HIP, why);
        if (c->comms.empty()) {
            std::vector<int> devs(D);
            for (size_t d = 0; d < D; d++) devs[d] = c->shards[d]->device;
            c->comms.assign(D, nullptr);
            ncclResult_t e = r->comm_init_all(c->comms.data(), (int)D, devs.data());
            if (e != ncclSuccess) {
                c->comms.clear();
                return fail(c, TFHE_ERR_HIP, std::string("ncclCommInitAll: ") + r->error_string(e));
            }
        }
        ncclResult_t e = r->group_start();
        for (size_t d = 0; d < D && e == ncclSuccess; d++) {
            tfhe_gpu_ctx *s = c->shards[d];
            e = r->broadcast(c->d_bk, s->d_bk, c->bk_bytes, ncclUint8, 0, c->comms[d], s->stream);
            if (e == ncclSuccess) e = r->broadcast(c->d_ksk, s->d_ksk, c->ksk_bytes, ncclUint8, 0, c->comms[d], s->stream);
        }
        ncclResult_t e2 = r->group_end();
        if (e == ncclSuccess) e = e2;
        if (e != ncclSuccess) return fail(c, TFHE_ERR_HIP, std::string("ncclBroadcast: ") + r->error_string(e));
    } else {
        for (size_t d = 1; d < D; d++) {
            tfhe_gpu_ctx *s = c->shards[d];
            HIPCHK(c, hipSetDevice(s->device));
            HIPCHK(c, hipMemcpyPeerAsync(s->d_bk, s->device, c->d_bk, c->device, c->bk_bytes, s->stream));
            HIPCHK(c, hipMemcpyPeerAsync(s->d_ksk, s->device, c->d_ksk, c->device, c->ksk_bytes, s->stream));
        }
    }
    for (size_t d = 1; d < D; d++) {
        tfhe_gpu_ctx *s = c->shards[d];
        HIPCHK(c, hipSetDevice(s->device));
        HIPCHK(c, hipStreamSynchronize(s->stream));
        s->ksk_gemm_ok = false;
    }
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // every copy must fingerprint like the root's before a shard may use it
    uint64_t bk0 = 0, ksk0 = 0;
    int rc = key_fingerprint(c, bk0, ksk0);
    if (rc) return rc;
    for (size_t d = 1; d < D; d++) {
        tfhe_gpu_ctx *s = c->shards[d];
        uint64_t bk = 0, ksk = 0;
        rc = key_fingerprint(s, bk, ksk);
        if (rc) return fail(c, rc, s->err);
        if (bk != bk0 || ksk != ksk0)
            return fail(c, TFHE_ERR_HIP, "key broadcast: the copy on device " + std::to_string(s->device) +
                                             " differs from device " + std::to_string(c->device) + "'s");
        s->bk_absmax = c->bk_absmax;  // same bits, same admission
        s->bk_row_rms = c->bk_row_rms;
        s->opts.key_fused_ok = c->opts.key_fused_ok;
        s->has_key = true;
    }
    HIPCHK(c, hipSetDevice(c->device));
    return TFHE_OK;
}

// f(shard, first item, count) on every device's contiguous slice of B items
// (ceil(B/D) each), concurrently: one host thread per device beyond the first.
template <class F>
int run_sharded(tfhe_gpu_ctx *c, size_t B, F f) {
    const size_t D = c->shards.size(), per = (B + D - 1) / D;
    std::vector<int> rc(D, TFHE_OK);
    std::vector<std::thread> th;
    for (size_t d = 1; d < D; d++) {
        const size_t b0 = std::min(B, d * per), n = std::min(B, b0 + per) - b0;
        if (n) th.emplace_back([&, d, b0, n] { rc[d] = f(c->shards[d], b0, n); });
    }
    if (B) rc[0] = f(c, 0, std::min(B, per));
    for (std::thread &t : th) t.join();
    for (size_t d = 1; d < D; d++)
        if (rc[d]) return fail(c, rc[d], "device " + std::to_string(c->shards[d]->device) + ": " + c->shards[d]->err);
    return rc[0];
}

struct Dsu {
    std::vector<uint32_t> p;
    explicit Dsu(size_t n) : p(n) { std::iota(p.begin(), p.end(), 0u); }
    uint32_t find(uint32_t x) {
        while (p[x] != x) x = p[x] = p[p[x]];
        return x;
    }
    void unite(uint32_t a, uint32_t b) { p[find(a)] = find(b); }
};

// Device of every gate (dev_of_gate[g] < D) for circuit_eval_multi: the
// connected components of the gate DAG under gate-to-gate wires (primary
// inputs do not join gates: they are replicated), largest first (by
// bootstrapped gates) onto the least-loaded device.
void partition_gates(size_t n_inputs, size_t n_gates, const uint8_t *ops, const uint32_t *in_a, const uint32_t *in_b,
                     size_t D, std::vector<uint32_t> &dev_of_gate) {
    Dsu dsu(std::max<size_t>(n_gates, 1));
    auto join = [&](size_t g, uint32_t w) {
        if (w >= n_inputs) dsu.unite((uint32_t)g, (uint32_t)(w - n_inputs));
    };
    for (size_t g = 0; g < n_gates; g++) {
        join(g, in_a[g]);
        if (ops[g] <= TFHE_GATE_ORYN) join(g, in_b[g]);
    }
    std::vector<uint64_t> weight(n_gates, 0);
    for (size_t g = 0; g < n_gates; g++)
        if (ops[g] != TFHE_GATE_NOT) weight[dsu.find((uint32_t)g)]++;
    std::vector<uint32_t> roots;
    for (size_t g = 0; g < n_gates; g++)
        if (dsu.find((uint32_t)g) == g) roots.push_back((uint32_t)g);
    std::stable_sort(roots.begin(), roots.end(), [&](uint32_t a, uint32_t b) { return weight[a] > weight[b]; });
    std::vector<uint32_t> dev_of_root(n_gates, 0);
    std::vector<uint64_t> load(D, 0);
    for (uint32_t r : roots) {
        const size_t d = std::min_element(load.begin(), load.end()) - load.begin();
        dev_of_root[r] = (uint32_t)d;
        load[d] += weight[r];
    }
    dev_of_gate.resize(n_gates);
    for (size_t g = 0; g < n_gates; g++) dev_of_gate[g] = dev_of_root[dsu.find((uint32_t)g)];
}

// Level split or components (TFHE_OPT_CIRCUIT_SPLIT: 0 auto, 1 components, 2
// levels).  Auto: levels when the component placement leaves the busiest device
// more than 10 % above an even share of at least one whole-form round per device
// (e.g. one big connected circuit); components otherwise (independent gates,
// MUXes and adders place evenly, and nothing crosses devices).
bool split_by_levels(const tfhe_gpu_ctx *c, size_t n_gates, const uint8_t *ops, const std::vector<uint32_t> &dev) {
    if (c->circuit_split != 0) return c->circuit_split == 2;
    const size_t D = c->shards.size();
    std::vector<uint64_t> load(D, 0);
    uint64_t total = 0;
    for (size_t g = 0; g < n_gates; g++)
        if (ops[g] != TFHE_GATE_NOT) {
            load[dev[g]]++;
            total++;
        }
    const uint64_t even = (total + D - 1) / D;
    return even >= 4 * device_cus() && *std::max_element(load.begin(), load.end()) * 10 > even * 11;
}

// circuit_eval over the devices, level by level ("a level barrier
// across GPUs"), for circuits whose gates form one dominant connected
// component.  Every device holds the whole wire table in the same layout (the
// plan of circuit_eval_one, its level packing modelled on all devices' CUs)
// and the primary inputs.  Per level, device d bootstraps its contiguous slice
// of the level's gates into its table; each slice is then copied to every other
// device (peer copies over xGMI, ordered by an event on the producer's stream:
// an all-gather), and every device applies the level's NOTs itself.  Outputs
// come from the first device's table.
int circuit_eval_levels(tfhe_gpu_ctx *c, size_t n_inputs, const uint32_t *inputs, size_t n_gates, const uint8_t *ops,
                        const uint32_t *in_a, const uint32_t *in_b, size_t n_outputs, const uint32_t *out_wires,
                        uint32_t *outputs, uint32_t *levels_out) {
    const size_t W = n_inputs + n_gates, D = c->shards.size(), w1 = tlwe0_words(c);
    CircuitPlan pl;
    if (const char *why = plan_circuit(n_inputs, n_gates, ops, in_a, in_b, n_outputs, out_wires, c->circuit_pack != 0,
                                       device_cus() * D, pl))
        return fail(c, TFHE_ERR_INVALID, why);
    std::vector<hipEvent_t> ev(D, nullptr);
    auto cleanup = [&] {
        for (size_t d = 0; d < D; d++)
            if (ev[d]) {
                (void)hipSetDevice(c->shards[d]->device);
                (void)hipEventDestroy(ev[d]);
            }
        (void)hipSetDevice(c->device);
    };
    int rc = TFHE_OK;
    for (size_t d = 0; d < D && !rc; d++) {
        tfhe_gpu_ctx *s = c->shards[d];
        rc = upload_plan(s, pl, W, n_inputs, inputs, n_outputs);
        if (!rc && hipEventCreateWithFlags(&ev[d], hipEventDisableTiming) != hipSuccess) rc = fail(s, TFHE_ERR_HIP, "hipEventCreate");
        if (rc) rc = fail(c, rc, "device " + std::to_string(s->device) + ": " + s->err);
    }
    size_t ip = 0, op_pos = 0, sp = n_inputs;
    // the per-level issue (launches, peer copies, event waits) runs on this one
    // host thread for all devices; it is asynchronous, so it costs wall time only
    // where it outruns the devices' per-level work (measured: DESIGN.md §7)
    const auto t_issue = std::chrono::steady_clock::now();
    for (uint32_t lv = 0; lv <= pl.max_level && !rc; lv++) {
        const size_t nb = pl.bs[lv].size(), nn = pl.nots[lv].size(), per = (nb + D - 1) / D;
        if (nb) {
            for (size_t d = 0; d < D && !rc; d++) {  // each device its slice
                tfhe_gpu_ctx *s = c->shards[d];
                const size_t lo = std::min(nb, d * per), n = std::min(nb, lo + per) - lo;
                if (!n) continue;
                if (hipSetDevice(s->device) != hipSuccess) { rc = fail(c, TFHE_ERR_HIP, "hipSetDevice"); break; }
                uint32_t *wires = (uint32_t *)s->s_wires.p;
                rc = run_bootstrap_dev(s, (const uint8_t *)s->s_cops.p + op_pos + lo, wires, wires, nullptr,
                                       wires + (sp + lo) * w1, n, RUN_BOOTSTRAP, (const uint32_t *)s->s_cidx.p + ip + 2 * lo);
                if (!rc && hipEventRecord(ev[d], s->stream) != hipSuccess) rc = fail(s, TFHE_ERR_HIP, "hipEventRecord");
                if (rc) rc = fail(c, rc, "device " + std::to_string(s->device) + ": " + s->err);
            }
            for (size_t e = 0; e < D && !rc; e++) {  // all-gather of the level's outputs
                tfhe_gpu_ctx *t = c->shards[e];
                if (hipSetDevice(t->device) != hipSuccess) { rc = fail(c, TFHE_ERR_HIP, "hipSetDevice"); break; }
                for (size_t d = 0; d < D && !rc; d++) {
                    const size_t lo = std::min(nb, d * per), n = std::min(nb, lo + per) - lo;
                    if (d == e || !n) continue;
                    tfhe_gpu_ctx *s = c->shards[d];
                    const size_t off = (sp + lo) * w1;
                    if (hipStreamWaitEvent(t->stream, ev[d], 0) != hipSuccess ||
                        hipMemcpyPeerAsync((uint32_t *)t->s_wires.p + off, t->device, (const uint32_t *)s->s_wires.p + off,
                                           s->device, n * w1 * 4, t->stream) != hipSuccess)
                        rc = fail(c, TFHE_ERR_HIP, "level all-gather to device " + std::to_string(t->device));
                }
            }
            ip += 2 * nb;
            op_pos += nb;
            sp += nb;
        }
        if (nn && !rc) {
            for (size_t d = 0; d < D && !rc; d++) {  // every device negates the level's NOT inputs itself
                tfhe_gpu_ctx *s = c->shards[d];
                uint32_t *wires = (uint32_t *)s->s_wires.p;
                if (hipSetDevice(s->device) != hipSuccess ||
                    launch_tlwe_gather(s->K, wires, (const uint32_t *)s->s_cidx.p + ip, wires + sp * w1, nn, true,
                                       s->stream) != hipSuccess)
                    rc = fail(c, TFHE_ERR_HIP, "NOT gather on device " + std::to_string(s->device));
            }
            ip += nn;
            sp += nn;
        }
    }
    c->level_issue_us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t_issue).count();
    for (size_t d = 1; d < D && !rc; d++) {  // every device's work done, its error word clean
        tfhe_gpu_ctx *s = c->shards[d];
        if (hipSetDevice(s->device) != hipSuccess) { rc = fail(c, TFHE_ERR_HIP, "hipSetDevice"); break; }
        rc = sync_check(s);
        if (rc) rc = fail(c, rc, "device " + std::to_string(s->device) + ": " + s->err);
    }
    if (!rc && hipSetDevice(c->device) != hipSuccess) rc = fail(c, TFHE_ERR_HIP, "hipSetDevice");
    if (!rc && n_outputs) {
        if (launch_tlwe_gather(c->K, (const uint32_t *)c->s_wires.p, (const uint32_t *)c->s_cidx.p + ip,
                               (uint32_t *)c->s_out.p, n_outputs, false, c->stream) != hipSuccess)
            rc = fail(c, TFHE_ERR_HIP, "output gather");
        else
            rc = d2h_sync(c, outputs, c->s_out.p, n_outputs * w1 * 4);
    } else if (!rc) {
        rc = sync_check(c);
    }
    cleanup();
    if (!rc && levels_out) *levels_out = pl.max_level;
    return rc;
}

// circuit_eval over the devices.  Primary inputs are read-only, so every
// device gets its own copy of the ones it reads; only gate-to-gate wires tie
// gates together.  The connected components of the gate DAG under those wires
// go whole to one device each, largest first onto the least-loaded device
// (bootstrapped gates), so each device evaluates an independent sub-circuit
// with its own level schedule and no wire crosses devices.  Config 4's
// independent AND/OR/XOR gates and MUXes over shared inputs (gates.zig:124-129)
// spread evenly; one adder (examples/add_two_numbers.zig:24-73) stays whole.
int circuit_eval_multi(tfhe_gpu_ctx *c, size_t n_inputs, const uint32_t *inputs, size_t n_gates, const uint8_t *ops,
                       const uint32_t *in_a, const uint32_t *in_b, size_t n_outputs, const uint32_t *out_wires,
                       uint32_t *outputs, uint32_t *levels_out) {
    const size_t W = n_inputs + n_gates, D = c->shards.size(), w1 = tlwe0_words(c);
    {  // validate the whole graph first (same errors as one device)
        std::vector<uint32_t> level;
        std::vector<std::vector<uint32_t>> bs, nots;
        uint32_t ml = 0;
        if (const char *why = schedule_levels(n_inputs, n_gates, ops, in_a, in_b, false, 256, level, ml, bs, nots))
            return fail(c, TFHE_ERR_INVALID, why);
        for (size_t o = 0; o < n_outputs; o++)
            if (out_wires[o] >= W) return fail(c, TFHE_ERR_INVALID, "output wire out of range");
    }
    std::vector<uint32_t> dev_of_gate;
    partition_gates(n_inputs, n_gates, ops, in_a, in_b, D, dev_of_gate);
    if (split_by_levels(c, n_gates, ops, dev_of_gate))
        return circuit_eval_levels(c, n_inputs, inputs, n_gates, ops, in_a, in_b, n_outputs, out_wires, outputs, levels_out);
    // per-device sub-circuits; wires renumbered: the device's inputs first, then its gates
    struct Sub {
        std::vector<uint32_t> inputs, in_a, in_b, out_wires, out_index;
        std::vector<uint8_t> ops;
        std::vector<uint32_t> outputs;
        uint32_t levels = 0;
        std::vector<uint32_t> input_id;  // global input -> local id (or none)
    };
    std::vector<Sub> sub(D);
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    auto gate_dev = [&](size_t g) { return dev_of_gate[g]; };
    // an output that is a primary input is copied out by device 0
    auto wire_dev = [&](uint32_t w) { return w < n_inputs ? 0u : gate_dev(w - n_inputs); };
    auto use_input = [&](uint32_t d, uint32_t w) {
        if (w >= n_inputs) return;
        Sub &s = sub[d];
        if (s.input_id.empty()) s.input_id.assign(n_inputs, NONE);
        if (s.input_id[w] == NONE) {
            s.input_id[w] = (uint32_t)s.inputs.size();
            s.inputs.push_back(w);
        }
    };
    for (size_t g = 0; g < n_gates; g++) {
        use_input(gate_dev(g), in_a[g]);
        if (ops[g] <= TFHE_GATE_ORYN) use_input(gate_dev(g), in_b[g]);
    }
    for (size_t o = 0; o < n_outputs; o++) use_input(wire_dev(out_wires[o]), out_wires[o]);
    std::vector<uint32_t> local_gate(n_gates), gate_count(D, 0);
    for (size_t g = 0; g < n_gates; g++) local_gate[g] = gate_count[gate_dev(g)]++;
    auto id = [&](uint32_t d, uint32_t w) {
        return w < n_inputs ? sub[d].input_id[w] : (uint32_t)sub[d].inputs.size() + local_gate[w - n_inputs];
    };
    for (size_t g = 0; g < n_gates; g++) {
        const uint32_t d = gate_dev(g);
        Sub &s = sub[d];
        s.ops.push_back(ops[g]);
        s.in_a.push_back(id(d, in_a[g]));
        s.in_b.push_back(ops[g] <= TFHE_GATE_ORYN ? id(d, in_b[g]) : 0u);
    }
    for (size_t o = 0; o < n_outputs; o++) {
        const uint32_t d = wire_dev(out_wires[o]);
        sub[d].out_wires.push_back(id(d, out_wires[o]));
        sub[d].out_index.push_back((uint32_t)o);
    }
    std::vector<int> rc(D, TFHE_OK);
    auto run = [&](size_t d) {
        Sub &s = sub[d];
        if (s.ops.empty() && s.out_wires.empty()) return;
        std::vector<uint32_t> in(s.inputs.size() * w1);
        for (size_t i = 0; i < s.inputs.size(); i++)
            std::memcpy(in.data() + i * w1, inputs + (size_t)s.inputs[i] * w1, w1 * 4);
        s.outputs.resize(s.out_wires.size() * w1);
        rc[d] = circuit_eval_one(c->shards[d], s.inputs.size(), in.data(), s.ops.size(), s.ops.data(), s.in_a.data(),
                                 s.in_b.data(), s.out_wires.size(), s.out_wires.data(), s.outputs.data(), &s.levels);
    };
    std::vector<std::thread> th;
    for (size_t d = 1; d < D; d++) th.emplace_back(run, d);
    run(0);
    for (std::thread &t : th) t.join();
    uint32_t depth = 0;
    for (size_t d = 0; d < D; d++) {
        if (rc[d]) return fail(c, rc[d], "device " + std::to_string(c->shards[d]->device) + ": " + c->shards[d]->err);
        const Sub &s = sub[d];
        for (size_t k = 0; k < s.out_index.size(); k++)
            std::memcpy(outputs + (size_t)s.out_index[k] * w1, s.outputs.data() + k * w1, w1 * 4);
        depth = std::max(depth, s.levels);
    }
    if (levels_out) *levels_out = depth;
    return TFHE_OK;
}

}  // namespace

extern "C" {

int tfhe_gpu_create_multi(const tfhe_params *params, int num_devices, const int *devices, tfhe_gpu_ctx **out) {
    if (!out || num_devices < 1) return TFHE_ERR_INVALID;
    *out = nullptr;
    std::vector<int> devs(num_devices);
    for (int d = 0; d < num_devices; d++) devs[d] = devices ? devices[d] : d;
    std::string why;
    if (!params_ok(params, why)) return create_fail(TFHE_ERR_INVALID, "tfhe_gpu_create_multi: " + why);
    if (ab_build_refused()) return create_fail(TFHE_ERR_INVALID, AB_REFUSAL);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) return create_fail(TFHE_ERR_HIP, "hipGetDeviceCount failed");
    for (int d : devs)
        if (d < 0 || d >= ndev)
            return create_fail(TFHE_ERR_HIP, "device " + std::to_string(d) + " does not exist (" +
                                                 std::to_string(ndev) + " HIP device(s) visible)");
    tfhe_gpu_ctx *root = nullptr;
    int rc = tfhe_gpu_create_on_device(params, devs[0], &root);
    if (rc) return rc;
    root->shards.push_back(root);
    for (int d = 1; d < num_devices; d++) {
        tfhe_gpu_ctx *s = nullptr;
        rc = tfhe_gpu_create_on_device(params, devs[d], &s);
        if (rc) {
            tfhe_gpu_destroy(root);
            return rc;
        }
        root->shards.push_back(s);
    }
    std::vector<int> sorted = devs;
    std::sort(sorted.begin(), sorted.end());
    root->distinct_devices = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    if (root->distinct_devices) {
        // every ordered pair: the level split all-gathers between all of them
        for (int a : devs)
            for (int b : devs) {
                if (a == b) continue;
                int can = 0;
                hipError_t e = hipDeviceCanAccessPeer(&can, a, b);
                if (e != hipSuccess || !can) {
                    tfhe_gpu_destroy(root);
                    return create_fail(TFHE_ERR_DEVICE, "device " + std::to_string(a) + " cannot access device " +
                                                            std::to_string(b) + "'s memory (hipDeviceCanAccessPeer" +
                                                            (e != hipSuccess ? std::string(": ") + hipGetErrorString(e) : "") +
                                                            "): the multi-device context needs xGMI peer access");
                }
                e = hipSetDevice(a);
                if (e == hipSuccess) e = hipDeviceEnablePeerAccess(b, 0);
                if (e == hipErrorPeerAccessAlreadyEnabled) {
                    (void)hipGetLastError();  // clear the sticky status of an already-enabled pair
                    e = hipSuccess;
                }
                if (e != hipSuccess) {
                    tfhe_gpu_destroy(root);
                    return create_fail(TFHE_ERR_DEVICE, "hipDeviceEnablePeerAccess(" + std::to_string(a) + " -> " +
                                                            std::to_string(b) + "): " + hipGetErrorString(e));
                }
            }
        (void)hipSetDevice(devs[0]);
    }
    *out = root;
    return TFHE_OK;
}

// SURVEY §8b's entry point: devices 0..num_devices-1 of this node (one device:
// a plain context on device 0; more: the multi-device context above).
int tfhe_gpu_create(const tfhe_params *params, int num_devices, tfhe_gpu_ctx **out) {
    if (!out) return TFHE_ERR_INVALID;
    *out = nullptr;
    std::string why;
    if (num_devices < 1 || !params_ok(params, why))
        return create_fail(TFHE_ERR_INVALID, num_devices < 1 ? "num_devices < 1" : "tfhe_gpu_create: " + why);
    if (ab_build_refused()) return create_fail(TFHE_ERR_INVALID, AB_REFUSAL);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || num_devices > ndev)
        return create_fail(TFHE_ERR_HIP, std::to_string(num_devices) + " device(s) requested, " +
                                             std::to_string(ndev) + " HIP device(s) visible");
    if (num_devices == 1) return tfhe_gpu_create_on_device(params, 0, out);
    return tfhe_gpu_create_multi(params, num_devices, nullptr, out);
}

int tfhe_gpu_num_devices(const tfhe_gpu_ctx *c) { return !c ? 0 : c->shards.empty() ? 1 : (int)c->shards.size(); }

int tfhe_gpu_near_tie_items(const tfhe_gpu_ctx *c, uint64_t *count) {
    if (!c || !count) return TFHE_ERR_INVALID;
    uint64_t n = c->near_tie_items;
    for (size_t d = 1; d < c->shards.size(); d++) n += c->shards[d]->near_tie_items;
    *count = n;
    return TFHE_OK;
}

int tfhe_gpu_device_bootstraps(const tfhe_gpu_ctx *c, uint64_t *counts, int max_devices) {
    if (!c || !counts || max_devices < 1) return TFHE_ERR_INVALID;
    const int D = tfhe_gpu_num_devices(c);
    for (int d = 0; d < D && d < max_devices; d++) counts[d] = c->shards.empty() ? c->bootstraps : c->shards[d]->bootstraps;
    return D;
}

int tfhe_gpu_bootstrap_batch(tfhe_gpu_ctx *c, const uint32_t *in, uint32_t *out, size_t B) {
    if (!is_multi(c)) return bootstrap_batch_one(c, in, out, B);
    if (B && (!in || !out)) return fail(c, TFHE_ERR_INVALID, "null argument");
    const size_t w = tlwe0_words(c);
    return run_sharded(c, B, [&](tfhe_gpu_ctx *s, size_t b0, size_t n) {
        return bootstrap_batch_one(s, in + b0 * w, out + b0 * w, n);
    });
}

int tfhe_gpu_bootstrap_without_key_switch_batch(tfhe_gpu_ctx *c, const uint32_t *in, uint32_t *out, size_t B) {
    if (!is_multi(c)) return bootstrap_without_key_switch_batch_one(c, in, out, B);
    if (B && (!in || !out)) return fail(c, TFHE_ERR_INVALID, "null argument");
    const size_t w = tlwe0_words(c);
    return run_sharded(c, B, [&](tfhe_gpu_ctx *s, size_t b0, size_t n) {
        return bootstrap_without_key_switch_batch_one(s, in + b0 * w, out + b0 * w, n);
    });
}

int tfhe_gpu_gate_batch(tfhe_gpu_ctx *c, const uint8_t *ops, const uint32_t *a, const uint32_t *b, uint32_t *out,
                        size_t B) {
    if (!is_multi(c)) return gate_batch_one(c, ops, a, b, out, B);
    if (B && (!ops || !a || !b || !out)) return fail(c, TFHE_ERR_INVALID, "null argument");
    const size_t w = tlwe0_words(c);
    return run_sharded(c, B, [&](tfhe_gpu_ctx *s, size_t b0, size_t n) {
        return gate_batch_one(s, ops + b0, a + b0 * w, b + b0 * w, out + b0 * w, n);
    });
}

int tfhe_gpu_blind_rotate_batch(tfhe_gpu_ctx *c, const uint32_t *in, const uint32_t *testvec, uint32_t *trlwe_out,
                                size_t B) {
    if (!is_multi(c)) return blind_rotate_batch_one(c, in, testvec, trlwe_out, B);
    if (B && (!in || !trlwe_out)) return fail(c, TFHE_ERR_INVALID, "null argument");
    const size_t w = tlwe0_words(c), wo = 2 * (size_t)c->P.N;
    return run_sharded(c, B, [&](tfhe_gpu_ctx *s, size_t b0, size_t n) {
        return blind_rotate_batch_one(s, in + b0 * w, testvec, trlwe_out + b0 * wo, n);
    });
}

int tfhe_gpu_bootstrap_lut_batch(tfhe_gpu_ctx *c, const uint32_t *in, const uint32_t *testvec, uint32_t *out,
                                 size_t B) {
    if (!is_multi(c)) return bootstrap_lut_batch_one(c, in, testvec, out, B);
    if (!testvec || (B && (!in || !out))) return fail(c, TFHE_ERR_INVALID, "null argument");
    const size_t w = tlwe0_words(c);
    return run_sharded(c, B, [&](tfhe_gpu_ctx *s, size_t b0, size_t n) {
        return bootstrap_lut_batch_one(s, in + b0 * w, testvec, out + b0 * w, n);
    });
}

int tfhe_gpu_key_switch_batch(tfhe_gpu_ctx *c, const uint32_t *in_lv1, uint32_t *out_lv0, size_t B) {
    if (!is_multi(c)) return key_switch_batch_one(c, in_lv1, out_lv0, B);
    if (B && (!in_lv1 || !out_lv0)) return fail(c, TFHE_ERR_INVALID, "null argument");
    const size_t w = tlwe0_words(c), wi = (size_t)c->P.N + 1;
    return run_sharded(c, B, [&](tfhe_gpu_ctx *s, size_t b0, size_t n) {
        return key_switch_batch_one(s, in_lv1 + b0 * wi, out_lv0 + b0 * w, n);
    });
}

int tfhe_gpu_reenc_key_load(tfhe_gpu_ctx *c, const uint32_t *key_encryptions, size_t len, uint32_t basebit,
                            uint32_t t, tfhe_gpu_reenc_key **out) {
    int rc = reenc_key_load_one(c, key_encryptions, len, basebit, t, out);
    if (rc || !is_multi(c)) return rc;
    for (size_t d = 1; d < c->shards.size(); d++) {  // one upload per device (host -> each HBM)
        tfhe_gpu_reenc_key *k = nullptr;
        rc = reenc_key_load_one(c->shards[d], key_encryptions, len, basebit, t, &k);
        if (rc) {
            tfhe_gpu_reenc_key_destroy(*out);
            *out = nullptr;
            return fail(c, rc, c->shards[d]->err);
        }
        (*out)->peers.push_back(k);
    }
    return TFHE_OK;
}

int tfhe_gpu_reencrypt_batch(tfhe_gpu_ctx *c, const tfhe_gpu_reenc_key *k, const uint32_t *in, uint32_t *out,
                             size_t B) {
    if (!is_multi(c)) return reencrypt_batch_one(c, k, in, out, B);
    if (!k || (B && (!in || !out))) return fail(c, TFHE_ERR_INVALID, "null argument");
    if (k->peers.size() + 1 != c->shards.size()) return fail(c, TFHE_ERR_INVALID, "key was not loaded on this context");
    const size_t w = tlwe0_words(c);
    return run_sharded(c, B, [&](tfhe_gpu_ctx *s, size_t b0, size_t n) {
        size_t d = 0;
        while (c->shards[d] != s) d++;
        return reencrypt_batch_one(s, d ? k->peers[d - 1] : k, in + b0 * w, out + b0 * w, n);
    });
}

int tfhe_gpu_reencrypt_batch_dev(tfhe_gpu_ctx *c, const tfhe_gpu_reenc_key *k, const uint32_t *in_dev,
                                 uint32_t *out_dev, size_t B) {
    if (is_multi(c)) return fail(c, TFHE_ERR_INVALID, "device-resident calls take a single-device context");
    return reencrypt_batch_dev_one(c, k, in_dev, out_dev, B);
}

int tfhe_circuit_partition(size_t n_inputs, size_t n_gates, const uint8_t *ops, const uint32_t *in_a,
                           const uint32_t *in_b, int num_devices, uint32_t *device_of_gate) {
    if ((n_gates && (!ops || !in_a || !in_b || !device_of_gate)) || num_devices < 1) return TFHE_ERR_INVALID;
    if (n_inputs + n_gates > 0xFFFFFFFFull) return TFHE_ERR_INVALID;
    std::vector<uint32_t> level;
    std::vector<std::vector<uint32_t>> bs, nots;
    uint32_t ml = 0;
    if (schedule_levels(n_inputs, n_gates, ops, in_a, in_b, false, 256, level, ml, bs, nots)) return TFHE_ERR_INVALID;
    std::vector<uint32_t> dev;
    partition_gates(n_inputs, n_gates, ops, in_a, in_b, (size_t)num_devices, dev);
    std::copy(dev.begin(), dev.end(), device_of_gate);
    return TFHE_OK;
}

int tfhe_gpu_circuit_eval_dev(tfhe_gpu_ctx *c, size_t n_inputs, const uint32_t *inputs_dev, size_t n_gates,
                              const uint8_t *ops, const uint32_t *in_a, const uint32_t *in_b, size_t n_outputs,
                              const uint32_t *out_wires, uint32_t *outputs_dev, uint32_t *levels) {
    if (is_multi(c)) return fail(c, TFHE_ERR_INVALID, "device-resident calls take a single-device context");
    return circuit_eval_one(c, n_inputs, inputs_dev, n_gates, ops, in_a, in_b, n_outputs, out_wires, outputs_dev,
                            levels, true);
}

int tfhe_gpu_circuit_eval(tfhe_gpu_ctx *c, size_t n_inputs, const uint32_t *inputs, size_t n_gates, const uint8_t *ops,
                          const uint32_t *in_a, const uint32_t *in_b, size_t n_outputs, const uint32_t *out_wires,
                          uint32_t *outputs, uint32_t *levels) {
    if (!is_multi(c))
        return circuit_eval_one(c, n_inputs, inputs, n_gates, ops, in_a, in_b, n_outputs, out_wires, outputs, levels);
    if ((n_inputs && !inputs) || (n_gates && (!ops || !in_a || !in_b)) || (n_outputs && (!out_wires || !outputs)))
        return fail(c, TFHE_ERR_INVALID, "null argument");
    if (!c->has_key) return fail(c, TFHE_ERR_NO_KEY, "no cloud key loaded");
    if (n_inputs + n_gates > 0xFFFFFFFFull) return fail(c, TFHE_ERR_INVALID, "too many wires");
    return circuit_eval_multi(c, n_inputs, inputs, n_gates, ops, in_a, in_b, n_outputs, out_wires, outputs, levels);
}

}  // extern "C"
