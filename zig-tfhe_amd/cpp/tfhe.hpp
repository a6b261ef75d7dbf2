// tfhe.hpp — C++ host-side mirror of zig-tfhe's public surface for the gate
// bootstrap path, over the C ABI (include/tfhe_gpu.h).  Header-only; link
// libtfhe_gpu.so.  Names and argument meaning follow the reference:
//   params.zig        -> tfhe::params::SECURITY_128_BIT() / SECURITY_80_BIT() / SECURITY_UINT4()
//   tlwe.zig TLWELv0  -> tfhe::TLWELv0 (p[n+1], b() last; encryptBool / decryptBool / neg / add / sub)
//   key.zig           -> tfhe::SecretKey, tfhe::CloudKey (device resident; keygen or load of host arrays)
//   bootstrap.zig     -> tfhe::HipBootstrap (bootstrap / bootstrapWithoutKeySwitch / name)
//   gates.zig Gates   -> tfhe::Gates (nandGate ... orYnGate, muxNaive, notGate, copy, constant,
//                        batchNand ... batchXnor — placeholders in the reference, implemented here)
//   proxy_reenc.zig   -> tfhe::PublicKeyLv0, tfhe::ProxyReencryptionKey, tfhe::HipReencryptor
//                        (reencryptTLWELv0 on the GPU)
// Zig error unions become tfhe::Error exceptions carrying the C status.
// There is no CPU path: every bootstrap runs on the GPU through the C ABI.
#pragma once

#include <tfhe_gpu.h>

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace tfhe {

using Torus = uint32_t;

class Error : public std::runtime_error {
  public:
    Error(int status, const std::string &what) : std::runtime_error(what), status(status) {}
    int status;
};

inline void check(int rc, const char *what, const tfhe_gpu_ctx *ctx = nullptr) {
    if (rc != TFHE_OK)
        throw Error(rc, std::string(what) + ": status " + std::to_string(rc) +
                            (ctx ? std::string(": ") + tfhe_gpu_last_error(ctx) : std::string()));
}

// params.zig:70-95, 350-375, 210-235; KSK/BSK alphas as the Python mirror
// (tfhe_amd.SECURITY_*): the 128-bit constants params.zig:419-422, and BSK
// noise 0 for UINT4
namespace params {
inline tfhe_params SECURITY_128_BIT() {
    return tfhe_params{700, 1024, 10, 3, 6, 2, 9, 0, 2.0e-5, 2.0e-8, 2.0e-5, 2.0e-8};
}
inline tfhe_params SECURITY_80_BIT() {
    return tfhe_params{550, 1024, 10, 3, 6, 2, 7, 0, 5.0e-5, 3.73e-8, 2.0e-5, 2.0e-8};
}
inline tfhe_params SECURITY_UINT4() {
    return tfhe_params{820, 1024, 10, 1, 22, 5, 3, 0, 0.00000251676160959795544987084234,
                       0.00000000000000022204460492503131, 0.00000251676160959795544987084234, 0.0};
}
}  // namespace params

// tlwe.zig:11-239
struct TLWELv0 {
    std::vector<Torus> p;  // a[0..n) then b
    TLWELv0() = default;
    explicit TLWELv0(size_t n) : p(n + 1, 0u) {}
    size_t n() const { return p.size() - 1; }
    Torus b() const { return p.back(); }
    Torus &bMut() { return p.back(); }
    TLWELv0 neg() const {  // tlwe.zig:160-177
        TLWELv0 r(n());
        for (size_t i = 0; i < p.size(); i++) r.p[i] = 0u - p[i];
        return r;
    }
    TLWELv0 add(const TLWELv0 &o) const {
        TLWELv0 r(n());
        for (size_t i = 0; i < p.size(); i++) r.p[i] = p[i] + o.p[i];
        return r;
    }
    TLWELv0 sub(const TLWELv0 &o) const {
        TLWELv0 r(n());
        for (size_t i = 0; i < p.size(); i++) r.p[i] = p[i] - o.p[i];
        return r;
    }
};

// key.zig:33-57: binary lv0 / lv1 keys
struct SecretKey {
    tfhe_params params{};
    std::vector<Torus> key_lv0, key_lv1;

    // TLWELv0.encryptBool (tlwe.zig:52-56) with a seeded DefaultPrng
    TLWELv0 encryptBool(bool bit, uint64_t seed) const {
        TLWELv0 ct(params.n);
        const uint8_t v = bit ? 1 : 0;
        check(tfhe_encrypt_bool_batch(&params, key_lv0.data(), &v, seed, ct.p.data(), 1), "encryptBool");
        return ct;
    }
    bool decryptBool(const TLWELv0 &ct) const {  // tlwe.zig:58-68
        uint8_t v = 0;
        check(tfhe_decrypt_bool_batch(&params, key_lv0.data(), ct.p.data(), &v, 1), "decryptBool");
        return v != 0;
    }
    TLWELv0 encryptLweMessage(uint32_t msg, uint32_t m, uint64_t seed) const {  // tlwe.zig:74-97
        TLWELv0 ct(params.n);
        check(tfhe_encrypt_lwe_message_batch(&params, key_lv0.data(), &msg, m, seed, ct.p.data(), 1),
              "encryptLweMessage");
        return ct;
    }
    uint32_t decryptLweMessage(const TLWELv0 &ct, uint32_t m) const {  // tlwe.zig:100-117
        uint32_t v = 0;
        check(tfhe_decrypt_lwe_message_batch(&params, key_lv0.data(), ct.p.data(), m, &v, 1), "decryptLweMessage");
        return v;
    }
    // SecretKey.new (key.zig:41-57) from DefaultPrng(seed)
    static SecretKey newWithSeed(const tfhe_params &p, uint64_t seed) {
        SecretKey sk;
        sk.params = p;
        sk.key_lv0.assign(p.n, 0u);
        sk.key_lv1.assign(p.N, 0u);
        check(tfhe_secret_key_new(&p, seed, sk.key_lv0.data(), sk.key_lv1.data()), "SecretKey.new");
        return sk;
    }
};

// proxy_reenc.zig:35-121.  Encryption e of newWithParams uses DefaultPrng(seed0 + e).
struct PublicKeyLv0 {
    tfhe_params params{};
    size_t size = 0;
    std::vector<Torus> encryptions;  // size x (n+1)

    static PublicKeyLv0 newWithParams(const SecretKey &sk, size_t size, double alpha, uint64_t seed0) {
        PublicKeyLv0 pk;
        pk.params = sk.params;
        pk.size = size;
        pk.encryptions.assign(size * (sk.params.n + 1), 0u);
        check(tfhe_public_key_gen(&sk.params, sk.key_lv0.data(), size, alpha, seed0, pk.encryptions.data()),
              "PublicKeyLv0.new");
        return pk;
    }
    static PublicKeyLv0 create(const SecretKey &sk, uint64_t seed0) {  // PublicKeyLv0.new: 2n, tlwe_lv0.ALPHA
        return newWithParams(sk, 2 * (size_t)sk.params.n, sk.params.alpha_lv0, seed0);
    }
    TLWELv0 encryptBool(bool bit, double alpha, uint64_t seed) const {  // :116-120
        TLWELv0 ct(params.n);
        const uint8_t v = bit ? 1 : 0;
        check(tfhe_public_key_encrypt_bool_batch(&params, encryptions.data(), size, &v, alpha, seed, ct.p.data(), 1),
              "PublicKeyLv0.encryptBool");
        return ct;
    }
};

// proxy_reenc.zig:124-257: key_encryptions[(base*t*i)+(base*j)+k]; the c-th encryption uses seed0 + c.
struct ProxyReencryptionKey {
    std::vector<Torus> key_encryptions;
    uint32_t basebit = 0, t = 0;
    size_t base() const { return (size_t)1 << basebit; }

    static ProxyReencryptionKey newSymmetricWithParams(const SecretKey &from, const SecretKey &to, double alpha,
                                                       uint32_t basebit, uint32_t t, uint64_t seed0) {
        ProxyReencryptionKey k = shaped(from.params, basebit, t);
        check(tfhe_reenc_key_gen_symmetric(&from.params, from.key_lv0.data(), to.key_lv0.data(), alpha, basebit, t,
                                           seed0, k.key_encryptions.data()),
              "ProxyReencryptionKey.newSymmetric");
        return k;
    }
    static ProxyReencryptionKey newAsymmetricWithParams(const SecretKey &from, const PublicKeyLv0 &to, double alpha,
                                                        uint32_t basebit, uint32_t t, uint64_t seed0) {
        ProxyReencryptionKey k = shaped(from.params, basebit, t);
        check(tfhe_reenc_key_gen_asymmetric(&from.params, from.key_lv0.data(), to.encryptions.data(), to.size, alpha,
                                            basebit, t, seed0, k.key_encryptions.data()),
              "ProxyReencryptionKey.newAsymmetric");
        return k;
    }
    // newSymmetric / newAsymmetric: KSK_ALPHA and the set's BASEBIT / IKS_T (:131-147, :199-212)
    static ProxyReencryptionKey newSymmetric(const SecretKey &from, const SecretKey &to, uint64_t seed0) {
        return newSymmetricWithParams(from, to, from.params.alpha_ksk, from.params.basebit, from.params.iks_t, seed0);
    }
    static ProxyReencryptionKey newAsymmetric(const SecretKey &from, const PublicKeyLv0 &to, uint64_t seed0) {
        return newAsymmetricWithParams(from, to, from.params.alpha_ksk, from.params.basebit, from.params.iks_t, seed0);
    }

  private:
    static ProxyReencryptionKey shaped(const tfhe_params &p, uint32_t basebit, uint32_t t) {
        ProxyReencryptionKey k;
        k.basebit = basebit;
        k.t = t;
        k.key_encryptions.assign(((size_t)p.n * t << basebit) * (p.n + 1), 0u);
        return k;
    }
};

// key.zig:61-118.  The cloud key lives in HBM inside one GPU context.
class CloudKey {
  public:
    // CloudKey.new (key.zig:70-77) from a seeded SecretKey.new: keys generated
    // with the restated DefaultPrng order, FFTs on the GPU.
    static std::pair<SecretKey, CloudKey> generate(const tfhe_params &p, uint64_t secret_seed, uint64_t cloud_seed,
                                                   int device = 0) {
        CloudKey ck(p, device);
        SecretKey sk;
        sk.params = p;
        sk.key_lv0.assign(p.n, 0u);
        sk.key_lv1.assign(p.N, 0u);
        check(tfhe_gpu_keygen(ck.ctx(), secret_seed, cloud_seed, sk.key_lv0.data(), sk.key_lv1.data(), nullptr,
                              nullptr),
              "CloudKey.generate", ck.ctx());
        return {std::move(sk), std::move(ck)};
    }
    // An existing CloudKey in the reference's host layout (decomposition_offset,
    // blind_rotate_testvec, bootstrapping_key.items, key_switching_key.items).
    static CloudKey load(const tfhe_params &p, Torus offset, const std::vector<Torus> &testvec_a,
                         const std::vector<Torus> &testvec_b, const std::vector<double> &bsk,
                         const std::vector<Torus> &ksk, int device = 0) {
        CloudKey ck(p, device);
        check(tfhe_gpu_load_cloud_key(ck.ctx(), offset, testvec_a.data(), testvec_b.data(), bsk.data(), bsk.size(),
                                      ksk.data(), ksk.size()),
              "CloudKey.load", ck.ctx());
        return ck;
    }
    // Key files (include/tfhe_gpu.h "Cloud-key files"): the reference has no
    // serialization; a saved key reloads bit-exact on any device.
    static CloudKey loadFile(const tfhe_params &p, const std::string &path, int device = 0) {
        CloudKey ck(p, device);
        check(tfhe_gpu_load_cloud_key_file(ck.ctx(), path.c_str()), "CloudKey.loadFile", ck.ctx());
        return ck;
    }
    // The same key resident on several GPUs (tfhe_gpu_create_multi): loaded on the
    // first, broadcast over RCCL; every batch call through it is sharded over them.
    static CloudKey loadFile(const tfhe_params &p, const std::string &path, const std::vector<int> &devices) {
        CloudKey ck(p, devices);
        check(tfhe_gpu_load_cloud_key_file(ck.ctx(), path.c_str()), "CloudKey.loadFile", ck.ctx());
        return ck;
    }
    static std::pair<SecretKey, CloudKey> generate(const tfhe_params &p, uint64_t secret_seed, uint64_t cloud_seed,
                                                   const std::vector<int> &devices) {
        CloudKey ck(p, devices);
        SecretKey sk;
        sk.params = p;
        sk.key_lv0.assign(p.n, 0u);
        sk.key_lv1.assign(p.N, 0u);
        check(tfhe_gpu_keygen(ck.ctx(), secret_seed, cloud_seed, sk.key_lv0.data(), sk.key_lv1.data(), nullptr,
                              nullptr),
              "CloudKey.generate", ck.ctx());
        return {std::move(sk), std::move(ck)};
    }
    int numDevices() const { return tfhe_gpu_num_devices(ctx()); }
    void save(const std::string &path) const {
        check(tfhe_gpu_save_cloud_key(ctx(), path.c_str()), "CloudKey.save", ctx());
    }
    tfhe_gpu_ctx *ctx() const { return ctx_.get(); }
    const tfhe_params &params() const { return p_; }

  private:
    struct Del {
        void operator()(tfhe_gpu_ctx *c) const { tfhe_gpu_destroy(c); }
    };
    CloudKey(const tfhe_params &p, int device) : p_(p) {
        tfhe_gpu_ctx *c = nullptr;
        check(tfhe_gpu_create_on_device(&p, device, &c), "tfhe_gpu_create_on_device");
        ctx_.reset(c);
    }
    CloudKey(const tfhe_params &p, const std::vector<int> &devices) : p_(p) {
        tfhe_gpu_ctx *c = nullptr;
        check(tfhe_gpu_create_multi(&p, (int)devices.size(), devices.data(), &c), "tfhe_gpu_create_multi");
        ctx_.reset(c);
    }
    tfhe_params p_{};
    std::unique_ptr<tfhe_gpu_ctx, Del> ctx_;
};

// reencryptTLWELv0 (proxy_reenc.zig:267-306) on the GPU: the key is uploaded once to HBM; a
// context of its own (no cloud key needed).
class HipReencryptor {
  public:
    HipReencryptor(const tfhe_params &p, const ProxyReencryptionKey &k, int device = 0) : p_(p) {
        tfhe_gpu_ctx *c = nullptr;
        check(tfhe_gpu_create_on_device(&p, device, &c), "tfhe_gpu_create_on_device");
        ctx_.reset(c);
        tfhe_gpu_reenc_key *h = nullptr;
        check(tfhe_gpu_reenc_key_load(c, k.key_encryptions.data(), k.key_encryptions.size(), k.basebit, k.t, &h),
              "reenc_key_load", c);
        key_.reset(h);
    }
    std::vector<TLWELv0> reencryptBatch(const std::vector<TLWELv0> &in) const {
        const size_t w = p_.n + 1;
        std::vector<Torus> x(in.size() * w), y(in.size() * w);
        for (size_t k = 0; k < in.size(); k++) std::copy(in[k].p.begin(), in[k].p.end(), x.begin() + k * w);
        check(tfhe_gpu_reencrypt_batch(ctx_.get(), key_.get(), x.data(), y.data(), in.size()), "reencrypt",
              ctx_.get());
        std::vector<TLWELv0> r(in.size(), TLWELv0(p_.n));
        for (size_t k = 0; k < in.size(); k++) std::copy(y.begin() + k * w, y.begin() + (k + 1) * w, r[k].p.begin());
        return r;
    }
    TLWELv0 reencryptTLWELv0(const TLWELv0 &ct) const { return reencryptBatch({ct})[0]; }

  private:
    struct DelCtx {
        void operator()(tfhe_gpu_ctx *c) const { tfhe_gpu_destroy(c); }
    };
    struct DelKey {
        void operator()(tfhe_gpu_reenc_key *k) const { tfhe_gpu_reenc_key_destroy(k); }
    };
    tfhe_params p_{};
    std::unique_ptr<tfhe_gpu_ctx, DelCtx> ctx_;
    std::unique_ptr<tfhe_gpu_reenc_key, DelKey> key_;  // declared after ctx_: destroyed first
};

// bootstrap.zig:30-47 strategy, vanilla.zig:38-75 semantics
class HipBootstrap {
  public:
    TLWELv0 bootstrap(const TLWELv0 &ctxt, const CloudKey &ck) const {
        TLWELv0 out(ctxt.n());
        check(tfhe_gpu_bootstrap_batch(ck.ctx(), ctxt.p.data(), out.p.data(), 1), "bootstrap", ck.ctx());
        return out;
    }
    TLWELv0 bootstrapWithoutKeySwitch(const TLWELv0 &ctxt, const CloudKey &ck) const {
        TLWELv0 out(ctxt.n());
        check(tfhe_gpu_bootstrap_without_key_switch_batch(ck.ctx(), ctxt.p.data(), out.p.data(), 1),
              "bootstrapWithoutKeySwitch", ck.ctx());
        return out;
    }
    const char *name() const { return "mi355x"; }
};

// gates.zig:25-299
class Gates {
  public:
    Gates() = default;
    explicit Gates(HipBootstrap b) : bootstrap_(b) {}  // Gates.withBootstrap
    const char *bootstrapStrategy() const { return bootstrap_.name(); }

    TLWELv0 nandGate(const TLWELv0 &a, const TLWELv0 &b, const CloudKey &ck) const { return one(TFHE_GATE_NAND, a, b, ck); }
    TLWELv0 orGate(const TLWELv0 &a, const TLWELv0 &b, const CloudKey &ck) const { return one(TFHE_GATE_OR, a, b, ck); }
    TLWELv0 andGate(const TLWELv0 &a, const TLWELv0 &b, const CloudKey &ck) const { return one(TFHE_GATE_AND, a, b, ck); }
    TLWELv0 xorGate(const TLWELv0 &a, const TLWELv0 &b, const CloudKey &ck) const { return one(TFHE_GATE_XOR, a, b, ck); }
    TLWELv0 xnorGate(const TLWELv0 &a, const TLWELv0 &b, const CloudKey &ck) const { return one(TFHE_GATE_XNOR, a, b, ck); }
    TLWELv0 norGate(const TLWELv0 &a, const TLWELv0 &b, const CloudKey &ck) const { return one(TFHE_GATE_NOR, a, b, ck); }
    TLWELv0 andNyGate(const TLWELv0 &a, const TLWELv0 &b, const CloudKey &ck) const { return one(TFHE_GATE_ANDNY, a, b, ck); }
    TLWELv0 andYnGate(const TLWELv0 &a, const TLWELv0 &b, const CloudKey &ck) const { return one(TFHE_GATE_ANDYN, a, b, ck); }
    TLWELv0 orNyGate(const TLWELv0 &a, const TLWELv0 &b, const CloudKey &ck) const { return one(TFHE_GATE_ORNY, a, b, ck); }
    TLWELv0 orYnGate(const TLWELv0 &a, const TLWELv0 &b, const CloudKey &ck) const { return one(TFHE_GATE_ORYN, a, b, ck); }

    // muxNaive (gates.zig:124-129): AND(a, b) and AND(NOT a, c) in one batch, then OR
    TLWELv0 muxNaive(const TLWELv0 &a, const TLWELv0 &b, const TLWELv0 &c, const CloudKey &ck) const {
        const std::vector<std::pair<TLWELv0, TLWELv0>> lvl1{{a, b}, {notGate(a), c}};
        const auto r = batch(TFHE_GATE_AND, lvl1, ck);
        return orGate(r[0], r[1], ck);
    }
    TLWELv0 notGate(const TLWELv0 &a) const { return a.neg(); }  // gates.zig:132-135
    TLWELv0 copy(const TLWELv0 &a) const { return a; }           // gates.zig:138-141
    TLWELv0 constant(bool value, size_t n) const {               // gates.zig:144-151
        TLWELv0 r(n);
        const Torus mu = 1u << 29;  // f64ToTorus(0.125)
        r.bMut() = value ? mu : 1u - mu;  // the reference's 1 -% mu
        return r;
    }

    // gates.zig:244-299 declares these (returning error.NotImplemented): one
    // batched GPU launch here
    using Pairs = std::vector<std::pair<TLWELv0, TLWELv0>>;
    std::vector<TLWELv0> batchNand(const Pairs &in, const CloudKey &ck) const { return batch(TFHE_GATE_NAND, in, ck); }
    std::vector<TLWELv0> batchAnd(const Pairs &in, const CloudKey &ck) const { return batch(TFHE_GATE_AND, in, ck); }
    std::vector<TLWELv0> batchOr(const Pairs &in, const CloudKey &ck) const { return batch(TFHE_GATE_OR, in, ck); }
    std::vector<TLWELv0> batchXor(const Pairs &in, const CloudKey &ck) const { return batch(TFHE_GATE_XOR, in, ck); }
    std::vector<TLWELv0> batchNor(const Pairs &in, const CloudKey &ck) const { return batch(TFHE_GATE_NOR, in, ck); }
    std::vector<TLWELv0> batchXnor(const Pairs &in, const CloudKey &ck) const { return batch(TFHE_GATE_XNOR, in, ck); }

    // mixed-op batch: ops[k] applied to (a[k], b[k])
    std::vector<TLWELv0> gateBatch(const std::vector<uint8_t> &ops, const std::vector<TLWELv0> &a,
                                   const std::vector<TLWELv0> &b, const CloudKey &ck) const {
        if (ops.size() != a.size() || a.size() != b.size()) throw Error(TFHE_ERR_INVALID, "gateBatch: size mismatch");
        const size_t w = ck.params().n + 1, B = ops.size();
        std::vector<Torus> fa(B * w), fb(B * w), fo(B * w);
        for (size_t k = 0; k < B; k++) {
            std::copy(a[k].p.begin(), a[k].p.end(), fa.begin() + k * w);
            std::copy(b[k].p.begin(), b[k].p.end(), fb.begin() + k * w);
        }
        check(tfhe_gpu_gate_batch(ck.ctx(), ops.data(), fa.data(), fb.data(), fo.data(), B), "gateBatch", ck.ctx());
        std::vector<TLWELv0> out(B, TLWELv0(ck.params().n));
        for (size_t k = 0; k < B; k++) std::copy(fo.begin() + k * w, fo.begin() + (k + 1) * w, out[k].p.begin());
        return out;
    }

  private:
    TLWELv0 one(uint8_t op, const TLWELv0 &a, const TLWELv0 &b, const CloudKey &ck) const {
        return gateBatch({op}, {a}, {b}, ck)[0];
    }
    std::vector<TLWELv0> batch(uint8_t op, const Pairs &in, const CloudKey &ck) const {
        std::vector<uint8_t> ops(in.size(), op);
        std::vector<TLWELv0> a, b;
        for (const auto &pr : in) {
            a.push_back(pr.first);
            b.push_back(pr.second);
        }
        return gateBatch(ops, a, b, ck);
    }
    HipBootstrap bootstrap_;
};

// Level-scheduled gate circuit (tfhe_gpu_circuit_eval)
class Circuit {
  public:
    using Wire = uint32_t;
    Wire input() {
        if (!ops_.empty()) throw Error(TFHE_ERR_INVALID, "Circuit: declare inputs before gates");
        return n_inputs_++;
    }
    Wire gate(uint8_t op, Wire a, Wire b) {
        const Wire w = (Wire)(n_inputs_ + ops_.size());
        if (a >= w || b >= w) throw Error(TFHE_ERR_INVALID, "Circuit: gate inputs must be existing wires");
        ops_.push_back(op);
        ia_.push_back(a);
        ib_.push_back(b);
        return w;
    }
    Wire andGate(Wire a, Wire b) { return gate(TFHE_GATE_AND, a, b); }
    Wire orGate(Wire a, Wire b) { return gate(TFHE_GATE_OR, a, b); }
    Wire xorGate(Wire a, Wire b) { return gate(TFHE_GATE_XOR, a, b); }
    Wire notGate(Wire a) { return gate(TFHE_GATE_NOT, a, a); }
    Wire muxNaive(Wire a, Wire b, Wire c) { return orGate(andGate(a, b), andGate(notGate(a), c)); }
    // examples/add_two_numbers.zig:24-47
    std::pair<Wire, Wire> fullAdder(Wire a, Wire b, Wire cin) {
        const Wire x = xorGate(a, b), ab = andGate(a, b), xc = andGate(x, cin);
        return {xorGate(x, cin), orGate(ab, xc)};
    }
    void output(Wire w) { outs_.push_back(w); }

    std::vector<TLWELv0> run(const CloudKey &ck, const std::vector<TLWELv0> &inputs, uint32_t *levels = nullptr) const {
        if (inputs.size() != n_inputs_) throw Error(TFHE_ERR_INVALID, "Circuit: wrong number of inputs");
        const size_t w = ck.params().n + 1;
        std::vector<Torus> in(inputs.size() * w), out(outs_.size() * w);
        for (size_t k = 0; k < inputs.size(); k++) std::copy(inputs[k].p.begin(), inputs[k].p.end(), in.begin() + k * w);
        check(tfhe_gpu_circuit_eval(ck.ctx(), n_inputs_, in.data(), ops_.size(), ops_.data(), ia_.data(), ib_.data(),
                                    outs_.size(), outs_.data(), out.data(), levels),
              "Circuit.run", ck.ctx());
        std::vector<TLWELv0> r(outs_.size(), TLWELv0(ck.params().n));
        for (size_t k = 0; k < outs_.size(); k++) std::copy(out.begin() + k * w, out.begin() + (k + 1) * w, r[k].p.begin());
        return r;
    }
    // Inputs (numInputs() TLWELv0 words, row-major) and outputs (numOutputs()) in HBM;
    // async on the context stream (tfhe_gpu_circuit_eval_dev). Returns the bootstrap depth.
    uint32_t runDevice(const CloudKey &ck, const Torus *inputs_dev, Torus *outputs_dev) const {
        uint32_t levels = 0;
        check(tfhe_gpu_circuit_eval_dev(ck.ctx(), n_inputs_, inputs_dev, ops_.size(), ops_.data(), ia_.data(),
                                        ib_.data(), outs_.size(), outs_.data(), outputs_dev, &levels),
              "Circuit.runDevice", ck.ctx());
        return levels;
    }
    size_t numInputs() const { return n_inputs_; }
    size_t numOutputs() const { return outs_.size(); }

  private:
    uint32_t n_inputs_ = 0;
    std::vector<uint8_t> ops_;
    std::vector<uint32_t> ia_, ib_, outs_;
};

}  // namespace tfhe
