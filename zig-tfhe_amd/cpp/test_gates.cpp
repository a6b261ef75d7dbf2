// C++ parity tests over the host-side mirror (tfhe.hpp), written as the
// reference's own gate tests are (src/gates.zig:374-544: each gate's truth
// table through encryptBool -> gate -> decryptBool, 128-bit parameters), plus
// muxNaive, notGate / copy / constant, the bootstrap strategy, the batch
// functions gates.zig:244-299 declares, a level-scheduled circuit, and the
// proxy re-encryption tests of src/proxy_reenc.zig:310-455.
// Runs on one MI355X; exit status 0 = all passed.
#include "tfhe.hpp"

#include <cstdio>
#include <functional>

namespace {
int failures = 0;
void expect(bool ok, const char *test, const char *what) {
    if (!ok) {
        std::printf("FAIL %s: %s\n", test, what);
        failures++;
    }
}
}  // namespace

int main() {
    using namespace tfhe;
    auto [sk, ck] = CloudKey::generate(params::SECURITY_128_BIT(), 42, 43);
    const Gates gates;
    uint64_t seed = 1000;
    auto enc = [&, &sk = sk](bool b) { return sk.encryptBool(b, seed++); };

    struct Case {
        const char *name;
        std::function<TLWELv0(const TLWELv0 &, const TLWELv0 &)> gate;
        std::function<bool(bool, bool)> truth;
    };
    const Case cases[] = {
        {"gates all NAND cases", [&, &ck = ck](auto &a, auto &b) { return gates.nandGate(a, b, ck); }, [](bool a, bool b) { return !(a && b); }},
        {"gates all AND cases", [&, &ck = ck](auto &a, auto &b) { return gates.andGate(a, b, ck); }, [](bool a, bool b) { return a && b; }},
        {"gates all OR cases", [&, &ck = ck](auto &a, auto &b) { return gates.orGate(a, b, ck); }, [](bool a, bool b) { return a || b; }},
        {"gates all XOR cases", [&, &ck = ck](auto &a, auto &b) { return gates.xorGate(a, b, ck); }, [](bool a, bool b) { return a != b; }},
        // the reference's xnorGate computes a - 2b + 1/4, which decrypts as XOR (tests/test_oracle.py)
        {"gates all XNOR cases (reference semantics)", [&, &ck = ck](auto &a, auto &b) { return gates.xnorGate(a, b, ck); }, [](bool a, bool b) { return a != b; }},
        {"gates all NOR cases", [&, &ck = ck](auto &a, auto &b) { return gates.norGate(a, b, ck); }, [](bool a, bool b) { return !(a || b); }},
        {"gates all ANDNY cases", [&, &ck = ck](auto &a, auto &b) { return gates.andNyGate(a, b, ck); }, [](bool a, bool b) { return !a && b; }},
        {"gates all ANDYN cases", [&, &ck = ck](auto &a, auto &b) { return gates.andYnGate(a, b, ck); }, [](bool a, bool b) { return a && !b; }},
        {"gates all ORNY cases", [&, &ck = ck](auto &a, auto &b) { return gates.orNyGate(a, b, ck); }, [](bool a, bool b) { return !a || b; }},
        {"gates all ORYN cases", [&, &ck = ck](auto &a, auto &b) { return gates.orYnGate(a, b, ck); }, [](bool a, bool b) { return a || !b; }},
    };
    for (const auto &c : cases) {
        for (int x = 0; x < 4; x++) {
            const bool a = x & 2, b = x & 1;
            const TLWELv0 r = c.gate(enc(a), enc(b));
            expect(sk.decryptBool(r) == c.truth(a, b), c.name, a ? (b ? "1,1" : "1,0") : (b ? "0,1" : "0,0"));
        }
        std::printf("ok   %s\n", c.name);
    }
    for (int x = 0; x < 8; x++) {  // gates.zig:124-129
        const bool a = x & 4, b = x & 2, c = x & 1;
        const TLWELv0 r = gates.muxNaive(enc(a), enc(b), enc(c), ck);
        expect(sk.decryptBool(r) == (a ? b : c), "gates mux", "case");
    }
    std::printf("ok   gates mux\n");
    for (bool a : {false, true}) {  // gates.zig:132-151
        expect(sk.decryptBool(gates.notGate(enc(a))) == !a, "gates not", "case");
        expect(sk.decryptBool(gates.copy(enc(a))) == a, "gates copy", "case");
        expect(sk.decryptBool(gates.constant(a, ck.params().n)) == a, "gates constant", "case");
    }
    std::printf("ok   gates not / copy / constant\n");
    expect(std::string(gates.bootstrapStrategy()) == "mi355x", "bootstrap strategy", "name");
    const HipBootstrap bs;
    for (bool a : {false, true}) {  // vanilla.zig:38-69
        const TLWELv0 ct = enc(a);
        expect(sk.decryptBool(bs.bootstrap(ct, ck)) == a, "bootstrap", "refresh keeps the bit");
        expect(bs.bootstrapWithoutKeySwitch(ct, ck).p.size() == ct.p.size(), "bootstrapWithoutKeySwitch", "size");
    }
    std::printf("ok   bootstrap strategy\n");
    Gates::Pairs pairs;  // gates.zig:244-299 (NotImplemented in the reference)
    std::vector<bool> want;
    for (int k = 0; k < 64; k++) {
        const bool a = (k * 7) & 1, b = (k * 13) & 2;
        pairs.push_back({enc(a), enc(b)});
        want.push_back(!(a && b));
    }
    const auto outs = gates.batchNand(pairs, ck);
    for (size_t k = 0; k < outs.size(); k++) expect(sk.decryptBool(outs[k]) == want[k], "batchNand", "element");
    std::printf("ok   batchNand (64 gates)\n");
    try {
        gates.gateBatch({0, 1}, {enc(true)}, {enc(true)}, ck);
        expect(false, "errors", "size mismatch not reported");
    } catch (const Error &e) {
        expect(e.status == TFHE_ERR_INVALID, "errors", "status");
    }
    std::printf("ok   error reporting\n");
    {  // examples/add_two_numbers.zig: 402 + 304 = 706 as one circuit
        Circuit c;
        std::vector<Circuit::Wire> A, B;
        for (int i = 0; i < 16; i++) A.push_back(c.input());
        for (int i = 0; i < 16; i++) B.push_back(c.input());
        Circuit::Wire carry = c.input();
        for (int i = 0; i < 16; i++) {
            auto [s, co] = c.fullAdder(A[i], B[i], carry);
            c.output(s);
            carry = co;
        }
        std::vector<TLWELv0> in;
        for (int i = 0; i < 16; i++) in.push_back(enc((402 >> i) & 1));
        for (int i = 0; i < 16; i++) in.push_back(enc((304 >> i) & 1));
        in.push_back(enc(false));
        uint32_t levels = 0;
        const auto sum = c.run(ck, in, &levels);
        uint32_t v = 0;
        for (int i = 0; i < 16; i++) v |= (uint32_t)sk.decryptBool(sum[i]) << i;
        expect(v == 706, "add_two_numbers circuit", "402 + 304");
        expect(levels == 33, "add_two_numbers circuit", "depth");
        std::printf("ok   add_two_numbers circuit (402 + 304 = %u, %u levels)\n", v, levels);
    }
    {  // proxy_reenc.zig:310-455: public key, symmetric, asymmetric, chain alice -> bob -> carol
        const tfhe_params p = params::SECURITY_128_BIT();
        const SecretKey alice = SecretKey::newWithSeed(p, 11), bob = SecretKey::newWithSeed(p, 12),
                        carol = SecretKey::newWithSeed(p, 13);
        const PublicKeyLv0 bob_pk = PublicKeyLv0::create(bob, 100000), carol_pk = PublicKeyLv0::create(carol, 200000);
        for (bool m : {true, false})
            expect(bob.decryptBool(bob_pk.encryptBool(m, p.alpha_lv0, 7 + m)) == m, "public key encryption", "bit");
        const HipReencryptor sym(p, ProxyReencryptionKey::newSymmetric(alice, bob, 5));
        const HipReencryptor ab(p, ProxyReencryptionKey::newAsymmetric(alice, bob_pk, 1000000));
        const HipReencryptor bc(p, ProxyReencryptionKey::newAsymmetric(bob, carol_pk, 3000000));
        for (bool m : {true, false}) {
            const TLWELv0 ct = alice.encryptBool(m, 50 + m);
            expect(bob.decryptBool(sym.reencryptTLWELv0(ct)) == m, "proxy reencryption symmetric", "bit");
            expect(bob.decryptBool(ab.reencryptTLWELv0(ct)) == m, "proxy reencryption asymmetric", "bit");
        }
        std::vector<TLWELv0> batch;
        std::vector<bool> bits;
        for (int k = 0; k < 100; k++) {
            bits.push_back((k * 2654435761u >> 7) & 1);
            batch.push_back(alice.encryptBool(bits.back(), 600 + k));
        }
        const auto carol_cts = bc.reencryptBatch(ab.reencryptBatch(batch));
        int ok = 0;
        for (int k = 0; k < 100; k++) ok += carol.decryptBool(carol_cts[k]) == bits[k];
        expect(ok >= 90, "proxy reencryption chain asymmetric", "accuracy");
        std::printf("ok   proxy reencryption (symmetric, asymmetric, chain: %d/100)\n", ok);
    }
    {  // key file: CloudKey.save -> CloudKey.loadFile drives the same gate (no reference counterpart)
        const std::string path = "/tmp/tfhe_cpp_mirror_ck128.key";
        ck.save(path);
        const CloudKey ck2 = CloudKey::loadFile(params::SECURITY_128_BIT(), path);
        const TLWELv0 x = enc(true), y = enc(false);
        expect(gates.nandGate(x, y, ck).p == gates.nandGate(x, y, ck2).p, "key file", "same NAND bits");
        std::printf("ok   key file save / loadFile\n");
        // the same key on a two-shard multi-device context (one GPU listed twice): a
        // batch split over both shards gives the single-device bits
        const CloudKey ckm = CloudKey::loadFile(params::SECURITY_128_BIT(), path, std::vector<int>{0, 0});
        expect(ckm.numDevices() == 2, "multi-device", "two shards");
        std::vector<std::pair<TLWELv0, TLWELv0>> in;
        for (int k = 0; k < 7; k++) in.push_back({enc(k & 1), enc((k >> 1) & 1)});
        const auto one = gates.batchNand(in, ck), two = gates.batchNand(in, ckm);
        bool same = one.size() == two.size();
        for (size_t k = 0; same && k < one.size(); k++) same = one[k].p == two[k].p;
        expect(same, "multi-device", "same NAND batch bits");
        std::remove(path.c_str());
        std::printf("ok   multi-device context (two shards) batch\n");
    }
    std::printf("%s (%d failures)\n", failures ? "FAILED" : "PASSED", failures);
    return failures ? 1 : 0;
}
