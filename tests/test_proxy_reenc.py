"""Proxy re-encryption: proxy_reenc.zig.

CPU part: the oracle restates PublicKeyLv0 / ProxyReencryptionKey /
reencryptTLWELv0 (proxy_reenc.zig:35-306) and passes the reference's own tests
(proxy_reenc.zig:310-455, restated below with fixed seeds in place of
getUniqueSeed()); the product library's host key generation is bit-identical to
the oracle's.  GPU part (-m gpu): HipReencryptor (the key-switch lane kernel
over a TLWELv0 input) is bit-exact against oracle.reencrypt.
"""
import ctypes as C

import numpy as np
import pytest

import tfhe_amd
from conftest import rng

N128 = "128"


@pytest.fixture(scope="module")
def P():
    from oracle import params
    return params(N128)


@pytest.fixture(scope="module")
def TP():
    return tfhe_amd.make_params(N128)


@pytest.fixture(scope="module")
def keys(oracle, P):
    """alice / bob / carol lv0 keys (SecretKey.new, key.zig:41-57) and bob's / carol's public keys
    (PublicKeyLv0.new: 2n encryptions of zero at tlwe_lv0.ALPHA, proxy_reenc.zig:44-54)."""
    ks = {name: oracle.secret_key(P, seed)[0] for name, seed in (("alice", 11), ("bob", 12), ("carol", 13))}
    pks = {name: oracle.public_key_gen(P.n, ks[name], 2 * P.n, P.alpha_lv0, seed)
           for name, seed in (("bob", 100_000), ("carol", 200_000))}
    return ks, pks


@pytest.fixture(scope="module")
def reenc_ab(oracle, P, keys):
    """ProxyReencryptionKey.newAsymmetric(alice, bob_public) (proxy_reenc.zig:131-147)."""
    ks, pks = keys
    return oracle.reenc_key_gen(P.n, ks["alice"], P.alpha_ksk, P.basebit, P.iks_t, 1_000_000, pk=pks["bob"])


def _zig_bools(oracle, seed, count):
    """std.Random.DefaultPrng.init(seed).random().boolean() x count (the tests' message stream)."""
    r = (C.c_uint64 * 4)()
    oracle.lib.oracle_rng_init(C.byref(r), C.c_uint64(seed))
    return [bool(oracle.lib.oracle_rng_bool(C.byref(r))) for _ in range(count)]


# ---- the reference's tests (proxy_reenc.zig:310-455) on the oracle ---------------------------------

def test_public_key_encryption(oracle, P, keys):
    """proxy_reenc.zig:310-323."""
    ks, pks = keys
    for i, msg in enumerate((True, False)):
        ct = oracle.public_key_encrypt_f64(P.n, pks["bob"], 0.125 if msg else -0.125, P.alpha_lv0, 7 + i)
        assert oracle.tlwe_decrypt_bool(P.n, ct, ks["bob"]) == msg


def test_public_key_encryption_multiple(oracle, P, keys):
    """proxy_reenc.zig:325-345: 100 messages from DefaultPrng(42), accuracy > 0.95."""
    ks, pks = keys
    msgs = _zig_bools(oracle, 42, 100)
    ok = sum(oracle.tlwe_decrypt_bool(P.n, oracle.public_key_encrypt_f64(
        P.n, pks["bob"], 0.125 if m else -0.125, P.alpha_lv0, 300 + i), ks["bob"]) == m for i, m in enumerate(msgs))
    assert ok / 100 > 0.95


def test_reencryption_asymmetric(oracle, P, keys, reenc_ab):
    """proxy_reenc.zig:347-374."""
    ks, _ = keys
    for i, msg in enumerate((True, False)):
        ct = oracle.tlwe_encrypt_bool(P.n, msg, P.alpha_lv0, ks["alice"], 40 + i)
        assert oracle.tlwe_decrypt_bool(P.n, ct, ks["alice"]) == msg
        bob_ct = oracle.reencrypt(P.n, P.basebit, P.iks_t, ct, reenc_ab)
        assert oracle.tlwe_decrypt_bool(P.n, bob_ct, ks["bob"]) == msg


def test_reencryption_symmetric(oracle, P, keys):
    """proxy_reenc.zig:376-398."""
    ks, _ = keys
    key = oracle.reenc_key_gen(P.n, ks["alice"], P.alpha_ksk, P.basebit, P.iks_t, 2_000_000, key_to=ks["bob"])
    for i, msg in enumerate((True, False)):
        ct = oracle.tlwe_encrypt_bool(P.n, msg, P.alpha_lv0, ks["alice"], 50 + i)
        assert oracle.tlwe_decrypt_bool(P.n, ct, ks["alice"]) == msg
        bob_ct = oracle.reencrypt(P.n, P.basebit, P.iks_t, ct, key)
        assert oracle.tlwe_decrypt_bool(P.n, bob_ct, ks["bob"]) == msg


def test_reencryption_asymmetric_multiple(oracle, P, keys, reenc_ab):
    """proxy_reenc.zig:400-425: accuracy > 0.90 over 100 messages."""
    ks, _ = keys
    msgs = _zig_bools(oracle, 42, 100)
    ok = 0
    for i, m in enumerate(msgs):
        ct = oracle.tlwe_encrypt_bool(P.n, m, P.alpha_lv0, ks["alice"], 600 + i)
        ok += oracle.tlwe_decrypt_bool(P.n, oracle.reencrypt(P.n, P.basebit, P.iks_t, ct, reenc_ab), ks["bob"]) == m
    assert ok / 100 > 0.90


def test_reencryption_chain_asymmetric(oracle, P, TP, keys, reenc_ab):
    """proxy_reenc.zig:427-455: alice -> bob -> carol.  The bob -> carol key comes from the product
    library's host key generation (bit-identical to the oracle's, next test)."""
    ks, pks = keys
    bob = tfhe_amd.SecretKey(TP, ks["bob"], np.zeros(TP.N, np.uint32))
    pk_c = tfhe_amd.PublicKeyLv0.__new__(tfhe_amd.PublicKeyLv0)
    pk_c.params, pk_c.encryptions = TP, pks["carol"]
    bc = tfhe_amd.ProxyReencryptionKey.new_asymmetric(bob, pk_c, 3_000_000).key_encryptions
    ct = oracle.tlwe_encrypt_bool(P.n, True, P.alpha_lv0, ks["alice"], 77)
    bob_ct = oracle.reencrypt(P.n, P.basebit, P.iks_t, ct, reenc_ab)
    assert oracle.tlwe_decrypt_bool(P.n, bob_ct, ks["bob"])
    carol_ct = oracle.reencrypt(P.n, P.basebit, P.iks_t, bob_ct, bc)
    assert oracle.tlwe_decrypt_bool(P.n, carol_ct, ks["carol"])


# ---- the product's host key generation == the oracle's ------------------------------------------

def test_host_keygen_matches_oracle(oracle, P, TP, keys, reenc_ab):
    ks, pks = keys
    alice = tfhe_amd.secret_key_new(TP, 11)
    assert np.array_equal(alice.key_lv0, ks["alice"])
    assert np.array_equal(alice.key_lv1, oracle.secret_key(P, 11)[1])
    bob = tfhe_amd.secret_key_new(TP, 12)
    pk = tfhe_amd.PublicKeyLv0(bob, 100_000)
    assert np.array_equal(pk.encryptions, pks["bob"])
    # encryptBool through the public key, item i on DefaultPrng(seed0 + i)
    bits = rng(3).integers(0, 2, 8).astype(np.uint8)
    got = pk.encrypt_bool(bits, seed0=900)
    want = [oracle.public_key_encrypt_f64(P.n, pks["bob"], 0.125 if b else -0.125, P.alpha_lv0, 900 + i)
            for i, b in enumerate(bits)]
    assert np.array_equal(got, np.array(want))
    assert np.array_equal(bob.decrypt_bool(got), bits.astype(bool))
    # asymmetric and symmetric re-encryption keys
    ab = tfhe_amd.ProxyReencryptionKey.new_asymmetric(alice, pk, 1_000_000)
    assert (ab.basebit, ab.t) == (P.basebit, P.iks_t)
    assert np.array_equal(ab.key_encryptions, reenc_ab)
    sym = tfhe_amd.ProxyReencryptionKey.new_symmetric(alice, bob, 5, basebit=4, t=4)
    want = oracle.reenc_key_gen(P.n, ks["alice"], P.alpha_ksk, 4, 4, 5, key_to=ks["bob"])
    assert np.array_equal(sym.key_encryptions, want)
    # k = 0 entries stay zero (proxy_reenc.zig:162-165)
    assert not sym.key_encryptions.reshape(P.n, 4, 16, P.n + 1)[:, :, 0].any()


def test_reencrypt_edge_digits(oracle, P, keys, reenc_ab):
    """Inputs whose digits are all 0 / all (base-1), and the rounding carry out of the top digit."""
    ks, _ = keys
    for fill in (0, 0xFFFFFFFF, 0x7FFFFFFF, 1 << (32 - (1 + P.basebit * P.iks_t))):
        ct = np.full(P.n + 1, fill, np.uint32)
        out = oracle.reencrypt(P.n, P.basebit, P.iks_t, ct, reenc_ab)
        # the result decrypts (under bob) to what the input decrypts to under alice, up to key noise
        ph_in = int(oracle.tlwe_phase(P.n, ct, ks["alice"]))
        ph_out = int(oracle.tlwe_phase(P.n, out, ks["bob"]))
        d = (ph_out - ph_in) & 0xFFFFFFFF
        assert min(d, 2**32 - d) < 2**32 // 8
    zero = np.zeros(P.n + 1, np.uint32)
    assert not oracle.reencrypt(P.n, P.basebit, P.iks_t, zero, reenc_ab).any()


# ---- GPU: HipReencryptor bit-exact against the oracle -------------------------------------------

def _random_cts(P, B, seed):
    return rng(seed).integers(0, 2**32, (B, P.n + 1), dtype=np.uint64).astype(np.uint32)


@pytest.mark.gpu
def test_gpu_reencrypt_matches_oracle(oracle, P, keys, reenc_ab):
    ks, _ = keys
    ctx = tfhe_amd.Context(N128, device=0)
    hr = tfhe_amd.HipReencryptor(ctx, tfhe_amd.ProxyReencryptionKey(reenc_ab, P.basebit, P.iks_t))
    # real ciphertexts: decrypt under bob after the GPU re-encryption
    msgs = rng(5).integers(0, 2, 257).astype(bool)
    cts = np.array([oracle.tlwe_encrypt_bool(P.n, m, P.alpha_lv0, ks["alice"], 10_000 + i)
                    for i, m in enumerate(msgs)])
    got = hr.reencrypt(cts)
    for i in range(0, len(msgs), 16):
        assert np.array_equal(got[i], oracle.reencrypt(P.n, P.basebit, P.iks_t, cts[i], reenc_ab))
    dec = np.array([oracle.tlwe_decrypt_bool(P.n, c, ks["bob"]) for c in got])
    assert (dec == msgs).mean() > 0.98
    # uniformly random inputs (every digit value, every rounding carry), ragged batch sizes
    for B in (1, 63, 65, 300):
        x = _random_cts(P, B, B)
        g = hr.reencrypt(x)
        for i in sorted({0, B // 2, B - 1}):
            assert np.array_equal(g[i], oracle.reencrypt(P.n, P.basebit, P.iks_t, x[i], reenc_ab)), (B, i)
    hr.close()
    ctx.close()


@pytest.mark.gpu
def test_gpu_reencrypt_gemm_and_lanes_agree(oracle, P, keys, reenc_ab):
    """The one-hot GEMM key switch (the default at basebit 2)
    over the n = 700 input coefficients (88 blocks of 8, the last half padding)
    against the lane form, bit for bit, and the oracle on samples."""
    ctx = tfhe_amd.Context(N128, device=0)
    hr = tfhe_amd.HipReencryptor(ctx, tfhe_amd.ProxyReencryptionKey(reenc_ab, P.basebit, P.iks_t))
    x = _random_cts(P, 1500, 1500)
    g = hr.reencrypt(x)
    assert "k_key_switch_gemm<9,2>" in ctx.last_kernels()
    with ctx.options(ks_form=0):
        lanes = hr.reencrypt(x)
        assert "k_key_switch_lanes<" in ctx.last_kernels()
    assert np.array_equal(g, lanes)
    for i in (0, 511, 512, 1499):
        assert np.array_equal(g[i], oracle.reencrypt(P.n, P.basebit, P.iks_t, x[i], reenc_ab)), i
    hr.close()
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("ks_form", [3, 0])
def test_gpu_reencrypt_device_resident(oracle, P, keys, reenc_ab, ks_form):
    """tfhe_gpu_reencrypt_batch_dev (device buffers, async on the context stream):
    the host-buffer call's words for ragged batches, in both key-switch forms,
    with the input buffer sized exactly (the GEMM's whole-block reads go through
    the staging copy's slack), and the oracle on samples."""
    import torch
    ctx = tfhe_amd.Context(N128, device=0)
    hr = tfhe_amd.HipReencryptor(ctx, tfhe_amd.ProxyReencryptionKey(reenc_ab, P.basebit, P.iks_t))
    try:
        with ctx.options(ks_form=ks_form):
            for B in (1, 65, 1500):
                x = _random_cts(P, B, 300 + B)
                want = hr.reencrypt(x)
                t_in = torch.from_numpy(x.view(np.int32)).to("cuda:0")
                t_out = torch.zeros_like(t_in)
                ctx.set_stream(torch.cuda.current_stream().cuda_stream)
                hr.reencrypt_dev(t_in.data_ptr(), t_out.data_ptr(), B)
                ctx.sync()
                got = t_out.cpu().numpy().view(np.uint32)
                assert np.array_equal(got, want), B
                assert np.array_equal(got[B - 1], oracle.reencrypt(P.n, P.basebit, P.iks_t, x[B - 1], reenc_ab))
    finally:
        ctx.set_stream(None)
        hr.close()
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("pname,basebit,t", [("80", 2, 7), ("128", 4, 4), ("uint4", 5, 3)])
def test_gpu_reencrypt_other_bases(oracle, pname, basebit, t):
    from oracle import params
    p = params(pname)
    a0 = oracle.secret_key(p, 21)[0]
    b0 = oracle.secret_key(p, 22)[0]
    key = oracle.reenc_key_gen(p.n, a0, p.alpha_ksk, basebit, t, 99, key_to=b0)
    ctx = tfhe_amd.Context(pname, device=0)
    hr = tfhe_amd.HipReencryptor(ctx, tfhe_amd.ProxyReencryptionKey(key, basebit, t))
    x = _random_cts(p, 130, 7)
    g = hr.reencrypt(x)
    for i in (0, 64, 129):
        assert np.array_equal(g[i], oracle.reencrypt(p.n, basebit, t, x[i], key)), i
    hr.close()
    ctx.close()


@pytest.mark.gpu
def test_gpu_reencrypt_chain(oracle, P, keys, reenc_ab):
    """alice -> bob -> carol entirely on the GPU (proxy_reenc.zig:427-455)."""
    ks, pks = keys
    bc = oracle.reenc_key_gen(P.n, ks["bob"], P.alpha_ksk, P.basebit, P.iks_t, 3_000_000, pk=pks["carol"])
    ctx = tfhe_amd.Context(N128, device=0)
    h_ab = tfhe_amd.HipReencryptor(ctx, tfhe_amd.ProxyReencryptionKey(reenc_ab, P.basebit, P.iks_t))
    h_bc = tfhe_amd.HipReencryptor(ctx, tfhe_amd.ProxyReencryptionKey(bc, P.basebit, P.iks_t))
    msgs = rng(9).integers(0, 2, 64).astype(bool)
    cts = np.array([oracle.tlwe_encrypt_bool(P.n, m, P.alpha_lv0, ks["alice"], 20_000 + i)
                    for i, m in enumerate(msgs)])
    carol = h_bc.reencrypt(h_ab.reencrypt(cts))
    dec = np.array([oracle.tlwe_decrypt_bool(P.n, c, ks["carol"]) for c in carol])
    assert (dec == msgs).mean() > 0.95
    h_ab.close()
    h_bc.close()
    ctx.close()


def test_reenc_key_load_rejects_bad_shapes(TP):
    """Argument checks run before any device work (no GPU needed for the error path)."""
    lib = tfhe_amd.load_library()
    h = C.c_void_p()
    assert lib.tfhe_gpu_reenc_key_load(None, None, 0, 2, 9, C.byref(h)) != 0
    assert lib.tfhe_gpu_reencrypt_batch(None, None, None, None, 0) != 0
