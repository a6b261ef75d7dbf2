"""GPU parity tests: every stage of the MI355X path, through the C ABI,
bit-exact against the CPU oracle (oracle/tfhe_oracle.c) on the same seeded
inputs, plus size-independent properties at full batch size.

Bit-exact means equal u32 words; for the f64 FFT stage it means equal f64
values (+0.0 == -0.0: signs of zero never reach an output integer).
"""
import os

import numpy as np
import pytest

import tfhe_amd
from conftest import crafted_near_tie_case, get_keys, rng

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def u32rand(g, *shape):
    return g.integers(0, 1 << 32, shape, dtype=np.uint64).astype(np.uint32)


_CTX = {}


def ctx_for(oracle, pname):
    """Context with the oracle's seeded cloud key loaded (sk 42, ck 43)."""
    if pname not in _CTX:
        k = get_keys(oracle, pname)
        c = tfhe_amd.Context(pname, 0)
        c.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk, k.ck.ksk)
        _CTX[pname] = (c, k)
    return _CTX[pname]


# ---- FFT (fft.zig:293-443) -------------------------------------------------
def test_fft_forward_golden_and_random(oracle):
    c, _ = ctx_for(oracle, "80")
    g = np.load(os.path.join(GOLDEN, "oracle_vectors.npz"))
    assert np.array_equal(c.fft_forward(g["fft_in"]), g["fft_fwd"])
    x = u32rand(rng(1), 64, 1024)
    want = np.array([oracle.ifft(p) for p in x])
    assert np.array_equal(c.fft_forward(x), want)


def test_fft_inverse_golden_and_random(oracle):
    c, _ = ctx_for(oracle, "80")
    g = np.load(os.path.join(GOLDEN, "oracle_vectors.npz"))
    assert np.array_equal(c.fft_inverse(g["fft_fwd"]), g["fft_inv"])
    # MAC-like spectra: sums of products of digits and key spectra
    f = rng(2).normal(0, 2.0 ** 40, (64, 1024))
    want = np.array([oracle.fft(v) for v in f])
    assert np.array_equal(c.fft_inverse(f), want)


@pytest.mark.parametrize("small_b", [True, False])
def test_poly_mul(oracle, small_b):  # fft.zig:458-492
    c, _ = ctx_for(oracle, "80")
    g = rng(3)
    a = u32rand(g, 32, 1024)
    b = u32rand(g, 32, 1024)
    if small_b:
        b %= 64
    want = np.array([oracle.poly_mul(x, y) for x, y in zip(a, b)])
    assert np.array_equal(c.poly_mul(a, b), want)


# ---- external product / key switch (trgsw.zig) -----------------------------
@pytest.mark.parametrize("pname", ["128", "uint4"])
def test_external_product_vs_oracle(oracle, pname):
    c, k = ctx_for(oracle, pname)
    p = k.p
    g = rng(4)
    x = u32rand(g, 8, 2048)
    trgsw = oracle.trgsw_encrypt_torus_fft(p, 1, p.alpha_bsk, k.k1, 17)
    want = np.array([oracle.external_product(p, trgsw, t, k.ck.offset) for t in x])
    assert np.array_equal(c.external_product(x, trgsw_fft=trgsw), want)
    # against a row of the resident key
    want = np.array([oracle.external_product(p, k.ck.bk[5], t, k.ck.offset) for t in x])
    assert np.array_equal(c.external_product(x, bk_index=5), want)


@pytest.mark.parametrize("form", ["lanes", "lanes-narrow", "sel", "gemm"])
@pytest.mark.parametrize("pname,B", [("128", 9), ("128", 130), ("80", 1), ("80", 65), ("uint4", 17), ("uint4", 300)])
def test_key_switch_vs_oracle(oracle, pname, B, form):
    """All key-switch forms (lane = item in wide / narrow blocks, lane = word,
    one-hot GEMM on the matrix cores) bit-exact, ragged B."""
    c, k = ctx_for(oracle, pname)
    lv1 = u32rand(rng(5), B, 1025)
    want = np.array([oracle.identity_key_switch(k.p, v, k.ck.ksk) for v in lv1])
    with c.options(ks_form={"sel": 1, "gemm": 2}.get(form, 0), ks_narrow=int(form.endswith("narrow"))):
        assert np.array_equal(c.key_switch(lv1), want)
        if form == "gemm":
            assert "k_key_switch_gemm<" in c.last_kernels()


@pytest.mark.parametrize("B", [1024, 1500])
def test_key_switch_gemm_full_batches(oracle, B):
    """The gemm form at the headline batch (5 K splits over 220 workgroups) and
    a ragged one: bit-identical to the lane form, and to the oracle on samples
    from the first and last item groups and the last output tile."""
    c, k = ctx_for(oracle, "128")
    lv1 = u32rand(rng(B), B, 1025)
    lanes = c.key_switch(lv1)
    with c.options(ks_form=2):
        got = c.key_switch(lv1)
        assert "k_key_switch_gemm<9,2>" in c.last_kernels()
    assert np.array_equal(got, lanes)
    for i in (0, 511, 512, B - 1):
        assert np.array_equal(got[i], oracle.identity_key_switch(k.p, lv1[i], k.ck.ksk))


# ---- blind rotation / bootstrap ---------------------------------------------
@pytest.mark.parametrize("form", ["whole", "whole-reference", "wide", "wide-reference", "octo", "octo-reference"])
@pytest.mark.parametrize("pname,B", [("80", 3), ("128", 2), ("uint4", 2)])
def test_blind_rotate_vs_oracle(oracle, pname, B, form):
    """Every product kernel form (1 wave per item with loader waves / 8 waves
    per item / the octo form's 8 items per workgroup at L = 1), fused or
    reference arithmetic, bit-exact.  The octo form exists at L = 1 only: the
    option is refused at L = 3."""
    c, k = ctx_for(oracle, pname)
    if form.startswith("octo") and pname != "uint4":
        with pytest.raises(tfhe_amd.TfheError, match="L = 1 only"):
            c.set_option("br_form", "octo")
        assert c.get_option("br_form") == 0
        return
    cts = u32rand(rng(6), B, k.p.n + 1)  # uniform TLWE: bit-exactness only
    want = np.array([oracle.blind_rotate(k.p, t, k.ck.testvec, k.ck.bk, k.ck.offset) for t in cts])
    # odd batch sizes leave idle item slots in the last workgroup
    cts5 = u32rand(rng(16), 5, k.p.n + 1)
    want5 = np.array([oracle.blind_rotate(k.p, t, k.ck.testvec, k.ck.bk, k.ck.offset) for t in cts5])
    with c.options(br_form=form.split("-")[0], arith=int(form.endswith("reference"))):
        assert np.array_equal(c.blind_rotate_batch(cts), want)
        # fused arithmetic only where the external product is exact (SMALL)
        assert c.last_kernels().split(" + ")[0].endswith("fused)") == (pname != "uint4" and not form.endswith("reference"))
        # the whole form at L = 3 with the fused arithmetic is the loader-assist kernel
        assist = form == "whole" and pname != "uint4"
        prefix = {"whole": "k_blind_rotate_assist<" if assist else "k_blind_rotate<", "octo": "k_blind_rotate_octo<",
                  "wide": "k_blind_rotate_wide<"}
        assert c.last_kernels().startswith(prefix[form.split("-")[0]])
        assert np.array_equal(c.blind_rotate_batch(cts5), want5)


@pytest.mark.parametrize("form,pname", [("whole", "80"), ("octo", "uint4")])
def test_whole_form_every_idle_slot_count(oracle, form, pname):
    """Whole form at B = 1..8: the last workgroup has 3, 2, 1 or 0 idle gate slots
    (clamped copies of the last item: they read in bounds, follow the slot
    schedule and store nothing); the octo form (8 items per workgroup, L = 1) at
    B = 1..9 has 7..0 idle slots.  Regression for the round-1 development fault
    in test_blind_rotate_vs_oracle[80-3-whole]."""
    c, k = ctx_for(oracle, pname)
    cts = u32rand(rng(17), 9, k.p.n + 1)
    want = np.array([oracle.blind_rotate(k.p, t, k.ck.testvec, k.ck.bk, k.ck.offset) for t in cts])
    with c.options(br_form=form):
        for B in range(1, 10 if form == "octo" else 9):
            assert np.array_equal(c.blind_rotate_batch(cts[:B]), want[:B]), B


@pytest.mark.parametrize("name,value", [("br_form", 6), ("br_form", 7), ("br_form", 2), ("br_form", 4),
                                        ("br_loader", 0), ("br_sync", 0)])
def test_ab_only_forms_are_refused(oracle, name, value):
    """The product library carries only its dispatchable forms: the duo and
    split-transform latency forms (A/B libraries, tools/ab/), the removed split
    and pair forms and the gate-wave-DMA / per-pair-barrier variants are
    refused, and the context keeps its defaults."""
    assert tfhe_amd.build_kind() == tfhe_amd.BUILD_PRODUCT
    c, _ = ctx_for(oracle, "80")
    with pytest.raises(tfhe_amd.TfheError):
        c.set_option(name, value)
    assert c.get_option(name) == tfhe_amd.OPTION_DEFAULTS[name]


@pytest.mark.parametrize("form,pname", [("whole", "80"), ("wide", "80"), ("octo", "uint4")])
def test_bootstrap_without_key_switch(oracle, form, pname):
    """VanillaBootstrap.bootstrapWithoutKeySwitch (vanilla.zig:58-69) and the
    strategy mirror: blind rotation + the hybrid sampleExtractIndex2."""
    c, k = ctx_for(oracle, pname)
    cts = u32rand(rng(26), 3, k.p.n + 1)
    want = np.array([oracle.bootstrap_without_key_switch(k.p, t, k.ck) for t in cts])
    want1 = oracle.bootstrap(k.p, cts[1], k.ck)
    with c.options(br_form=form):
        assert np.array_equal(c.bootstrap_without_key_switch_batch(cts), want)
        bs = tfhe_amd.HipBootstrap(c)
        assert np.array_equal(bs.bootstrap_without_key_switch(cts[0]), want[0])
        assert np.array_equal(bs.bootstrap(cts[1]), want1)
        assert bs.name() == "mi355x"


def test_gate_golden_vectors(oracle):
    """All ten reference gates, committed inputs/outputs (80-bit, seeds 42/43)."""
    c, _ = ctx_for(oracle, "80")
    g = np.load(os.path.join(GOLDEN, "oracle_vectors.npz"))
    assert np.array_equal(c.gate_batch(g["gate_ops"], g["gate_a"], g["gate_b"]), g["gate_out"])


def test_gates_128_all_ops_bit_exact(oracle):
    c, k = ctx_for(oracle, "128")
    p = k.p
    g = rng(7)
    ops = np.repeat(np.arange(10, dtype=np.uint8), 2)
    A = np.array([oracle.tlwe_encrypt_bool(p.n, int(b), p.alpha_lv0, k.k0, 100 + i)
                  for i, b in enumerate(g.integers(0, 2, ops.size))])
    B = np.array([oracle.tlwe_encrypt_bool(p.n, int(b), p.alpha_lv0, k.k0, 200 + i)
                  for i, b in enumerate(g.integers(0, 2, ops.size))])
    want = oracle.gate_batch(p, ops, A, B, k.ck, threads=8)
    got = c.gate_batch(ops, A, B)
    assert np.array_equal(got, want)
    # and the same through the Gates mirror
    gates = tfhe_amd.Gates(c)
    assert np.array_equal(gates.nand_gate(A[:1], B[:1]), oracle.gate_batch(p, ops[:1] * 0, A[:1], B[:1], k.ck)[0])


def test_bootstrap_edge_rotations(oracle):
    """a~ in {0, 2N} (skipped CMUX), b near the 2^32 wrap, empty and single batches."""
    c, k = ctx_for(oracle, "80")
    p = k.p
    cts = u32rand(rng(8), 4, p.n + 1)
    cts[0, : p.n // 2] = 0                      # a~ = 0
    cts[1, : p.n // 2] = 0xFFFFFFFF             # a~ = 2048 (64-bit add, no wrap)
    cts[1, p.n] = 0xFFFFFFFF                    # b~ = 0
    cts[2, p.n] = (1 << 20) - 1                 # b~ = 2N exactly
    cts[3, ::2] = 0xFFF00000                    # a~ = 2048 boundary (0xFFF00000 + 2^20 = 2^32)
    want = np.array([oracle.bootstrap(p, t, k.ck) for t in cts])
    assert np.array_equal(c.bootstrap_batch(cts), want)
    assert c.bootstrap_batch(np.zeros((0, p.n + 1), np.uint32)).shape == (0, p.n + 1)
    assert np.array_equal(c.bootstrap_batch(cts[:1]), want[:1])


def test_nand_batch_1024_128bit(oracle):
    """BASELINE config 2 shape: 1024 NAND, 128-bit; truth table for all, bits for a sample."""
    c, k = ctx_for(oracle, "128")
    p = k.p
    sk = tfhe_amd.SecretKey(c.params, k.k0, k.k1)
    g = rng(9)
    a_bits = g.integers(0, 2, 1024).astype(np.uint8)
    b_bits = g.integers(0, 2, 1024).astype(np.uint8)
    A = sk.encrypt_bool(a_bits, seed0=10_000)
    B = sk.encrypt_bool(b_bits, seed0=20_000)
    out = c.gate_batch(np.zeros(1024, np.uint8), A, B)
    assert np.array_equal(sk.decrypt_bool(out), ~(a_bits.astype(bool) & b_bits.astype(bool)))
    idx = g.choice(1024, 6, replace=False)
    want = oracle.gate_batch(p, np.zeros(idx.size, np.uint8), A[idx], B[idx], k.ck, threads=6)
    assert np.array_equal(out[idx], want)
    # determinism
    assert np.array_equal(c.gate_batch(np.zeros(64, np.uint8), A[:64], B[:64]), out[:64])


def test_gate_batch_rounds_and_tail(oracle):
    """2,348 mixed gates (80-bit): two whole-form rounds of 1,024 plus a 300-gate tail
    that launch_blind_rotate hands to the latency form, on the plain (non-gathered)
    input path whose tail pointers it offsets.  Truth table for all, oracle bits at
    the round and tail boundaries."""
    c, k = ctx_for(oracle, "80")
    sk = tfhe_amd.SecretKey(c.params, k.k0, k.k1)
    g = rng(31)
    n = 2 * 1024 + 300
    ops = g.integers(0, 10, n).astype(np.uint8)
    a_bits = g.integers(0, 2, n).astype(np.uint8)
    b_bits = g.integers(0, 2, n).astype(np.uint8)
    A = sk.encrypt_bool(a_bits, seed0=31_000)
    B = sk.encrypt_bool(b_bits, seed0=41_000)
    out = c.gate_batch(ops, A, B)
    ab, bb = a_bits.astype(bool), b_bits.astype(bool)
    want_bits = np.zeros(n, bool)
    for o in range(10):  # TRUTH below works on numpy bool arrays
        m = ops == o
        want_bits[m] = TRUTH[o](ab[m], bb[m])
    assert np.array_equal(sk.decrypt_bool(out), want_bits)
    idx = np.array([0, 1023, 1024, 2047, 2048, n - 1])
    want = oracle.gate_batch(k.p, ops[idx], A[idx], B[idx], k.ck, threads=6)
    assert np.array_equal(out[idx], want)
    # the host-buffer pipeline (TFHE_OPT_HOST_PIPELINE: 256-item chunks on 4 streams
    # through pinned staging) gives the same words
    with c.options(host_pipeline=1):
        assert np.array_equal(c.gate_batch(ops, A, B), out)
        assert "k_key_switch_gemm<" in c.last_kernels()  # every chunk: the same key-switch form


TRUTH = {0: lambda a, b: ~(a & b), 1: lambda a, b: a | b, 2: lambda a, b: a & b, 3: lambda a, b: a ^ b,
         4: lambda a, b: a ^ b,  # reference xnorGate computes a - 2b + 1/4: decrypts as XOR (test_oracle.py)
         5: lambda a, b: ~(a | b), 6: lambda a, b: ~a & b, 7: lambda a, b: a & ~b, 8: lambda a, b: ~a | b,
         9: lambda a, b: a | ~b}


def test_all_ops_ragged_batch_1027_128bit(oracle):
    """Full-size mixed batch, 1027 gates (ragged last workgroup, whole form): every
    gate's truth table, a bit-exact sample vs the oracle, and the first 300 again
    through the latency form (B <= 512) — the two forms agree bit for bit."""
    c, k = ctx_for(oracle, "128")
    p = k.p
    sk = tfhe_amd.SecretKey(c.params, k.k0, k.k1)
    g = rng(19)
    B = 1027
    ops = g.integers(0, 10, B).astype(np.uint8)
    a_bits = g.integers(0, 2, B).astype(bool)
    b_bits = g.integers(0, 2, B).astype(bool)
    A = sk.encrypt_bool(a_bits.astype(np.uint8), seed0=30_000)
    Bc = sk.encrypt_bool(b_bits.astype(np.uint8), seed0=40_000)
    out = c.gate_batch(ops, A, Bc)
    want_bits = np.array([TRUTH[int(o)](x, y) for o, x, y in zip(ops, a_bits, b_bits)], bool)
    assert np.array_equal(sk.decrypt_bool(out), want_bits)
    idx = np.concatenate([g.choice(B - 3, 5, replace=False), [B - 3, B - 2, B - 1]])
    want = oracle.gate_batch(p, ops[idx], A[idx], Bc[idx], k.ck, threads=8)
    assert np.array_equal(out[idx], want)
    assert np.array_equal(c.gate_batch(ops[:300], A[:300], Bc[:300]), out[:300])


def test_lut_pbs_uint4(oracle):
    """BASELINE config 5 semantics: f(x) = (x+1) mod 16 over all 16 messages."""
    c, k = ctx_for(oracle, "uint4")
    p = k.p
    f = lambda x: (x + 1) % 16
    tv = tfhe_amd.lut_generate(c.params, 16, f)
    sk = tfhe_amd.SecretKey(c.params, k.k0, k.k1)
    msgs = np.tile(np.arange(16, dtype=np.uint32), 2)
    cts = sk.encrypt_lwe_message(msgs, 16, seed0=77)
    out = c.bootstrap_lut_batch(cts, tv)
    want = np.array([oracle.gate_batch(p, np.array([255], np.uint8), t[None], t[None], k.ck, testvec=tv)[0]
                     for t in cts[:4]])
    assert np.array_equal(out[:4], want)
    assert np.array_equal(sk.decrypt_lwe_message(out, 16), (msgs + 1) % 16)


@pytest.mark.parametrize("pname,B", [("uint4", 4096), ("uint4", 33), ("128", 1500)])
def test_lut_device_resident(oracle, pname, B):
    """tfhe_gpu_bootstrap_lut_batch_dev (device buffers, test vector on the device,
    async on the context stream): the host-buffer call's words (config 5's full
    4,096 items on the octo form, a ragged batch, and a 128-bit LUT), the oracle
    on a sample."""
    import torch
    c, k = ctx_for(oracle, pname)
    m = 16 if pname == "uint4" else 4
    tv = tfhe_amd.lut_generate(c.params, m, lambda x: (3 * x + 1) % m)
    sk = tfhe_amd.SecretKey(c.params, k.k0, k.k1)
    msgs = (np.arange(B) % m).astype(np.uint32)
    cts = sk.encrypt_lwe_message(msgs, m, seed0=4040 + B)
    want = c.bootstrap_lut_batch(cts, tv)
    t_in = torch.from_numpy(np.ascontiguousarray(cts).view(np.int32)).to("cuda:0")
    t_tv = torch.from_numpy(np.ascontiguousarray(tv, np.uint32).view(np.int32)).to("cuda:0")
    t_out = torch.zeros_like(t_in)
    try:
        c.set_stream(torch.cuda.current_stream().cuda_stream)
        c.bootstrap_lut_batch_dev(t_in.data_ptr(), t_tv.data_ptr(), t_out.data_ptr(), B)
        c.sync()
    finally:
        c.set_stream(None)
    got = t_out.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want)
    one = oracle.gate_batch(k.p, np.array([255], np.uint8), cts[B - 1][None], cts[B - 1][None], k.ck, testvec=tv)[0]
    assert np.array_equal(got[B - 1], one)


def test_lut_uint4_on_a_key_with_the_reference_noise_constants(oracle):
    """the reference draws every KSK with KSK_ALPHA = 2e-5 and
    every BSK with BSK_ALPHA = 2e-8, the 128-bit constants, for all sets
    (params.zig:419-422, key.zig:166,202); this build's UINT4 keys use alpha_ksk =
    alpha_lv0 and alpha_bsk = 0.  A UINT4 cloud key generated by
    the oracle with the REFERENCE's constants loads and runs: the LUT bootstrap is
    bit-exact vs the oracle on it.  Decryption is not asserted: with Bg = 2^22 the
    L = 1 gadget amplifies that BSK noise (the fraction decrypting correctly is
    printed for the record)."""
    from oracle import OracleParams, PARAM_SETS
    p = OracleParams(**dict(PARAM_SETS["uint4"], alpha_ksk=2.0e-5, alpha_bsk=2.0e-8))
    k0, k1 = oracle.secret_key(p, 42)
    ck = oracle.cloud_key(p, 43, k0, k1)
    c = tfhe_amd.Context("uint4", 0)
    try:
        c.load_cloud_key(ck.offset, ck.testvec, ck.bk, ck.ksk)
        m = 16
        tv = tfhe_amd.lut_generate(c.params, m, lambda x: (x + 1) % m)
        sk = tfhe_amd.SecretKey(c.params, k0, k1)
        msgs = np.tile(np.arange(m, dtype=np.uint32), 4)
        cts = sk.encrypt_lwe_message(msgs, m, seed0=7070)
        out = c.bootstrap_lut_batch(cts, tv)
        want = np.array([oracle.gate_batch(p, np.array([255], np.uint8), t[None], t[None], ck, testvec=tv)[0]
                         for t in cts[:8]])
        assert np.array_equal(out[:8], want)
        ok = float(np.mean(sk.decrypt_lwe_message(out, m) == (msgs + 1) % m))
        print(f"reference-constant UINT4 key: {ok:.2%} of {len(msgs)} LUT outputs decrypt to f(m)")
    finally:
        c.close()


def test_lut_config5_full_4096_uint4(oracle):
    """BASELINE config 5 at its full size on one GPU: 4,096 UINT4 programmable
    bootstraps of f(x) = x^2 + 3 mod 16 (bench.py --workload lut).  Every item
    decrypts to f(m); samples in the first and the last blocks of the ring-form
    key switch (256 items each) and across the blind rotation's 1,024-item rounds
    bit-exact vs the oracle."""
    c, k = ctx_for(oracle, "uint4")
    m = 16
    tv = tfhe_amd.lut_generate(c.params, m, lambda x: (x * x + 3) % m)
    sk = tfhe_amd.SecretKey(c.params, k.k0, k.k1)
    msgs = rng(4096).integers(0, m, 4096).astype(np.uint32)
    cts = sk.encrypt_lwe_message(msgs, m, seed0=40960)
    out = c.bootstrap_lut_batch(cts, tv)
    assert "k_key_switch_gemm<3,5>" in c.last_kernels()
    assert np.array_equal(sk.decrypt_lwe_message(out, m), (msgs * msgs + 3) % m)
    idx = [0, 1, 255, 1023, 1024, 2047, 3071, 3840, 4000, 4095]
    want = oracle.gate_batch(k.p, np.full(len(idx), 255, np.uint8), cts[idx], cts[idx], k.ck, testvec=tv,
                             threads=len(idx))
    assert np.array_equal(out[idx], want)


@pytest.mark.parametrize("extra,form", [(0, "octo"), (300, "whole"), (1500, "octo"), (-1848, "wide")])
def test_lut_uint4_dispatch_plans(oracle, extra, form):
    """L = 1 dispatch (blind_rotate_plan): 8 x #CUs items and 8 x #CUs + 1,500
    run the octo form (1.9 whole-form rounds per octo round), 8 x #CUs + 300 the
    whole form in one launch (3 rounds beat 2 octo rounds), 200 items the latency
    form.  Bit-identical to the forced whole form, and to the oracle at the
    round boundaries."""
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    c, k = ctx_for(oracle, "uint4")
    B = 8 * cus + extra * cus // 256
    tv = tfhe_amd.lut_generate(c.params, 16, lambda x: (3 * x + 1) % 16)
    sk = tfhe_amd.SecretKey(c.params, k.k0, k.k1)
    msgs = rng(B).integers(0, 16, B).astype(np.uint32)
    cts = sk.encrypt_lwe_message(msgs, 16, seed0=B)
    out = c.bootstrap_lut_batch(cts, tv)
    prefix = {"octo": "k_blind_rotate_octo<1,", "whole": "k_blind_rotate<1,", "wide": "k_blind_rotate_wide<1,"}[form]
    assert c.last_kernels().startswith(prefix), c.last_kernels()
    with c.options(br_form="whole"):
        assert np.array_equal(c.bootstrap_lut_batch(cts, tv), out)
    assert np.array_equal(sk.decrypt_lwe_message(out, 16), (3 * msgs + 1) % 16)
    idx = sorted({0, min(4 * cus, B - 1), min(8 * cus - 1, B - 1), min(8 * cus, B - 1), B - 1})
    want = oracle.gate_batch(k.p, np.full(len(idx), 255, np.uint8), cts[idx], cts[idx], k.ck, testvec=tv,
                             threads=len(idx))
    assert np.array_equal(out[idx], want)


def test_lut_uint4_gemm_key_switch(oracle):
    """UINT4 key switch as the one-hot GEMM (basebit 5: one MFMA K-step per
    coefficient and level; the default) on 1,300 LUT bootstraps: bit-identical
    to the ring form (TFHE_OPT_KS_FORM = 0) and decrypting to f(m)."""
    c, k = ctx_for(oracle, "uint4")
    tv = tfhe_amd.lut_generate(c.params, 16, lambda x: (5 * x + 2) % 16)
    sk = tfhe_amd.SecretKey(c.params, k.k0, k.k1)
    msgs = rng(1300).integers(0, 16, 1300).astype(np.uint32)
    cts = sk.encrypt_lwe_message(msgs, 16, seed0=13000)
    with c.options(ks_form=0):
        ring = c.bootstrap_lut_batch(cts, tv)
        assert "k_key_switch_ring<" in c.last_kernels()
    got = c.bootstrap_lut_batch(cts, tv)
    assert "k_key_switch_gemm<3,5>" in c.last_kernels()
    assert np.array_equal(got, ring)
    assert np.array_equal(sk.decrypt_lwe_message(got, 16), (5 * msgs + 2) % 16)


def test_lut_uint4_golden_fixture(oracle):
    """The committed config-5 fixture (tests/golden/lut_uint4.npz) through
    tfhe_gpu_bootstrap_lut_batch with the oracle's seeded UINT4 key: bit-identical."""
    g = np.load(os.path.join(GOLDEN, "lut_uint4.npz"))
    c, _ = ctx_for(oracle, "uint4")
    tv = tfhe_amd.lut_generate(c.params, 16, lambda x: (x + 1) % 16)
    assert np.array_equal(tv, g["testvec"])
    assert np.array_equal(c.bootstrap_lut_batch(g["cts"], tv), g["out"])


def test_keygen_matches_oracle(oracle):
    """tfhe_gpu_keygen (host RNG + device FFTs) == oracle CloudKey.new, bit for bit."""
    p = get_keys(oracle, "80").p
    c = tfhe_amd.Context("80", 0)
    sk, (bk, ksk) = c.keygen(42, 43, want_host_copy=True)
    k0, k1 = oracle.secret_key(p, 42)
    assert np.array_equal(sk.key_lv0, k0) and np.array_equal(sk.key_lv1, k1)
    ck = oracle.cloud_key(p, 43, k0, k1)
    assert np.array_equal(ksk, ck.ksk)
    assert np.array_equal(bk, ck.bk)
    c.close()


@pytest.mark.slow
def test_add_two_numbers_gpu(oracle):
    """examples/add_two_numbers.zig: 16-bit ripple-carry, 402 + 304 = 706."""
    c, k = ctx_for(oracle, "128")
    sk = tfhe_amd.SecretKey(c.params, k.k0, k.k1)
    gates = tfhe_amd.Gates(c)
    A = sk.encrypt_bool([(402 >> i) & 1 for i in range(16)], seed0=1)
    Bc = sk.encrypt_bool([(304 >> i) & 1 for i in range(16)], seed0=101)
    carry = sk.encrypt_bool([0], seed0=999)[0]
    bits = []
    for i in range(16):
        x = gates.xor_gate(A[i], Bc[i])
        ab = gates.and_gate(A[i], Bc[i])
        xc = gates.and_gate(x, carry)
        bits.append(gates.xor_gate(x, carry))
        carry = gates.or_gate(ab, xc)
    val = sum(int(b) << i for i, b in enumerate(sk.decrypt_bool(np.array(bits))))
    assert val == 706
    # word for word: the same gate sequence through the oracle (80 bootstraps)
    p = k.p
    one = lambda op, x, y: oracle.gate_batch(p, np.array([op], np.uint8), x[None], y[None], k.ck)[0]
    wc = sk.encrypt_bool([0], seed0=999)[0]
    want = []
    for i in range(16):
        x = one(tfhe_amd.XOR, A[i], Bc[i])
        ab = one(tfhe_amd.AND, A[i], Bc[i])
        xc = one(tfhe_amd.AND, x, wc)
        want.append(one(tfhe_amd.XOR, x, wc))
        wc = one(tfhe_amd.OR, ab, xc)
    assert np.array_equal(np.array(bits), np.array(want)) and np.array_equal(carry, wc)


def test_device_resident_api_with_torch(oracle):
    """tfhe_gpu_gate_batch_dev on torch-allocated HBM buffers and torch's stream."""
    torch = pytest.importorskip("torch")
    c, k = ctx_for(oracle, "80")
    p = k.p
    g = rng(11)
    ops = np.arange(10, dtype=np.uint8)
    A = u32rand(g, 10, p.n + 1)
    B = u32rand(g, 10, p.n + 1)
    want = c.gate_batch(ops, A, B)
    dev = torch.device("cuda", 0)
    t_ops = torch.from_numpy(ops).to(dev)
    t_a = torch.from_numpy(A.view(np.int32)).to(dev)
    t_b = torch.from_numpy(B.view(np.int32)).to(dev)
    t_o = torch.zeros_like(t_a)
    c.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    try:
        c.gate_batch_dev(t_ops.data_ptr(), t_a.data_ptr(), t_b.data_ptr(), t_o.data_ptr(), 10)
        torch.cuda.synchronize(dev)
    finally:
        c.set_stream(None)
    assert np.array_equal(t_o.cpu().numpy().view(np.uint32), want)


def test_dev_entry_ordered_on_torch_default_stream(oracle):
    """ABI 7: torch's default stream has handle 0, the device's null stream, and
    tfhe_gpu_set_stream(ctx, NULL) now means that stream (up to ABI 6 it meant the
    context's own non-blocking stream, so a torch op right after a _dev call could
    read the outputs before they were written: tools/soak_fused.py found it).  A
    4,096-gate batch (tens of ms) followed by a torch copy on the same stream, with
    no device-wide synchronisation in between: the copy sees every output word."""
    torch = pytest.importorskip("torch")
    c, k = ctx_for(oracle, "128")
    g = rng(12)
    B = 4096
    ops = (np.arange(B) % 10).astype(np.uint8)
    A, Bc = u32rand(g, B, k.p.n + 1), u32rand(g, B, k.p.n + 1)
    want = c.gate_batch(ops, A, Bc)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    assert stream.cuda_stream == 0  # the default stream: the case that used to race
    t_ops = torch.from_numpy(ops).to(dev)
    t_a = torch.from_numpy(A.view(np.int32)).to(dev)
    t_b = torch.from_numpy(Bc.view(np.int32)).to(dev)
    t_o = torch.zeros_like(t_a)
    torch.cuda.synchronize(dev)
    c.set_stream(stream.cuda_stream)
    try:
        c.gate_batch_dev(t_ops.data_ptr(), t_a.data_ptr(), t_b.data_ptr(), t_o.data_ptr(), B)
        snap = t_o.clone()  # queued on torch's stream right behind the library's launches
        got = snap.cpu().numpy().view(np.uint32)
    finally:
        c.set_stream(None)
    c.sync()
    assert np.array_equal(got, want)


@pytest.mark.parametrize("gw", [0, 1, 2, 4, 8])
def test_lut_uint4_key_switch_item_groups(oracle, gw):
    """UINT4 key switch under TFHE_OPT_KS_FORM = 0: the ring form (gw 0: 4 item
    groups sharing one 4-deep ring per block) and the lane form with 1, 2, 4 or 8
    item groups per block (TFHE_OPT_KS_ITEM_GROUPS): 300 LUT bootstraps, samples
    past the first group bit-exact vs the oracle."""
    c, k = ctx_for(oracle, "uint4")
    tv = tfhe_amd.lut_generate(c.params, 16, lambda x: (3 * x + 5) % 16)
    sk = tfhe_amd.SecretKey(c.params, k.k0, k.k1)
    msgs = rng(23).integers(0, 16, 300).astype(np.uint32)
    cts = sk.encrypt_lwe_message(msgs, 16, seed0=4242)
    with c.options(ks_item_groups=gw, ks_form=0):
        out = c.bootstrap_lut_batch(cts, tv)
        assert ("k_key_switch_ring<" in c.last_kernels()) == (gw == 0)
    assert np.array_equal(sk.decrypt_lwe_message(out, 16), (3 * msgs + 5) % 16)
    for i in (0, 63, 64, 200, 299):
        want = oracle.gate_batch(k.p, np.array([255], np.uint8), cts[i][None], cts[i][None], k.ck, testvec=tv)[0]
        assert np.array_equal(out[i], want)


def test_gates128_golden_fixture():
    """BASELINE config 2's parameter set against committed bits, no oracle on the box:
    tfhe_gpu_keygen(42, 43) (bit-equal to the oracle's keygen, test_keygen_matches_oracle)
    then one gate of each op plus NANDs vs tests/golden/gates128.npz."""
    import hashlib
    g = np.load(os.path.join(GOLDEN, "gates128.npz"))
    c = tfhe_amd.Context("128", 0)
    c.keygen(42, 43)
    out = c.gate_batch(g["ops"], g["a"], g["b"])
    assert hashlib.sha256(np.ascontiguousarray(out, np.uint32).tobytes()).hexdigest() == str(g["out_sha256"])
    assert np.array_equal(out, g["out"])
    c.close()


# ---- twiddle-table source (TFHE_OPT_TWIDDLES) ------------------
def test_twiddle_source_uint4_matches_oracle_under_each_table(oracle):
    """Where the libm choice matters (UINT4: Bg = 2^22, inexact external products),
    the engine matches the oracle built with the same table, for both candidate
    libms of a Zig build (glibc / fdlibm-musl), and the two tables give different
    bits.  Keys from the oracle's keygen under each table (seeds 42/43)."""
    p = get_keys(oracle, "uint4").p
    tv = tfhe_amd.lut_generate(tfhe_amd.make_params("uint4"), 16, lambda x: (x + 1) % 16)
    k0, k1 = oracle.secret_key(p, 42)
    sk = tfhe_amd.SecretKey(tfhe_amd.make_params("uint4"), k0, k1)
    msgs = np.arange(6, dtype=np.uint32) * 3 % 16
    cts = sk.encrypt_lwe_message(msgs, 16, seed0=515)
    outs = {}
    for src in (0, 1):
        try:
            oracle.set_trig_source(src)
            ck = oracle.cloud_key(p, 43, k0, k1)
            want = oracle.gate_batch(p, np.full(msgs.size, 255, np.uint8), cts, cts, ck, testvec=tv, threads=6)
        finally:
            oracle.set_trig_source(0)
        c = tfhe_amd.Context("uint4", 0)
        c.set_option("twiddles", src)
        assert c.get_option("twiddles") == src
        c.load_cloud_key(ck.offset, ck.testvec, ck.bk, ck.ksk)
        outs[src] = c.bootstrap_lut_batch(cts, tv)
        c.close()
        assert np.array_equal(outs[src], want)
        assert np.array_equal(sk.decrypt_lwe_message(outs[src], 16), (msgs + 1) % 16)
    assert (outs[0] != outs[1]).any()


def test_gates128_fdlibm_golden_fixture():
    """The 128-bit gate fixture regenerated under the fdlibm twiddles
    (tests/golden/gates128_fdlibm.npz) from seeds on the GPU with TFHE_OPT_TWIDDLES =
    fdlibm (keygen transforms the key with those tables)."""
    import hashlib
    g = np.load(os.path.join(GOLDEN, "gates128_fdlibm.npz"))
    c = tfhe_amd.Context("128", 0)
    c.set_option("twiddles", tfhe_amd.TWIDDLES_FDLIBM)
    c.keygen(42, 43)
    out = c.gate_batch(g["ops"], g["a"], g["b"])
    assert hashlib.sha256(np.ascontiguousarray(out, np.uint32).tobytes()).hexdigest() == str(g["out_sha256"])
    c.close()


def test_fused_and_reference_arithmetic_agree_1024(oracle):
    """The headline shape (1,024 NAND, 128-bit, whole form): the fused-multiply-add
    kernel and the reference-expression-tree kernel give identical words for every
    gate (each CMUX rounds the same exact integer polynomial), and a sample is
    bit-exact vs the oracle in both of its arithmetic modes."""
    c, k = ctx_for(oracle, "128")
    sk = tfhe_amd.SecretKey(c.params, k.k0, k.k1)
    g = rng(93)
    a_bits, b_bits = g.integers(0, 2, 1024).astype(np.uint8), g.integers(0, 2, 1024).astype(np.uint8)
    A, B = sk.encrypt_bool(a_bits, seed0=93_000), sk.encrypt_bool(b_bits, seed0=94_000)
    ops = np.zeros(1024, np.uint8)
    fused = c.gate_batch(ops, A, B)
    assert "fused" in c.last_kernels()
    with c.options(arith=tfhe_amd.ARITH_REFERENCE):
        ref = c.gate_batch(ops, A, B)
        assert "fused" not in c.last_kernels()
    assert np.array_equal(fused, ref)
    idx = np.array([0, 511, 1023])
    for mode in (0, 1):
        try:
            oracle.set_fused(mode)
            want = oracle.gate_batch(k.p, ops[idx], A[idx], B[idx], k.ck, threads=3)
        finally:
            oracle.set_fused(0)
        assert np.array_equal(fused[idx], want)


def test_options_validation_and_report(oracle):
    """tfhe_gpu_set_option rejects unknown keys / values; the last-kernel report
    names the default forms (the latency form below 512 items, the one-hot GEMM key
    switch; the lane key switch under ks_form = 0)."""
    c, k = ctx_for(oracle, "128")
    with pytest.raises(tfhe_amd.TfheError):
        c.set_option("br_form", 9)
    assert c.lib.tfhe_gpu_set_option(c.h, 99, 0) == -1
    for removed in (2, 4, 6, 7):  # split, pair (removed in round 4); duo, wide2 (A/B libraries only)
        assert c.lib.tfhe_gpu_set_option(c.h, 1, removed) == -1
    assert c.get_option("br_form") == 0
    g = rng(91)
    cts = u32rand(g, 3, k.p.n + 1)
    c.bootstrap_batch(cts)
    gemm = "k_key_switch_gemm<9,2> + k_ks_gemm_reduce"
    assert c.last_kernels() == "k_blind_rotate_wide<3,true,true> (latency form, fused) + " + gemm
    with c.options(arith=tfhe_amd.ARITH_REFERENCE):
        c.bootstrap_batch(cts)
        assert c.last_kernels() == "k_blind_rotate_wide<3,true,false> (latency form) + " + gemm
    with c.options(br_form="whole"):
        c.bootstrap_batch(cts)
        assert c.last_kernels() == "k_blind_rotate_assist<true> (whole form, loader waves own polynomial b, fused) + " + gemm
    with c.options(ks_form=0):
        c.bootstrap_batch(cts)
        assert c.last_kernels().endswith("k_key_switch_lanes<9,2,32,4,1>")


def test_whole_form_full_and_ragged_headline_batches(oracle):
    """The whole form (slot-counter protocol) on a full and a ragged headline-size
    batch (256 / 257 workgroups, every CU): identical to the reference-tree
    kernel, the NAND truth table decrypts right, and a sample matches the oracle."""
    c, k = ctx_for(oracle, "128")
    sk = tfhe_amd.SecretKey(c.params, k.k0, k.k1)
    g = rng(95)
    for Bn in (1024, 1027):
        a_bits, b_bits = g.integers(0, 2, Bn).astype(np.uint8), g.integers(0, 2, Bn).astype(np.uint8)
        A, B = sk.encrypt_bool(a_bits, seed0=95_000), sk.encrypt_bool(b_bits, seed0=96_000)
        ops = np.zeros(Bn, np.uint8)
        with c.options(br_form="whole"):
            fused = c.gate_batch(ops, A, B)
            assert c.last_kernels().startswith("k_blind_rotate_assist<true>")
        with c.options(br_form="whole", arith=tfhe_amd.ARITH_REFERENCE):
            ref = c.gate_batch(ops, A, B)
            assert c.last_kernels().startswith("k_blind_rotate<3,true,false>")
        assert np.array_equal(fused, ref)
        assert np.array_equal(sk.decrypt_bool(fused), ~(a_bits.astype(bool) & b_bits.astype(bool)))
        idx = np.array([0, Bn - 1])
        assert np.array_equal(fused[idx], oracle.gate_batch(k.p, ops[idx], A[idx], B[idx], k.ck, threads=2))


@pytest.mark.parametrize("form", ["auto", "whole", "wide"])
def test_margin_guard_recomputes_near_ties(oracle, form):
    """under a crafted key (conftest.crafted_near_tie_case) the
    unguarded fused arithmetic parts from the reference (the oracle's fused mode
    differs from its reference mode).  Every fused form returns the REFERENCE's
    words: the items that rounded a value 1/4 or more off its integer were flagged by
    the margin guard and redone by the reference-tree recompute, which
    tfhe_gpu_near_tie_items counts.  (Honest batches never trigger it:
    test_margin_guard_quiet_on_honest_batches.)"""
    p = get_keys(oracle, "128").p
    tv, bk, ct = crafted_near_tie_case(oracle, p)
    ksk = np.zeros((p.N * p.iks_t * (1 << p.basebit), p.n + 1), np.uint32)
    off = oracle.decomposition_offset(p)
    c = tfhe_amd.Context("128", 0)
    try:
        c.load_cloud_key(off, tv, bk, ksk)
        g = rng(4242)
        cts = np.concatenate([u32rand(g, 2, p.n + 1), ct[None], u32rand(g, 3, p.n + 1)])
        want, fused = [], []
        try:
            for mode, dst in ((0, want), (1, fused)):
                oracle.set_fused(mode)
                dst.extend(oracle.blind_rotate(p, x, tv, bk, off) for x in cts)
        finally:
            oracle.set_fused(0)
        want, fused = np.array(want), np.array(fused)
        parted = int((fused != want).any(axis=1).sum())
        assert not np.array_equal(fused[2], want[2]) and parted >= 1
        # the crafted key's BK concentrates its spectrum (2^41.3 > 2^39): the key
        # admission refuses it the fused arithmetic, so the default runs the reference's
        # trees and recomputes nothing; the guard itself is exercised by forcing fused
        assert c.get_option("fused_admitted") == 0
        before = c.near_tie_items()
        with c.options(br_form=form):
            assert np.array_equal(c.blind_rotate_batch(cts, tv), want)
            assert not c.last_kernels().split(" + ")[0].endswith("fused)")
        assert c.near_tie_items() == before
        with c.options(br_form=form, arith=tfhe_amd.ARITH_FUSED_FORCED):
            got = c.blind_rotate_batch(cts, tv)
        assert parted <= c.near_tie_items() - before <= len(cts)
        assert np.array_equal(got, want)
    finally:
        c.close()


def test_key_admission_of_the_fused_arithmetic(oracle):
    """DESIGN.md §6.1 key admission: keygen'd keys (BK spectra up to ~2^38.3, row
    RMS ~0.6 x 2^31) keep the fused arithmetic; a loaded key whose BK spectrum
    reaches past 2^39 (one row of constant 2^31 - 1), or one of whose rows has an
    RMS past 0.65 x 2^31 (+-(2^31 - 1), random signs: spectrum only 2^38.7), is
    refused it and runs the reference's trees, with the same words as the
    oracle; the refusal follows the key, not the context (a later admitted key
    gets the fused arithmetic back)."""
    c, k = ctx_for(oracle, "80")
    assert c.get_option("fused_admitted") == 1
    p = k.p
    bk = np.array(k.ck.bk, copy=True)
    row = np.full(1024, (1 << 31) - 1, np.int64)
    bk[3, 0, 0] = oracle.ifft((row % (1 << 32)).astype(np.uint32))  # BK[3], row 0, part a
    c2 = tfhe_amd.Context("80", 0)
    try:
        c2.load_cloud_key(k.ck.offset, k.ck.testvec, bk, k.ck.ksk)
        assert c2.get_option("fused_admitted") == 0
        cts = u32rand(rng(99), 3, p.n + 1)
        want = np.array([oracle.blind_rotate(p, t, k.ck.testvec, bk, k.ck.offset) for t in cts])
        assert np.array_equal(c2.blind_rotate_batch(cts), want)
        assert not c2.last_kernels().split(" + ")[0].endswith("fused)")
        c2.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk, k.ck.ksk)
        assert c2.get_option("fused_admitted") == 1
        c2.blind_rotate_batch(cts[:1])
        assert c2.last_kernels().split(" + ")[0].endswith("fused)")
        with pytest.raises(tfhe_amd.TfheError):
            c2.set_option("fused_admitted", 1)  # read-only
        assert 545_000 < c2.get_option("key_row_rms_ppm") < 620_000  # keygen'd rows: RMS ~0.6 x 2^31
        # round 5's row-energy rule: one row of +-(2^31 - 1) with random signs has a spectrum
        # of ~2^38.7 (the round-4 rule admitted it) but RMS 1.0 > 0.65: refused, reference trees
        g = rng(98)
        bk2 = np.array(k.ck.bk, copy=True)
        row = np.where(g.random(1024) < 0.5, (1 << 31) - 1, -((1 << 31) - 1)).astype(np.int64)
        bk2[7, 2, 1] = oracle.ifft((row % (1 << 32)).astype(np.uint32))
        assert np.abs(bk2[7, 2, 1]).max() < 2.0 ** 39
        c2.load_cloud_key(k.ck.offset, k.ck.testvec, bk2, k.ck.ksk)
        assert c2.get_option("fused_admitted") == 0
        assert 999_000 < c2.get_option("key_row_rms_ppm") <= 1_000_000
        want = np.array([oracle.blind_rotate(p, t, k.ck.testvec, bk2, k.ck.offset) for t in cts[:2]])
        assert np.array_equal(c2.blind_rotate_batch(cts[:2]), want)
        assert not c2.last_kernels().split(" + ")[0].endswith("fused)")
    finally:
        c2.close()


def test_margin_guard_quiet_on_honest_batches(oracle):
    """The seeded key and a 1,024-gate NAND batch of fresh encryptions (the
    headline shape): no value comes 1/4 off its integer (honest rotations stay
    within ~0.11 of an integer), nothing is recomputed."""
    c, k = ctx_for(oracle, "128")
    sk = tfhe_amd.SecretKey(c.params, k.k0, k.k1)
    g = rng(5151)
    a, b = g.integers(0, 2, 1024).astype(np.uint8), g.integers(0, 2, 1024).astype(np.uint8)
    A, B = sk.encrypt_bool(a, seed0=51_000), sk.encrypt_bool(b, seed0=52_000)
    before = c.near_tie_items()
    out = c.gate_batch(np.zeros(1024, np.uint8), A, B)
    assert c.near_tie_items() == before
    assert np.array_equal(sk.decrypt_bool(out), ~(a.astype(bool) & b.astype(bool)))


@pytest.mark.parametrize("pname", ["128", "80"])
def test_fused_equals_reference_soak_all_gates(oracle, pname):
    """Soak of the default arithmetic at scale: 65,536 gate bootstraps of every
    op (the ten gates in turn) over fresh encryptions, in 16 batches of 4,096
    (whole form, every CU), fused (the default) against the reference's
    expression trees on the same device: identical words for every gate, the
    truth tables decrypt, and the margin guard's recompute counter moves by at
    most a handful (honest rotations stay ~0.1 from an integer). Complements
    the oracle comparisons, which the CPU's speed caps at small batches."""
    c, k = ctx_for(oracle, pname)
    sk = tfhe_amd.SecretKey(c.params, k.k0, k.k1)
    g = rng(7070 + int(pname))
    B = 4096
    before = c.near_tie_items()
    for rep in range(16):
        a, b = g.integers(0, 2, B).astype(np.uint8), g.integers(0, 2, B).astype(np.uint8)
        ops = ((np.arange(B) + rep) % 10).astype(np.uint8)
        A, Bc = sk.encrypt_bool(a, seed0=700_000 + 2 * rep), sk.encrypt_bool(b, seed0=700_001 + 2 * rep)
        fused = c.gate_batch(ops, A, Bc)
        assert "fused" in c.last_kernels()
        with c.options(arith=tfhe_amd.ARITH_REFERENCE):
            ref = c.gate_batch(ops, A, Bc)
        assert np.array_equal(fused, ref), f"rep {rep}: {(fused != ref).any(axis=1).sum()} gates differ"
        if rep == 0:
            want = np.zeros(B, bool)
            for o in range(10):
                m = ops == o
                want[m] = TRUTH[o](a.astype(bool)[m], b.astype(bool)[m])
            assert np.array_equal(sk.decrypt_bool(fused), want)
    assert c.near_tie_items() - before <= 4


def test_worst_admitted_key_under_the_product_guard(oracle):
    """the worst admitted key tools/admission_search.py found
    (tests/golden/admission_worst.npz; gap 0.125 between the fused and the reference
    trees) on the GPU.  BK[0] holds its rows, the other steps zero; the test vector
    makes step 0's tmp the digits sign-aligned with those rows at the searched
    output (a~_0 = N: tmp = -2 acc; b~ = 2N), so step 0 is the largest external
    product the key admits and the rest add exact zeros.  The key is admitted (the
    default runs the fused arithmetic under the margin guard), and every word of the
    GPU's blind rotation equals the oracle's reference trees."""
    from test_oracle import _aligned_x
    f = np.load(os.path.join(GOLDEN, "admission_worst.npz"))
    p = get_keys(oracle, "128").p
    rows = f["rows"].astype(np.int64)
    x = _aligned_x(oracle, p, rows, int(f["k"]), int(f["part"])).astype(np.uint64)
    tv = (((1 << 32) - x) % (1 << 32) // 2).astype(np.uint32)  # -2 tv == x (mod 2^32): x is even
    assert np.array_equal((np.uint64(0) - 2 * tv.astype(np.uint64)) % (1 << 32), x)
    bk = np.zeros((p.n, 2 * p.L, 2, p.N))
    for i in range(2 * p.L):
        for part in range(2):
            bk[0, i, part] = oracle.ifft((rows[i][part] % (1 << 32)).astype(np.uint32))
    off = oracle.decomposition_offset(p)
    ksk = np.zeros((p.N * p.iks_t * (1 << p.basebit), p.n + 1), np.uint32)
    g = rng(9191)
    cts = g.integers(0, 1 << 32, (5, p.n + 1), dtype=np.uint64).astype(np.uint32)
    cts[:, 0], cts[:, p.n] = 1 << 31, 0  # a~_0 = N, b~ = 2N
    c = tfhe_amd.Context("128", 0)
    try:
        c.load_cloud_key(off, tv, bk, ksk)
        assert c.get_option("fused_admitted") == 1
        got = c.blind_rotate_batch(cts)
        want = np.array([oracle.blind_rotate(p, ct, tv, bk, off) for ct in cts])
        assert np.array_equal(got, want)
        print(f"worst admitted key: {c.near_tie_items()} item(s) recomputed by the guard")
    finally:
        c.close()
