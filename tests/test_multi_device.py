"""Multi-device contexts (tfhe_gpu_create_multi): batches
sharded over the devices in contiguous slices, the cloud key broadcast once
(RCCL ncclBroadcast for distinct devices, a device-to-device copy for a device
listed twice).  The GPU box has one MI355X, so the sharding is exercised with
device 0 listed twice (two shards, two streams, two host threads) and the RCCL
path with a one-device communicator; outputs must be bit-identical to a
single-device context and to the oracle."""
import numpy as np
import pytest

import tfhe_amd
from conftest import get_keys, rng

pytestmark = pytest.mark.gpu


def u32rand(g, *shape):
    return g.integers(0, 1 << 32, shape, dtype=np.uint64).astype(np.uint32)


def loaded(oracle, pname, devices=None):
    k = get_keys(oracle, pname)
    c = tfhe_amd.Context(pname, 0) if devices is None else tfhe_amd.Context.multi(pname, devices=devices)
    c.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk, k.ck.ksk)
    return c, k


def test_rccl_broadcast_one_device(oracle):
    """devices=[0]: ncclCommInitAll over one device + the in-place ncclBroadcast of the
    BK/KSK; gates bit-exact vs the oracle."""
    c, k = loaded(oracle, "80", devices=[0])
    assert c.num_devices == 1
    g = rng(71)
    ops = np.arange(10, dtype=np.uint8)
    A, B = u32rand(g, 10, k.p.n + 1), u32rand(g, 10, k.p.n + 1)
    assert np.array_equal(c.gate_batch(ops, A, B), oracle.gate_batch(k.p, ops, A, B, k.ck, threads=8))
    c.close()


@pytest.mark.parametrize("B", [1, 37, 1100])
def test_two_shards_gate_batch(oracle, B):
    """Two shards on one GPU: ragged slices (1 item leaves the second shard idle,
    1,100 = 550 + 550 runs the latency form on each), outputs in the caller's order."""
    single, k = loaded(oracle, "80")
    multi, _ = loaded(oracle, "80", devices=[0, 0])
    assert multi.num_devices == 2
    g = rng(72 + B)
    ops = g.integers(0, 10, B).astype(np.uint8)
    A, Bc = u32rand(g, B, k.p.n + 1), u32rand(g, B, k.p.n + 1)
    want = single.gate_batch(ops, A, Bc)
    assert np.array_equal(multi.gate_batch(ops, A, Bc), want)
    idx = np.unique([0, B // 2, B - 1])
    assert np.array_equal(want[idx], oracle.gate_batch(k.p, ops[idx], A[idx], Bc[idx], k.ck, threads=3))
    single.close()
    multi.close()


def test_two_shards_every_batch_entry(oracle):
    """bootstrap / bootstrap without key switch / blind rotation / key switch / LUT /
    re-encryption through a two-shard context: identical to one device."""
    single, k = loaded(oracle, "80")
    multi, _ = loaded(oracle, "80", devices=[0, 0])
    g = rng(73)
    cts = u32rand(g, 9, k.p.n + 1)
    assert np.array_equal(multi.bootstrap_batch(cts), single.bootstrap_batch(cts))
    assert np.array_equal(multi.bootstrap_without_key_switch_batch(cts), single.bootstrap_without_key_switch_batch(cts))
    assert np.array_equal(multi.blind_rotate_batch(cts[:5]), single.blind_rotate_batch(cts[:5]))
    lv1 = u32rand(g, 7, 1025)
    assert np.array_equal(multi.key_switch(lv1), single.key_switch(lv1))
    tv = tfhe_amd.lut_generate(single.params, 4, lambda x: (x + 1) % 4)
    assert np.array_equal(multi.bootstrap_lut_batch(cts, tv), single.bootstrap_lut_batch(cts, tv))
    alice, bob = tfhe_amd.secret_key_new(single.params, 11), tfhe_amd.secret_key_new(single.params, 12)
    key = tfhe_amd.ProxyReencryptionKey.new_symmetric(alice, bob, 1000)
    bits = g.integers(0, 2, 13).astype(np.uint8)
    enc = alice.encrypt_bool(bits, seed0=5)
    r1, r2 = tfhe_amd.HipReencryptor(single, key), tfhe_amd.HipReencryptor(multi, key)
    out = r2.reencrypt(enc)
    assert np.array_equal(out, r1.reencrypt(enc))
    assert np.array_equal(bob.decrypt_bool(out), bits.astype(bool))
    r1.close()
    r2.close()
    # options reach every shard
    with multi.options(br_form="whole"):
        assert np.array_equal(multi.bootstrap_batch(cts), single.bootstrap_batch(cts))
    single.close()
    multi.close()


def test_two_shards_keygen_broadcast(oracle):
    """Keygen on the first device, D2D broadcast to the second: every shard's
    result equals the oracle keygen's."""
    p = get_keys(oracle, "80").p
    multi = tfhe_amd.Context.multi("80", devices=[0, 0])
    sk, _ = multi.keygen(42, 43)
    k = get_keys(oracle, "80")
    g = rng(74)
    cts = u32rand(g, 4, p.n + 1)
    want = np.array([oracle.bootstrap(p, t, k.ck) for t in cts])
    assert np.array_equal(multi.bootstrap_batch(cts), want)  # items 2, 3 run on the second shard
    multi.close()


def test_two_shards_circuit_components(oracle):
    """circuit_eval over two shards: two independent 16-bit adders (one component
    each) land on different shards; 402 + 304 and 1234 + 4321, outputs identical to
    one device, depth 33."""
    single, k = loaded(oracle, "80")
    multi, _ = loaded(oracle, "80", devices=[0, 0])
    sk = tfhe_amd.SecretKey(single.params, k.k0, k.k1)
    c = tfhe_amd.Circuit()
    A = [[c.input() for _ in range(16)] for _ in range(2)]
    Bw = [[c.input() for _ in range(16)] for _ in range(2)]
    cin = [c.input() for _ in range(2)]
    for j in range(2):
        s, _ = c.ripple_add(A[j], Bw[j], cin[j])
        c.output(*s)
    xa, xb = [402, 1234], [304, 4321]
    bits = [(xa[j] >> i) & 1 for j in range(2) for i in range(16)] + \
           [(xb[j] >> i) & 1 for j in range(2) for i in range(16)] + [0, 0]
    inputs = sk.encrypt_bool(bits, seed0=303)
    got, depth = c.run(multi, inputs)
    want, d1 = c.run(single, inputs)
    assert depth == d1 == 33 and np.array_equal(got, want)
    dec = sk.decrypt_bool(got).reshape(2, 16)
    assert [sum(int(b) << i for i, b in enumerate(row)) for row in dec] == [706, 5555]
    with pytest.raises(RuntimeError):  # device-resident circuits take a single-device context
        c.run_dev(multi, 0, 0)
    single.close()
    multi.close()


def test_two_shards_connected_circuit_by_levels(oracle):
    """SURVEY §8e's level split (TFHE_OPT_CIRCUIT_SPLIT auto): one connected
    circuit — 2,200 XOR/AND gates over 64 shared inputs, then 2,200 ORs chaining
    neighbours, so every gate is in one component — is split level by level over
    two shards, each level's outputs all-gathered before the next.  Both shards
    run half of every level; the words equal one device's, a sample the oracle's."""
    single, k = loaded(oracle, "80")
    multi, _ = loaded(oracle, "80", devices=[0, 0])
    sk = tfhe_amd.SecretKey(single.params, k.k0, k.k1)
    g = rng(75)
    n = 2200
    c = tfhe_amd.Circuit()
    ins = [c.input() for _ in range(64)]
    pairs = g.integers(0, 64, (n, 2))
    l1 = [c.xor(ins[x], ins[y]) if i % 2 else c.and_(ins[x], ins[y]) for i, (x, y) in enumerate(pairs)]
    l2 = [c.or_(l1[i], l1[(i + 1) % n]) for i in range(n)]
    c.output(*l2[::7], *l1[:5])
    bits = g.integers(0, 2, 64).astype(np.uint8)
    inputs = sk.encrypt_bool(bits, seed0=7500)
    assert len(set(c.partition(2).tolist())) == 1  # one component
    before = multi.device_bootstraps()
    got, depth = c.run(multi, inputs)
    ran = multi.device_bootstraps() - before
    want, d1 = c.run(single, inputs)
    assert depth == d1 == 2 and np.array_equal(got, want)
    assert ran.sum() == 2 * n and abs(int(ran[0]) - int(ran[1])) <= 2
    b1 = np.array([(bits[x] ^ bits[y]) if i % 2 else (bits[x] & bits[y]) for i, (x, y) in enumerate(pairs)], bool)
    b2 = np.array([b1[i] | b1[(i + 1) % n] for i in range(n)], bool)
    assert np.array_equal(sk.decrypt_bool(got), np.concatenate([b2[::7], b1[:5]]))
    # forced component placement puts everything on one shard, same words
    with multi.options(circuit_split=1):
        before = multi.device_bootstraps()
        again, _ = c.run(multi, inputs)
        assert (multi.device_bootstraps() - before).min() == 0
    assert np.array_equal(again, want)
    single.close()
    multi.close()


def test_two_shards_adder_forced_level_split(oracle):
    """The level split on a 33-level adder (levels of 1-32 gates, NOTs none):
    forced (TFHE_OPT_CIRCUIT_SPLIT = 2), 402 + 304 = 706, words equal one device's."""
    single, k = loaded(oracle, "80")
    multi, _ = loaded(oracle, "80", devices=[0, 0])
    sk = tfhe_amd.SecretKey(single.params, k.k0, k.k1)
    c = tfhe_amd.Circuit()
    A, Bw = [c.input() for _ in range(16)], [c.input() for _ in range(16)]
    s, carry = c.ripple_add(A, Bw, c.input())
    m = c.mux(A[0], carry, Bw[3])  # a NOT inside a level, too
    c.output(*s, m)
    bits = [(402 >> i) & 1 for i in range(16)] + [(304 >> i) & 1 for i in range(16)] + [0]
    inputs = sk.encrypt_bool(bits, seed0=808)
    with multi.options(circuit_split=2):
        got, depth = c.run(multi, inputs)
    want, d1 = c.run(single, inputs)
    assert depth == d1 and np.array_equal(got, want)
    assert sum(int(b) << i for i, b in enumerate(sk.decrypt_bool(got[:16]))) == 706
    # the one host thread's per-level issue for both shards (what an
    # 8-device level split would pay per level, measured here on two shards)
    issue_us = multi.get_option("level_issue_us")
    print(f"level split issue: {issue_us} us for {depth + 1} levels on 2 shards")
    assert 0 < issue_us
    single.close()
    multi.close()


def test_create_multi_distinct_devices(oracle):
    """Distinct devices: on a one-GPU box, devices = [0, 1] fails cleanly (no
    crash, no context) with the reason in tfhe_gpu_last_error(NULL); with two or
    more GPUs the create enables peer access for every pair and the level split
    and the key broadcast give one device's words (never run on this pool: one
    GPU per box)."""
    import torch
    ndev = torch.cuda.device_count()
    if ndev < 2:
        with pytest.raises(tfhe_amd.TfheError) as e:
            tfhe_amd.Context.multi("80", devices=[0, 1])
        assert e.value.status == tfhe_amd.ERR_HIP and "does not exist" in str(e.value)
        c = tfhe_amd.Context.multi("80", devices=[0, 0])  # the library is still usable
        c.close()
        return
    single, k = loaded(oracle, "80")
    multi, _ = loaded(oracle, "80", devices=[0, 1])
    assert multi.key_fingerprint() == single.key_fingerprint()
    sk = tfhe_amd.SecretKey(single.params, k.k0, k.k1)
    c = tfhe_amd.Circuit()
    A, Bw = [c.input() for _ in range(16)], [c.input() for _ in range(16)]
    s, carry = c.ripple_add(A, Bw, c.input())
    c.output(*s, carry)
    bits = [(402 >> i) & 1 for i in range(16)] + [(304 >> i) & 1 for i in range(16)] + [0]
    inputs = sk.encrypt_bool(bits, seed0=808)
    with multi.options(circuit_split=2):
        got, _ = c.run(multi, inputs)
    assert np.array_equal(got, c.run(single, inputs)[0])
    single.close()
    multi.close()


def test_key_fingerprint(oracle):
    """tfhe_gpu_key_fingerprint: equal for the same key in two contexts (and on
    both shards of a two-shard context, which the in-library broadcast checks),
    different for a key with one BK word changed; no key -> TFHE_ERR_NO_KEY."""
    a, k = loaded(oracle, "80")
    b, _ = loaded(oracle, "80", devices=[0, 0])
    assert a.key_fingerprint() == b.key_fingerprint()
    bk = np.array(k.ck.bk, copy=True)
    bk[5, 1, 0, 3] += 1.0
    c = tfhe_amd.Context("80", 0)
    c.load_cloud_key(k.ck.offset, k.ck.testvec, bk, k.ck.ksk)
    fa, fc = a.key_fingerprint(), c.key_fingerprint()
    assert fa[0] != fc[0] and fa[1] == fc[1]
    empty = tfhe_amd.Context("80", 0)
    with pytest.raises(tfhe_amd.TfheError) as e:
        empty.key_fingerprint()
    assert e.value.status == tfhe_amd.ERR_NO_KEY
    for x in (a, b, c, empty):
        x.close()


def test_eight_shards_on_one_gpu(oracle):
    """the 8-way split an 8-GPU node runs, rehearsed with
    device 0 listed eight times (8 shards, 8 streams, 8 host threads, the key
    copied to each and fingerprint-checked).  A ragged gate batch (1,027 = 7 x
    129 + 124, the latency form on every shard), a config-4-style circuit placed
    by components and by the forced level split, and the UINT4 LUT batch: every
    word equal to one device's, a sample equal to the oracle's, and the work
    spread over all eight shards."""
    single, k = loaded(oracle, "80")
    multi, _ = loaded(oracle, "80", devices=[0] * 8)
    assert multi.num_devices == 8 and multi.key_fingerprint() == single.key_fingerprint()
    sk = tfhe_amd.SecretKey(single.params, k.k0, k.k1)
    g = rng(81)
    B = 1027
    ops = g.integers(0, 10, B).astype(np.uint8)
    A, Bc = u32rand(g, B, k.p.n + 1), u32rand(g, B, k.p.n + 1)
    before = multi.device_bootstraps()
    got = multi.gate_batch(ops, A, Bc)
    ran = multi.device_bootstraps() - before
    assert ran.tolist() == [129] * 7 + [124]
    assert np.array_equal(got, single.gate_batch(ops, A, Bc))
    idx = np.array([0, 128, 129, 903, B - 1])  # shard boundaries
    assert np.array_equal(got[idx], oracle.gate_batch(k.p, ops[idx], A[idx], Bc[idx], k.ck, threads=5))
    # config 4's shape: independent AND / OR / XOR / MUX gates over their own inputs
    n = 1600
    c = tfhe_amd.Circuit()
    ins = [c.input() for _ in range(3 * n)]
    kinds = g.integers(0, 4, n)
    for j in range(n):
        x, y, z = ins[3 * j: 3 * j + 3]
        c.output([c.and_, c.or_, c.xor][kinds[j]](x, y) if kinds[j] < 3 else c.mux(x, y, z))
    bits = g.integers(0, 2, 3 * n).astype(np.uint8)
    inputs = sk.encrypt_bool(bits, seed0=8100)
    want, depth1 = c.run(single, inputs)
    for split in (1, 2):  # components, then every level split over the 8 shards
        with multi.options(circuit_split=split):
            before = multi.device_bootstraps()
            got, depth = c.run(multi, inputs)
            ran = multi.device_bootstraps() - before
        assert depth == depth1 and np.array_equal(got, want), split
        assert ran.sum() == sum(1 for o in c.ops if o != tfhe_amd.NOT) and ran.min() > 0, ran
        assert ran.max() - ran.min() <= (len(c.ops) // 8) // 10 + 8, ran  # within ~10 % of an even share
        if split == 2:
            print(f"8-shard level split: issue {multi.get_option('level_issue_us')} us for {depth + 1} levels")
    b3 = bits.reshape(n, 3).astype(bool)
    truth = np.where(kinds == 0, b3[:, 0] & b3[:, 1], np.where(kinds == 1, b3[:, 0] | b3[:, 1],
                     np.where(kinds == 2, b3[:, 0] ^ b3[:, 1], np.where(b3[:, 0], b3[:, 1], b3[:, 2]))))
    assert np.array_equal(sk.decrypt_bool(want), truth)
    single.close()
    multi.close()
    # UINT4 programmable bootstrap over 8 shards (config 5's 8-GPU leg, 300 items)
    single, k = loaded(oracle, "uint4")
    multi, _ = loaded(oracle, "uint4", devices=[0] * 8)
    sk = tfhe_amd.SecretKey(single.params, k.k0, k.k1)
    tv = tfhe_amd.lut_generate(single.params, 16, lambda x: (x * x + 3) % 16)
    msgs = g.integers(0, 16, 300).astype(np.uint32)
    cts = sk.encrypt_lwe_message(msgs, 16, seed0=8200)
    got = multi.bootstrap_lut_batch(cts, tv)
    assert np.array_equal(got, single.bootstrap_lut_batch(cts, tv))
    assert np.array_equal(sk.decrypt_lwe_message(got, 16), (msgs * msgs + 3) % 16)
    single.close()
    multi.close()


def test_lut_dev_refuses_multi_device_context(oracle):
    """tfhe_gpu_bootstrap_lut_batch_dev takes single-device contexts, like its
    _dev siblings: a multi-device context is refused (TFHE_ERR_INVALID) instead
    of silently running on the first device."""
    multi, _ = loaded(oracle, "80", devices=[0, 0])
    with pytest.raises(tfhe_amd.TfheError) as e:
        multi.bootstrap_lut_batch_dev(64, 64, 64, 1)  # never dereferenced: refused first
    assert e.value.status == tfhe_amd.ERR_INVALID and "single-device" in str(e.value)
    multi.close()


def test_host_staging_modes_same_words(oracle):
    """TFHE_OPT_HOST_STAGING (round 6): the host-buffer entries of an
    8-shard context through pageable copies (0, the default) and per-device pinned
    staging (1) give the same words as one device, on a ragged gate batch, a bootstrap
    batch and a blind rotation (TRLWE outputs, the largest D2H), the arena reused
    across calls; staging forced on a single-device context too."""
    single, k = loaded(oracle, "80")
    multi, _ = loaded(oracle, "80", devices=[0] * 8)
    assert multi.get_option("host_staging") == tfhe_amd.STAGING_PAGEABLE
    g = rng(83)
    B = 1030
    ops = g.integers(0, 10, B).astype(np.uint8)
    A, Bc = u32rand(g, B, k.p.n + 1), u32rand(g, B, k.p.n + 1)
    want = single.gate_batch(ops, A, Bc)
    want_bs = single.bootstrap_batch(A[:77])
    want_br = single.blind_rotate_batch(Bc[:40])
    for mode in (tfhe_amd.STAGING_PINNED, tfhe_amd.STAGING_PAGEABLE):
        with multi.options(host_staging=mode):
            for _ in range(2):  # the arena reused from offset 0 after each synchronisation
                assert np.array_equal(multi.gate_batch(ops, A, Bc), want), mode
            assert np.array_equal(multi.bootstrap_batch(A[:77]), want_bs), mode
            assert np.array_equal(multi.blind_rotate_batch(Bc[:40]), want_br), mode
    with single.options(host_staging=tfhe_amd.STAGING_PINNED):  # forced on one device
        assert np.array_equal(single.gate_batch(ops, A, Bc), want)
    idx = np.array([0, 129, 903, B - 1])
    assert np.array_equal(want[idx], oracle.gate_batch(k.p, ops[idx], A[idx], Bc[idx], k.ck, threads=4))
    single.close()
    multi.close()
