"""A/B check of the whole form at L = 3 (since round 5 the loader-assist kernel,
k_blind_rotate_assist) against round 4's whole form (A/B form 8 "plain",
tools/ab/tfhe_ab_forms.hip) and the oracle: every idle-slot count, the three output
modes; then timing of one form (BR_FORM=whole|plain|auto).
Run with TFHE_ALLOW_AB_BUILD=1 TFHE_GPU_LIB=tools/bin/lib_ab.so.

    python tools/ab_assist_check.py parity        (FORM=n checks TFHE_OPT_BR_FORM n instead of the whole form)
    FORM=n python tools/ab_assist_check.py parity_sets   (the 80-bit and UINT4 sets)
    python tools/ab_assist_check.py time STEPS
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("zig-tfhe_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, sub))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (HIP runtime first)

import tfhe_amd  # noqa: E402


def u32rand(g, *shape):
    return g.integers(0, 1 << 32, shape, dtype=np.uint64).astype(np.uint32)


def parity():
    from oracle import Oracle, params
    f = os.environ.get("FORM", "whole")
    form = int(f) if f.isdigit() else f
    o = Oracle()
    p = params("128")
    k0, k1 = o.secret_key(p, 42)
    ck = o.cloud_key(p, 43, k0, k1)
    c = tfhe_amd.Context("128", 0)
    c.load_cloud_key(ck.offset, ck.testvec, ck.bk, ck.ksk)
    c.set_option("br_spin_cap", 1 << 16)  # a broken hand-off ends in ms, with TFHE_ERR_DEVICE
    g = np.random.default_rng(5)
    cts = u32rand(g, 9, p.n + 1)
    want = np.array([o.blind_rotate(p, t, ck.testvec, ck.bk, ck.offset) for t in cts[:3]])
    with c.options(br_form=form):
        got = c.blind_rotate_batch(cts[:3])
        print("kernel:", c.last_kernels())
    assert np.array_equal(got, want), "assist TRLWE != oracle"
    with c.options(br_form="plain"):
        ref9 = c.blind_rotate_batch(cts)
    with c.options(br_form=form):
        for B in range(1, 10):
            assert np.array_equal(c.blind_rotate_batch(cts[:B]), ref9[:B]), f"idle slots B={B}"
    print("TRLWE outputs bit-exact (oracle on 3, round 4's whole form at B = 1..9)")
    sk = tfhe_amd.SecretKey(c.params, k0, k1)
    a, b = g.integers(0, 2, 1024).astype(np.uint8), g.integers(0, 2, 1024).astype(np.uint8)
    A, Bc = sk.encrypt_bool(a, seed0=1), sk.encrypt_bool(b, seed0=5000)
    ops = g.integers(0, 10, 1024).astype(np.uint8)
    with c.options(br_form="plain"):
        ref = c.gate_batch(ops, A, Bc)
        ref2 = c.bootstrap_without_key_switch_batch(A[:37])
    with c.options(br_form=form):
        out = c.gate_batch(ops, A, Bc)
        out2 = c.bootstrap_without_key_switch_batch(A[:37])
    assert np.array_equal(out, ref), f"gate batch: {(out != ref).any(axis=1).sum()} gates differ"
    assert np.array_equal(out2, ref2)
    idx = np.array([0, 513, 1023])
    assert np.array_equal(out[idx], o.gate_batch(p, ops[idx], A[idx], Bc[idx], ck, threads=3))
    print("1,024 mixed gates and 37 bootstraps without key switch: identical to round 4's whole form; oracle sample ok")
    print("near-tie items recomputed:", c.near_tie_items())
    c.close()


def parity_sets():
    """FORM=n at the 80-bit and UINT4 sets (UINT4: reference trees, L = 1): the oracle on 3
    rotations, and the product's default form (auto) on 64, every output word."""
    from oracle import Oracle, params
    form = int(os.environ["FORM"])
    o = Oracle()
    for name in ("80", "uint4"):
        p = params(name)
        k0, k1 = o.secret_key(p, 42)
        ck = o.cloud_key(p, 43, k0, k1)
        c = tfhe_amd.Context(name, 0)
        c.load_cloud_key(ck.offset, ck.testvec, ck.bk, ck.ksk)
        g = np.random.default_rng(7)
        cts = u32rand(g, 64, p.n + 1)
        want = np.array([o.blind_rotate(p, t, ck.testvec, ck.bk, ck.offset) for t in cts[:3]])
        ref = c.blind_rotate_batch(cts)
        auto = c.last_kernels()
        with c.options(br_form=form):
            got = c.blind_rotate_batch(cts)
            kern = c.last_kernels()
        assert np.array_equal(got[:3], want), f"{name}: form {form} != oracle"
        assert np.array_equal(got, ref), f"{name}: form {form} != {auto}"
        print(f"{name}: {kern}: oracle on 3, the default form ({auto}) on 64: identical")
        c.close()


def timing(steps):
    c = tfhe_amd.Context("128", 0)
    sk, _ = c.keygen(42, 43)
    form = os.environ.get("BR_FORM", "auto")
    g = np.random.default_rng(1)
    a, b = g.integers(0, 2, 1024).astype(np.uint8), g.integers(0, 2, 1024).astype(np.uint8)
    dev = torch.device("cuda", 0)
    t_a = torch.from_numpy(sk.encrypt_bool(a, seed0=1).view(np.int32)).to(dev)
    t_b = torch.from_numpy(sk.encrypt_bool(b, seed0=5000).view(np.int32)).to(dev)
    t_o = torch.zeros_like(t_a)
    t_ops = torch.zeros(1024, dtype=torch.uint8, device=dev)
    c.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    c.set_option("br_form", form)
    for _ in range(3):
        c.gate_batch_dev(t_ops.data_ptr(), t_a.data_ptr(), t_b.data_ptr(), t_o.data_ptr(), 1024)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        c.gate_batch_dev(t_ops.data_ptr(), t_a.data_ptr(), t_b.data_ptr(), t_o.data_ptr(), 1024)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    c.sync()
    ok = np.array_equal(sk.decrypt_bool(t_o.cpu().numpy().view(np.uint32)), ~(a.astype(bool) & b.astype(bool)))
    print(f"{form} ({tfhe_amd.build_id()}): {el / steps * 1e3:.3f} ms per 1,024 NAND, {1024 * steps / el:.0f}/s, "
          f"decrypt {ok}, {c.last_kernels()}")
    c.set_stream(None)
    c.close()


if __name__ == "__main__":
    if sys.argv[1] == "parity":
        parity()
    elif sys.argv[1] == "parity_sets":
        parity_sets()
    else:
        timing(int(sys.argv[2]))
