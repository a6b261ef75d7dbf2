"""Error behaviour of the C ABI on a device (include/tfhe_gpu.h status codes).

The reference reports failures as Zig error unions (`!TLWELv0`, `vanilla.zig:38`;
`CloudKey.new` / `Gates` calls, `key.zig:70-77`, `gates.zig:48-121`); the drop-in
boundary maps them to negative status codes.  These tests pin that mapping: a
bootstrap before any cloud key is TFHE_ERR_NO_KEY, a bad argument is
TFHE_ERR_INVALID, and a refused call leaves the context usable — the next valid
batch is still bit-exact against the oracle.
"""
import ctypes as C

import numpy as np
import pytest

import tfhe_amd
from conftest import get_keys

pytestmark = pytest.mark.gpu

ERR_INVALID, ERR_NO_KEY = -1, -3


def _status(exc: tfhe_amd.TfheError) -> int:
    msg = str(exc)
    return int(msg.split("status ")[1].split(":")[0])


def _inputs(p, B, seed):
    g = np.random.default_rng(seed)
    return g.integers(0, 1 << 32, (B, p.n + 1), dtype=np.uint64).astype(np.uint32)


def test_bootstrap_before_cloud_key_is_no_key():
    ctx = tfhe_amd.Context("80", 0)
    try:
        p = ctx.params
        a, b = _inputs(p, 3, 1), _inputs(p, 3, 2)
        calls = [
            lambda: ctx.gate_batch(np.zeros(3, np.uint8), a, b),
            lambda: ctx.bootstrap_batch(a),
            lambda: ctx.blind_rotate_batch(a),
        ]
        for call in calls:
            with pytest.raises(tfhe_amd.TfheError) as e:
                call()
            assert _status(e.value) == ERR_NO_KEY
            assert "no cloud key" in str(e.value)
    finally:
        ctx.close()


def test_refused_calls_leave_the_context_usable(oracle):
    k = get_keys(oracle, "80")
    p = k.p
    ctx = tfhe_amd.Context("80", 0)
    try:
        # a key of the wrong shape is refused and nothing is loaded
        with pytest.raises(tfhe_amd.TfheError) as e:
            ctx.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk.reshape(-1)[:-1], k.ck.ksk)
        assert _status(e.value) == ERR_INVALID
        with pytest.raises(tfhe_amd.TfheError) as e:
            ctx.gate_batch(np.zeros(1, np.uint8), _inputs(p, 1, 3), _inputs(p, 1, 4))
        assert _status(e.value) == ERR_NO_KEY

        ctx.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk, k.ck.ksk)
        a, b = _inputs(p, 5, 5), _inputs(p, 5, 6)
        # an op code outside gates.zig's ten (and not COPY) is refused before any launch
        bad = np.array([0, 1, 2, 10, 3], np.uint8)
        with pytest.raises(tfhe_amd.TfheError) as e:
            ctx.gate_batch(bad, a, b)
        assert _status(e.value) == ERR_INVALID and "bad gate op" in str(e.value)

        # null buffers with B > 0, straight through the C ABI
        lib = ctx.lib
        rc = lib.tfhe_gpu_gate_batch(ctx.h, None, None, None, None, C.c_size_t(4))
        assert rc == ERR_INVALID
        rc = lib.tfhe_gpu_bootstrap_batch(ctx.h, None, None, C.c_size_t(4))
        assert rc == ERR_INVALID
        # B = 0 with null buffers is a no-op, not an error
        assert lib.tfhe_gpu_gate_batch(ctx.h, None, None, None, None, C.c_size_t(0)) == 0

        # the context still computes the reference's words
        ops = np.array([0, 1, 2, 9, 3], np.uint8)
        got = ctx.gate_batch(ops, a, b)
        want = oracle.gate_batch(p, ops, a, b, k.ck, threads=4)
        assert np.array_equal(got, want)
    finally:
        ctx.close()


def test_slot_protocol_failure_is_reported_not_returned(oracle):
    """The whole form's slot-counter waits are bounded (tfhe_kernels.hip
    spin_until_ge).  A wait that gives up must fail the call, never hand back
    the words of a broken launch as TFHE_OK: with the bound forced down to one
    poll (TFHE_OPT_BR_SPIN_CAP = 1; a loader waits ~24 k cycles per step for
    the gates) the gate batch returns TFHE_ERR_DEVICE, the device error word is
    cleared, and with the default bound the same context is bit-exact again."""
    k = get_keys(oracle, "128")
    p = k.p
    ctx = tfhe_amd.Context("128", 0)
    try:
        ctx.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk, k.ck.ksk)
        ctx.set_option("br_form", "whole")  # the slot-counter form at any batch size
        assert ctx.get_option("br_sync") == 1 and ctx.get_option("br_loader") == 1
        a, b = _inputs(p, 8, 11), _inputs(p, 8, 12)
        ops = np.zeros(8, np.uint8)
        with ctx.options(br_spin_cap=1):
            with pytest.raises(tfhe_amd.TfheError) as e:
                ctx.gate_batch(ops, a, b)
            assert e.value.status == tfhe_amd.ERR_DEVICE
            assert "slot-counter protocol failure" in str(e.value)
            # the device-pointer path surfaces it at the next synchronisation
            import torch
            dev = torch.device("cuda", 0)
            t_ops = torch.zeros(8, dtype=torch.uint8, device=dev)
            t_a = torch.from_numpy(a.view(np.int32)).to(dev)
            t_b = torch.from_numpy(b.view(np.int32)).to(dev)
            t_o = torch.zeros_like(t_a)
            torch.cuda.synchronize(dev)
            ctx.gate_batch_dev(t_ops.data_ptr(), t_a.data_ptr(), t_b.data_ptr(), t_o.data_ptr(), 8)
            with pytest.raises(tfhe_amd.TfheError) as e:
                ctx.sync()
            assert e.value.status == tfhe_amd.ERR_DEVICE
        assert ctx.get_option("br_spin_cap") == 0
        ctx.sync()  # cleared: nothing pending
        got = ctx.gate_batch(ops, a, b)
        want = oracle.gate_batch(p, ops, a, b, k.ck, threads=8)
        assert np.array_equal(got, want)
    finally:
        ctx.close()
