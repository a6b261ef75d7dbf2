"""Multi-process paths: contiguous batch sharding, the one-time
cloud-key broadcast, and the gathered sharded gate batch.

CPU tests run world_size 2 over gloo with a host stand-in for the device
context (the protocol under test is tfhe_dist's, not the kernels'); the GPU
test round-trips a real key blob through export -> broadcast -> import into a
second context and checks gates through it against the oracle.
"""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import tfhe_dist


@pytest.mark.parametrize("total", [0, 1, 7, 1024, 1025, 65536])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_range_partitions(total, world):
    spans = [tfhe_dist.shard_range(total, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == total
    for (lo0, hi0), (lo1, hi1) in zip(spans, spans[1:]):
        assert hi0 == lo1
    sizes = [hi - lo for lo, hi in spans]
    assert max(sizes) - min(sizes) <= 1 and min(sizes) >= 0


class _HostParams:
    N = 1024


class HostCtx:
    """Stand-in for tfhe_amd.Context with 'device' buffers in host memory;
    gate_batch is a deterministic per-row function (not TFHE)."""

    params = _HostParams()

    def __init__(self, rank, bk_bytes=4096 + 16, ksk_bytes=8192 - 4):
        self.rank = rank
        self.sizes = (bk_bytes, ksk_bytes)
        g = np.random.default_rng(7)
        self.bk = g.integers(0, 256, bk_bytes, dtype=np.uint8)
        self.ksk = g.integers(0, 256, ksk_bytes, dtype=np.uint8)
        self.offset = 0x82080000
        self.tv = g.integers(0, 2**32, 2 * 1024, dtype=np.uint64).astype(np.uint32)
        if rank != 0:  # non-source ranks start without a key
            self.bk[:] = 0
            self.ksk[:] = 0
            self.offset, self.tv = 0, np.zeros_like(self.tv)

    def key_blob_bytes(self):
        return self.sizes

    def export_key_device(self, bk_ptr, ksk_ptr):
        ctypes.memmove(bk_ptr, self.bk.ctypes.data, self.bk.nbytes)
        ctypes.memmove(ksk_ptr, self.ksk.ctypes.data, self.ksk.nbytes)
        return self.offset, self.tv.copy()

    def import_key_device(self, bk_ptr, ksk_ptr, offset, tv):
        ctypes.memmove(self.bk.ctypes.data, bk_ptr, self.bk.nbytes)
        ctypes.memmove(self.ksk.ctypes.data, ksk_ptr, self.ksk.nbytes)
        self.offset, self.tv = offset, np.asarray(tv, np.uint32)
        if getattr(self, "corrupt_import", False):  # a broken transfer on this rank
            self.bk[17] ^= 0x40

    def key_fingerprint(self):
        """Stand-in for tfhe_gpu_key_fingerprint: an order-dependent 64-bit sum of the bytes."""
        def fp(a):
            w = np.arange(1, a.size + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
            return int(np.bitwise_xor.reduce(a.astype(np.uint64) * w + w) if a.size else 0)
        return fp(self.bk), fp(self.ksk)

    def gate_batch(self, ops, a, b):
        ops = np.asarray(ops, np.uint32)[:, None]
        return (np.asarray(a, np.uint32) * np.uint32(3) + np.asarray(b, np.uint32) + ops).astype(np.uint32)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = HostCtx(rank)
        nbytes = tfhe_dist.broadcast_cloud_key(ctx, "cpu", src=0)
        ref = HostCtx(0)
        key_ok = (np.array_equal(ctx.bk, ref.bk) and np.array_equal(ctx.ksk, ref.ksk)
                  and ctx.offset == ref.offset and np.array_equal(ctx.tv, ref.tv)
                  and nbytes == sum(ref.sizes))
        g = np.random.default_rng(11)
        B = 1001  # ragged over 2 ranks
        ops = g.integers(0, 10, B).astype(np.uint8)
        a = g.integers(0, 2**32, (B, 701), dtype=np.uint64).astype(np.uint32)
        b = g.integers(0, 2**32, (B, 701), dtype=np.uint64).astype(np.uint32)
        got = tfhe_dist.sharded_gate_batch(ctx, ops, a, b, rank, world)
        lo, hi = tfhe_dist.shard_range(B, rank, world)
        local = tfhe_dist.sharded_gate_batch(ctx, ops, a, b, rank, world, gather=False)
        out_ok = (np.array_equal(got, ctx.gate_batch(ops, a, b))
                  and np.array_equal(local, ctx.gate_batch(ops[lo:hi], a[lo:hi], b[lo:hi])))
        q.put((rank, key_ok, out_ok))
    finally:
        dist.destroy_process_group()


def _worker_corrupt(rank, world, port, bad_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = HostCtx(rank)
        ctx.corrupt_import = rank == bad_rank
        try:
            tfhe_dist.broadcast_cloud_key(ctx, "cpu", src=0)
            q.put((rank, "ok"))
        except RuntimeError as e:
            q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


def test_gloo_key_broadcast_fingerprint_mismatch_fails_every_rank():
    """A rank whose imported key differs from the source's (a flipped byte in
    its import) makes broadcast_cloud_key raise on EVERY rank, naming that rank
    (the cross-rank counterpart of the in-library broadcast's fingerprint check)."""
    world, bad = 3, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_corrupt, args=(r, world, port, bad, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r for r, _ in res] == list(range(world))
    for _, msg in res:
        assert "differs" in msg and f"[{bad}]" in msg, msg


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_key_broadcast_and_sharded_batch(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r for r, _, _ in res] == list(range(world))
    assert all(k for _, k, _ in res), res
    assert all(o for _, _, o in res), res


@pytest.mark.gpu
@pytest.mark.parametrize("backend", ["gloo", "nccl"])
def test_key_blob_roundtrip_through_broadcast(oracle, backend):
    """export (ctx 0) -> torch.distributed.broadcast (world 1, device tensors) ->
    import (ctx 1); gates through ctx 1 equal the oracle's.  The nccl case runs
    the bench's multi-rank key path through RCCL itself (one rank: the box has one
    GPU), fingerprint all-gather included."""
    import tfhe_amd
    from conftest import get_keys

    k = get_keys(oracle, "80")
    port = _free_port()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if backend == "nccl":
        torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=0, world_size=1)
    try:
        dev = torch.device("cuda", 0)
        c0 = tfhe_amd.Context("80", 0)
        c0.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk, k.ck.ksk)
        n = tfhe_dist.broadcast_cloud_key(c0, dev)  # src rank exports (and keeps) its key
        assert n == sum(c0.key_blob_bytes())
        bk_b, ksk_b = c0.key_blob_bytes()
        bk = torch.empty(bk_b, dtype=torch.uint8, device=dev)
        ksk = torch.empty(ksk_b, dtype=torch.uint8, device=dev)
        off, tv = c0.export_key_device(bk.data_ptr(), ksk.data_ptr())
        torch.cuda.synchronize(dev)
        c1 = tfhe_amd.Context("80", 0)
        c1.import_key_device(bk.data_ptr(), ksk.data_ptr(), off, tv)
        g = np.random.default_rng(3)
        ops = np.arange(10, dtype=np.uint8)
        A = np.array([oracle.tlwe_encrypt_bool(k.p.n, int(x), k.p.alpha_lv0, k.k0, 300 + i)
                      for i, x in enumerate(g.integers(0, 2, 10))])
        Bc = np.array([oracle.tlwe_encrypt_bool(k.p.n, int(x), k.p.alpha_lv0, k.k0, 400 + i)
                       for i, x in enumerate(g.integers(0, 2, 10))])
        want = oracle.gate_batch(k.p, ops, A, Bc, k.ck, threads=8)
        assert np.array_equal(c1.gate_batch(ops, A, Bc), want)
        assert np.array_equal(tfhe_dist.sharded_gate_batch(c1, ops, A, Bc, 0, 1), want)
        c0.close()
        c1.close()
    finally:
        dist.destroy_process_group()


def _worker_subgroup(rank, world, port, corrupt, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        group = dist.new_group([1, 2])  # every rank takes part in new_group
        if rank == 0:
            q.put((rank, "not in group", True))
            return
        ctx = HostCtx(0 if rank == 1 else 1)  # global rank 1 holds the key, rank 2 has none
        ctx.corrupt_import = corrupt and rank == 2
        try:
            tfhe_dist.broadcast_cloud_key(ctx, "cpu", src=1, group=group)
            ref = HostCtx(0)
            q.put((rank, "ok", np.array_equal(ctx.bk, ref.bk) and np.array_equal(ctx.ksk, ref.ksk)
                   and np.array_equal(ctx.tv, ref.tv)))
        except RuntimeError as e:
            q.put((rank, str(e), False))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("corrupt", [False, True])
def test_gloo_key_broadcast_in_a_subgroup(corrupt):
    """broadcast_cloud_key / check_key_fingerprints over a process subgroup
    {1, 2} of a world of 3 with src = global rank 1 (group rank 0): torch's
    broadcast takes the global rank, the all-gather list is indexed by group
    rank.  The key arrives on rank 2; a corrupted import there is
    named by its GLOBAL rank on both members."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_subgroup, args=(r, world, port, corrupt, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r for r, _, _ in res] == [0, 1, 2]
    for r, msg, ok in res[1:]:
        if corrupt:
            assert "differs" in msg and "[2]" in msg and "rank 1's" in msg, msg
        else:
            assert msg == "ok" and ok, (r, msg)
