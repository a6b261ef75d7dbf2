"""Multi-GPU plumbing: one process per MI355X, torch.distributed (RCCL over
xGMI) used only for the one-time cloud-key broadcast and for timing
reductions.  Gate batches shard into contiguous slices with no collective on
the data path: every gate bootstrap is independent.
"""
from __future__ import annotations

import os


def env_rank_world():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def shard_range(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous slice [lo, hi) of `total` items for `rank` (sizes differ by at most 1)."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _sync(device):
    import torch
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)


def _group_rank(group, global_rank: int) -> int:
    """Rank within `group` of a global rank (torch.distributed's collectives
    take `src` as a global rank; get_rank(group) and all_gather lists are
    indexed by group rank)."""
    import torch.distributed as dist
    return global_rank if group is None else dist.get_group_rank(group, global_rank)


def broadcast_cloud_key(ctx, device, src: int = 0, group=None):
    """Rank `src` (a global rank, a member of `group`) exports its device-resident key blob (BK in the device
    layout, KSK, decomposition offset, test vector); every rank receives it by
    torch.distributed.broadcast — RCCL over xGMI for the nccl backend, one
    bucket per tensor — and imports it.  Nothing else crosses devices: this
    replaces the reference's per-process CloudKey.new (key.zig:70-77) on ranks
    other than `src`.  Returns the number of bytes broadcast.

    `ctx` needs key_blob_bytes / export_key_device / import_key_device /
    params.N (tfhe_amd.Context; the gloo tests pass a host stand-in)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    is_src = dist.get_rank(group) == _group_rank(group, src)
    bk_bytes, ksk_bytes = ctx.key_blob_bytes()
    bk = torch.empty(bk_bytes, dtype=torch.uint8, device=device)
    ksk = torch.empty(ksk_bytes, dtype=torch.uint8, device=device)
    meta = torch.zeros(1 + 2 * ctx.params.N, dtype=torch.int64, device=device)
    if is_src:
        offset, tv = ctx.export_key_device(bk.data_ptr(), ksk.data_ptr())
        _sync(device)
        meta[0] = offset
        meta[1:] = torch.from_numpy(np.asarray(tv).astype(np.int64))
    for t in (bk, ksk, meta):
        dist.broadcast(t, src, group=group)
    if not is_src:
        _sync(device)
        m = meta.cpu().numpy()
        ctx.import_key_device(bk.data_ptr(), ksk.data_ptr(), int(m[0]), m[1:].astype(np.uint32))
    _sync(device)
    check_key_fingerprints(ctx, device, src, group)
    return bk_bytes + ksk_bytes


def check_key_fingerprints(ctx, device, src: int = 0, group=None):
    """Every rank's resident key must fingerprint like (global) rank `src`'s
    (tfhe_gpu_key_fingerprint, the same check the in-library multi-device
    broadcast makes): all-gather the (bk, ksk) sums and raise on any rank whose
    copy differs, naming it, on EVERY rank (no rank runs gates on a key that
    some rank holds differently)."""
    import torch
    import torch.distributed as dist

    bk_fp, ksk_fp = ctx.key_fingerprint()
    fdev = "cpu" if dist.get_backend(group) == "gloo" else device  # RCCL needs device tensors
    mine = torch.tensor([bk_fp - (1 << 63), ksk_fp - (1 << 63)], dtype=torch.int64, device=fdev)  # u64 -> i64
    parts = [torch.empty_like(mine) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, mine, group=group)
    want = parts[_group_rank(group, src)].cpu()
    bad = [r for r, t in enumerate(parts) if not torch.equal(t.cpu(), want)]
    if bad:  # name the global ranks
        bad = bad if group is None else [dist.get_global_rank(group, r) for r in bad]
        raise RuntimeError(f"cloud-key broadcast: the key on rank(s) {bad} differs from rank {src}'s "
                           f"(fingerprints {[tuple(int(x) + (1 << 63) for x in t.cpu()) for t in parts]})")


def sharded_gate_batch(ctx, ops, a, b, rank: int, world: int, gather: bool = True, group=None):
    """Data-parallel gate batch: rank r bootstraps the contiguous slice
    shard_range(B, r, world) of the global batch on its own GPU (no collective
    on the data path).  With gather=True the slices are all-gathered (host
    side, once, after the work) so every rank returns the whole batch's
    outputs in order — what a single Gates.*Gate loop over the batch returns."""
    import numpy as np

    lo, hi = shard_range(len(ops), rank, world)
    out = ctx.gate_batch(np.asarray(ops)[lo:hi], np.asarray(a)[lo:hi], np.asarray(b)[lo:hi])
    if not gather or world == 1:
        return out
    import torch.distributed as dist
    parts = [None] * world
    dist.all_gather_object(parts, (lo, out), group=group)
    return np.concatenate([o for _, o in sorted(parts, key=lambda x: x[0])], axis=0)
