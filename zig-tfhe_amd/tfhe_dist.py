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


def broadcast_cloud_key(ctx, device, src: int = 0, group=None):
    """Rank `src` exports its device-resident key blob, every rank receives it
    by torch.distributed.broadcast (RCCL over xGMI for the nccl backend) and
    imports it.  Returns the number of bytes broadcast."""
    import numpy as np
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    bk_bytes, ksk_bytes = ctx.key_blob_bytes()
    bk = torch.empty(bk_bytes, dtype=torch.uint8, device=device)
    ksk = torch.empty(ksk_bytes, dtype=torch.uint8, device=device)
    meta = torch.zeros(1 + 2 * ctx.params.N, dtype=torch.int64, device=device)
    if rank == src:
        offset, tv = ctx.export_key_device(bk.data_ptr(), ksk.data_ptr())
        meta[0] = offset
        meta[1:] = torch.from_numpy(tv.astype(np.int64))
    for t in (bk, ksk, meta):
        dist.broadcast(t, src, group=group)
    if rank != src:
        torch.cuda.synchronize(device)
        m = meta.cpu().numpy()
        ctx.import_key_device(bk.data_ptr(), ksk.data_ptr(), int(m[0]), m[1:].astype(np.uint32))
    torch.cuda.synchronize(device)
    return bk_bytes + ksk_bytes
