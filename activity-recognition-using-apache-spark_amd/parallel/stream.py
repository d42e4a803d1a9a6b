"""Sharded raw-stream featurization with halo exchange.

A long accelerometer stream is split into contiguous per-rank shards (one
process per GPU).  Windows are defined on the *global* sample index (window j
starts at ``j * stride``); rank r owns every window whose start falls inside its
shard.  A window that starts near the end of a shard runs into the next rank's
samples, so before featurizing each rank receives the first ``window - 1``
samples of its right neighbour — one point-to-point exchange per boundary
(``batch_isend_irecv``: RCCL over xGMI on the GPU, gloo on the CPU), a few KB per
rank, instead of an all-gather of the stream.  The concatenation over ranks of
the owned windows equals featurizing the un-sharded stream.

The reference never sees raw samples (WISDM ships pre-windowed rows); this is
the north-star raw-ingest path (BASELINE config 4).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist

from ..features.window import WindowFeaturizer, window_count
from .dist import DistContext


def shard_offsets(ctx: DistContext, local_len: int, device) -> Tuple[int, int]:
    """(global offset of this rank's shard, total samples) from an all-gather of shard lengths."""
    if not ctx.is_distributed:
        return 0, local_len
    t = torch.tensor([local_len], dtype=torch.long, device=device)
    allv = [torch.zeros_like(t) for _ in range(ctx.world_size)]
    dist.all_gather(allv, t, group=ctx.group)
    lens = [int(v.item()) for v in allv]
    return sum(lens[: ctx.rank]), sum(lens)


def exchange_halo(ctx: DistContext, local: torch.Tensor, halo: int) -> torch.Tensor:
    """Return the first ``halo`` samples of rank r+1's shard (empty on the last rank)."""
    A = local.shape[1]
    if not ctx.is_distributed or halo == 0:
        return local.new_zeros(0, A)
    if local.shape[0] < halo and ctx.rank > 0:
        raise ValueError(f"shard of {local.shape[0]} samples is shorter than the halo ({halo})")
    ops = []
    recv = None
    if ctx.rank > 0:
        ops.append(dist.P2POp(dist.isend, local[:halo].contiguous(), ctx.rank - 1, group=ctx.group))
    if ctx.rank < ctx.world_size - 1:
        recv = local.new_empty(halo, A)
        ops.append(dist.P2POp(dist.irecv, recv, ctx.rank + 1, group=ctx.group))
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    return recv if recv is not None else local.new_zeros(0, A)


def sharded_window_features(ctx: DistContext, local: torch.Tensor, featurizer: WindowFeaturizer,
                            offset: Optional[int] = None, total: Optional[int] = None):
    """Featurize this rank's shard ``local`` [S_r, A] of a global stream.

    Returns ``(features [n_owned, F], first_window)`` where ``first_window`` is the
    global index of the first owned window (labels / ids line up with it)."""
    W, st = featurizer.window, featurizer.stride
    if offset is None or total is None:
        offset, total = shard_offsets(ctx, local.shape[0], local.device)
    ext = torch.cat([local, exchange_halo(ctx, local, W - 1)], 0)
    p0 = -(-offset // st) * st                       # first window start inside the shard
    end = offset + local.shape[0]
    n_starts = max(0, -(-(end - p0) // st))
    n_fit = window_count(min(total, offset + ext.shape[0]) - p0, W, st) if p0 < end else 0
    n = min(n_starts, n_fit)
    if n == 0:
        return local.new_zeros(0, len(featurizer.names)), p0 // st
    seg = ext[p0 - offset: p0 - offset + (n - 1) * st + W]
    return featurizer.transform(seg), p0 // st
