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

from typing import List, Optional, Tuple

import torch

from ..features.window import WindowFeaturizer, window_count
from . import comm
from .dist import DistContext


def shard_lengths(ctx: DistContext, local_len: int, device) -> List[int]:
    """Every rank's shard length (one all-gather of one integer; one host read)."""
    if not ctx.is_distributed:
        return [local_len]
    t = torch.tensor([local_len], dtype=torch.long, device=device)
    allv = torch.zeros(ctx.world_size, dtype=torch.long, device=device)
    comm.all_gather_into_tensor(allv, t, group=ctx.group)
    return [int(v) for v in allv.cpu().tolist()]


def shard_offsets(ctx: DistContext, local_len: int, device, lens: Optional[List[int]] = None) -> Tuple[int, int]:
    """(global offset of this rank's shard, total samples) from an all-gather of shard lengths."""
    lens = lens if lens is not None else shard_lengths(ctx, local_len, device)
    return sum(lens[: ctx.rank]), sum(lens)


def exchange_halo(ctx: DistContext, local: torch.Tensor, halo: int, lens: Optional[List[int]] = None) -> torch.Tensor:
    """Return the first ``halo`` samples of rank r+1's shard (empty on the last rank).

    Every rank validates EVERY shard length (from ``lens`` or one all-gather) before
    any point-to-point op is posted, so a too-short shard makes all ranks raise
    together instead of leaving its neighbours blocked in ``batch_isend_irecv``."""
    A = local.shape[1]
    if not ctx.is_distributed or halo == 0:
        return local.new_zeros(0, A)
    lens = lens if lens is not None else shard_lengths(ctx, local.shape[0], local.device)
    short = [r for r in range(1, ctx.world_size) if lens[r] < halo]
    if short:
        raise ValueError(f"shard(s) of rank(s) {short} ({[lens[r] for r in short]} samples) are shorter than "
                         f"the halo ({halo} samples)")
    sends, recvs = [], []
    recv = None
    if ctx.rank > 0:
        sends.append((local[:halo].contiguous(), ctx.rank - 1))
    if ctx.rank < ctx.world_size - 1:
        recv = local.new_empty(halo, A)
        recvs.append((recv, ctx.rank + 1))
    comm.send_recv(sends, recvs, group=ctx.group)
    return recv if recv is not None else local.new_zeros(0, A)


def sharded_window_features(ctx: DistContext, local: torch.Tensor, featurizer: WindowFeaturizer,
                            offset: Optional[int] = None, total: Optional[int] = None, transform=None):
    """Featurize this rank's shard ``local`` [S_r, A] of a global stream.

    Returns ``(features [n_owned, F], first_window)`` where ``first_window`` is the
    global index of the first owned window (labels / ids line up with it).  ``transform``
    (segment -> rows) replaces ``featurizer.transform``, e.g. the window kernel's fused
    MLP-input mode (``window_features_mlp``)."""
    W, st = featurizer.window, featurizer.stride
    lens = shard_lengths(ctx, local.shape[0], local.device)
    if offset is None or total is None:
        offset, total = shard_offsets(ctx, local.shape[0], local.device, lens)
    halo = exchange_halo(ctx, local, W - 1, lens)
    L = local.shape[0]
    p0 = -(-offset // st) * st                       # first window start inside the shard
    end = offset + L
    n_starts = max(0, -(-(end - p0) // st))
    n_fit = window_count(min(total, end + halo.shape[0]) - p0, W, st) if p0 < end else 0
    n = min(n_starts, n_fit)
    fn = transform or featurizer.transform
    if n == 0:
        return local.new_zeros(0, len(featurizer.names)), p0 // st
    # the windows that end inside the shard are featurized from the shard itself; only the (at most
    # (W - 1) / stride + 1) windows that run into the halo go through a small [their samples + halo]
    # segment — no concatenated copy of the whole shard (12 GB per pass for config 4's 1B-sample GPU)
    r0 = p0 - offset
    n_in = min(n, window_count(L - r0, W, st)) if L - r0 >= W else 0
    parts = []
    if n_in > 0:
        parts.append(fn(local[r0: r0 + (n_in - 1) * st + W]))
    if n > n_in:
        t0 = r0 + n_in * st
        tail = torch.cat([local[t0:], halo], 0)[: (n - n_in - 1) * st + W]
        parts.append(fn(tail))
    return (parts[0] if len(parts) == 1 else torch.cat(parts, 0)), p0 // st
