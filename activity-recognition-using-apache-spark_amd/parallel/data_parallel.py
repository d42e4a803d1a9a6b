"""Data-parallel training over one process per GPU.

The reference's only parallelism is Spark's implicit row partitioning with
``treeAggregate`` / ``reduceByKey`` combines.  Here each
rank owns a contiguous shard of the windows (global row ids are preserved so
every Philox draw — split, folds, bootstrap — is shard-independent) and the
combines are RCCL collectives over xGMI:

* LogisticRegression: one flat ``all_reduce`` of [loss | dW | db] per objective
  evaluation (~75 KB per model: latency-bound, so one bucket, never per tensor);
* RandomForest: per level, the (tree, node, feature, bin, class) histograms are
  either summed with one ``all_reduce`` (every rank then searches every split), or
  — the default, ``NodeOwner`` — ``reduce_scatter``-ed by node owner: each rank sums
  and searches only its slice of the nodes and one ``all_gather`` of the packed
  winners (3 + 2K floats per node) gives everybody the level's splits.  Half the
  histogram bytes on the wire and no redundant split search (Spark:
  ``reduceByKey(node)`` + ``collectAsMap``);
* RandomForest, tree-parallel (``fit_forest_tree_parallel``): every rank grows a slice of the
  trees over all rows; one all-gather of the node arrays at the end;
* MLP: ONE all-reduce of the flat fp32 gradient per step (~0.34 MB: a latency-bound message on
  xGMI, where splitting it into buckets only adds per-collective latency), between the
  deterministic slab reduction and Adam — the N = 1 step runs the same kernels with Adam fused
  into the reduction (``MLPEngine.train_step``).

``gloo`` runs the identical code on CPU for the multi-process tests.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from ..ops import tree as T
from . import comm
from .dist import DistContext, shard_range


def allreduce_sum(ctx: Optional[DistContext]):
    if ctx is None or not ctx.collective:
        return None

    def _ar(t: torch.Tensor):
        comm.all_reduce(t, group=ctx.group)  # (staged when the placement is not the backend's)
    return _ar


def shard(X: torch.Tensor, y: torch.Tensor, ctx: DistContext):
    """This rank's contiguous row shard and its global row offset."""
    lo, hi = shard_range(X.shape[0], ctx.rank, ctx.world_size)
    return X[lo:hi], y[lo:hi], lo


def fit_logreg_dp(estimator, X_shard, y_shard, specs, num_classes, ctx: DistContext):
    return estimator.fit_many(X_shard, y_shard, specs, num_classes, allreduce=allreduce_sum(ctx))


def global_thresholds(X_shard: torch.Tensor, max_bins: int, ctx: DistContext, sample_rows: int = 10000,
                      seed: int = 0):
    """findSplits over the whole (sharded) table, as Spark samples the whole RDD.

    The sample is a Philox Bernoulli draw keyed by global row id (``T.threshold_sample_mask``),
    so it is the single-process sample for any world size.  Each rank keeps its sampled rows,
    one all-gather (sizes first: shards may differ) puts the union — in global row order — on
    every rank, and every rank runs the device findSplits on it: the same thresholds as a
    single process, on every rank, without a broadcast."""
    X = X_shard.detach().float()
    if not ctx.collective:
        return T.thresholds_for(X, max_bins, sample_rows, seed)
    P = ctx.world_size

    def gather_sizes(v: int):
        # one all-gather of a [1] tensor per rank, ONE host read of all P sizes
        t = torch.tensor([v], dtype=torch.int64, device=X.device)
        out = torch.empty(P, dtype=torch.int64, device=X.device)
        comm.all_gather_into_tensor(out, t, group=ctx.group)
        return out.tolist()

    shard_rows = gather_sizes(X.shape[0])
    n_total, row0 = sum(shard_rows), sum(shard_rows[:ctx.rank])
    keep = T.threshold_sample_mask(X.shape[0], max_bins, sample_rows, seed, row0, n_total, device=X.device)
    take = X if keep is None else X[keep]
    counts = gather_sizes(take.shape[0])
    buf = torch.zeros(max(counts), X.shape[1], dtype=X.dtype, device=X.device)
    buf[:take.shape[0]] = take
    parts = torch.empty(P * buf.shape[0], X.shape[1], dtype=X.dtype, device=X.device)
    comm.all_gather_into_tensor(parts, buf, group=ctx.group)
    parts = parts.view(P, buf.shape[0], X.shape[1])
    sample = torch.cat([parts[q, :c] for q, c in enumerate(counts)], 0)
    # already sampled: no second draw (n_total <= sample_rows disables it)
    return T.thresholds_for(sample, max_bins, sample_rows=max(sample_rows, sample.shape[0]), seed=seed)


class NodeOwner:
    """Owner-computes reduction of per-node tensors ``[A, ...]``: node ``a`` belongs to
    rank ``a // ceil(A / P)`` (contiguous slices, so a slice is one contiguous buffer).

    The send / receive buffers are grow-only workspaces kept for the lifetime of the object
    (one fit): a level reuses them as views instead of allocating and padding fresh tensors.
    ``stats`` counts the collectives issued and their bytes (bench records).  On a forced 1-rank
    group (``HAR_DIST_FORCE_PG=1``) the collectives are issued too (an identity over one rank), so
    the owner path runs through a real communicator on one GPU (tests/test_gpu_rccl.py)."""

    def __init__(self, ctx: DistContext):
        self.ctx = ctx
        self.solo = ctx.world_size == 1 and not ctx.forced  # no group: nothing to reduce
        self.allreduce = allreduce_sum(ctx) or (lambda t: None)
        self._ws = {}
        self.stats = {"reduce_scatter": 0, "all_gather": 0, "bytes": 0}

    def _buf(self, name: str, numel: int, dtype, device) -> torch.Tensor:
        key = (name, dtype, str(device))
        t = self._ws.get(key)
        if t is None or t.numel() < numel:
            t = torch.empty(max(numel, 2 * (0 if t is None else t.numel())), dtype=dtype, device=device)
            self._ws[key] = t
        return t[:numel]

    def _dev(self):
        # RCCL needs device tensors (host tensors are staged through HBM), gloo host tensors
        return self.ctx.device if self.ctx.backend == "nccl" else torch.device("cpu")

    def reduce_scatter(self, hist: torch.Tensor):
        P, r = self.ctx.world_size, self.ctx.rank
        A = hist.shape[0]
        S = max(1, -(-A // P))
        a0, a1 = min(A, r * S), min(A, (r + 1) * S)
        if self.solo:
            return hist, 0, A
        flat = hist.reshape(A, -1)
        w = flat.shape[1]
        dev = self._dev() or flat.device
        src = self._buf("rs_src", P * S * w, flat.dtype, dev).view(P * S, w)
        src[:A].copy_(flat)
        src[A:].zero_()  # only the pad rows of the last owner's slice
        out = self._buf("rs_out", S * w, flat.dtype, dev).view(S, w)
        comm.reduce_scatter_tensor(out, src, group=self.ctx.group)
        self.stats["reduce_scatter"] += 1
        self.stats["bytes"] += src.numel() * src.element_size()
        return out.to(hist.device).view(S, *hist.shape[1:]), a0, a1

    def reduce_scatter_store(self, store: torch.Tensor, A: int, narrow: bool = False):
        """Owner reduction of a per-node store that already has the owner padding ([P * S, w], rows
        past A never read): no staging copy when the store lives where the backend reduces (device
        tensors under RCCL); ``narrow`` sends it as fp16 (the caller guarantees exact values).
        Returns (this rank's summed slice [S, w] fp32, a0, a1)."""
        P, r = self.ctx.world_size, self.ctx.rank
        S = max(1, -(-A // P))
        a0, a1 = min(A, r * S), min(A, (r + 1) * S)
        if self.solo:
            return store[:A], 0, A
        w = store.shape[1]
        dev = self._dev() or store.device
        dt = torch.float16 if narrow else store.dtype
        src = store if (store.device == torch.device(dev) and dt == store.dtype) else store.to(dev, dt)
        out = self._buf("rs_out16" if narrow else "rs_out", S * w, dt, dev).view(S, w)
        comm.reduce_scatter_tensor(out, src, group=self.ctx.group)
        self.stats["reduce_scatter"] += 1
        self.stats["bytes"] += src.numel() * src.element_size()
        return out.to(store.device, torch.float32), a0, a1

    def words_buffer(self, numel: int, device) -> torch.Tensor:
        """The packed DP send buffer (int32 words, on the device the pack kernel writes)."""
        return self._buf("pk_src", numel, torch.int32, device)

    def reduce_scatter_words(self, send: torch.Tensor, wmax: int, device) -> torch.Tensor:
        """Integer-sum reduce-scatter of the packed [P, wmax] int32 rows (field-exact: see
        csrc/kernels/tree_dp.hip); returns this rank's summed row on ``device``."""
        P = self.ctx.world_size
        dev = self._dev() or device
        src = send if send.device == torch.device(dev) else send.to(dev)
        out = self._buf("pk_out", wmax, torch.int32, dev)
        comm.reduce_scatter_tensor(out, src, group=self.ctx.group)
        self.stats["reduce_scatter"] += 1
        self.stats["bytes"] += src.numel() * src.element_size()
        return out.to(device)

    def all_gather_ranges(self, local: torch.Tensor, bounds) -> torch.Tensor:
        """All-gather of per-rank rows of unequal counts (rank r holds rows bounds[r] .. bounds[r+1]-1):
        every rank pads to the largest range; returns the [bounds[-1], ...] concatenation."""
        P = self.ctx.world_size
        sizes = [bounds[q + 1] - bounds[q] for q in range(P)]
        S = max(1, max(sizes))
        inner = tuple(local.shape[1:])
        w = int(np.prod(inner)) if inner else 1
        dev = self._dev() or local.device
        buf = self._buf("ag_src", S * w, local.dtype, dev).view(S, w)
        buf[: local.shape[0]].copy_(local.reshape(local.shape[0], w))
        buf[local.shape[0]:].zero_()
        out = self._buf("ag_out", P * S * w, local.dtype, dev).view(P, S, w)
        comm.all_gather_into_tensor(out.view(P * S, w), buf, group=self.ctx.group)
        self.stats["all_gather"] += 1
        self.stats["bytes"] += out.numel() * out.element_size()
        full = torch.cat([out[q, :sizes[q]] for q in range(P)], 0)
        return full.view((bounds[-1],) + inner).to(local.device).clone()

    def all_gather(self, local: torch.Tensor, A: int) -> torch.Tensor:
        P = self.ctx.world_size
        if self.solo:
            return local
        S = max(1, -(-A // P))
        inner = tuple(local.shape[1:])
        w = int(np.prod(inner)) if inner else 1
        dev = self._dev() or local.device
        buf = self._buf("ag_src", S * w, local.dtype, dev).view(S, w)
        buf[: local.shape[0]].copy_(local.reshape(local.shape[0], w))
        buf[local.shape[0]:].zero_()
        out = self._buf("ag_out", P * S * w, local.dtype, dev).view(P * S, w)
        comm.all_gather_into_tensor(out, buf, group=self.ctx.group)
        self.stats["all_gather"] += 1
        self.stats["bytes"] += out.numel() * out.element_size()
        return out[:A].view((A,) + inner).to(local.device).clone()


def fit_forest_dp(estimator, X_shard, y_shard, num_classes: int, row_offset: int, ctx: DistContext,
                  reduction: str = "owner"):
    """``reduction``: ``owner`` (reduce-scatter + all-gather of winners) or ``allreduce``."""
    thr = global_thresholds(X_shard, estimator.maxBins, ctx, seed=estimator.seed)
    if reduction == "owner" and ctx.collective:
        return estimator.fit_tensors(X_shard, y_shard, num_classes, row_offset=row_offset, thresholds=thr,
                                     owner=NodeOwner(ctx))
    return estimator.fit_tensors(X_shard, y_shard, num_classes, allreduce=allreduce_sum(ctx), row_offset=row_offset,
                                 thresholds=thr)


def fit_forest_tree_parallel(estimator, X, y, num_classes: int, ctx: DistContext, thresholds=None, stats=None,
                             hybrid=None):
    """Tree parallelism: every rank holds ALL rows and grows its contiguous
    slice of the forest's trees — keyed by global tree id, so bootstraps and feature subsets
    are those of the single-process forest — with zero communication until ONE all-gather at the
    end: each rank packs its node arrays (feature, threshold, children, class stats, gains, node
    counts, depth) as 32-bit words into one [trees-per-rank, words] buffer.  The result equals the
    single-process forest.  Pays when the binned table fits every GPU (288 GB each: config 5's
    480k x 165 features is ~80 MB) — per-level communication is then zero; row-sharded DP
    (``fit_forest_dp``) pays when rows are too many to replicate.  ``stats`` (a dict) receives the
    collective count and bytes."""
    from ..models.tree import ForestArrays, RandomForestClassificationModel

    T_, P, r = estimator.numTrees, ctx.world_size, ctx.rank
    lo, hi = (T_ * r) // P, (T_ * (r + 1)) // P
    if thresholds is None:
        thresholds = T.thresholds_for(X, estimator.maxBins, seed=estimator.seed)
    part = estimator.fit_tensors(X, y, num_classes, thresholds=thresholds, tree_offset=lo, num_trees=hi - lo,
                                 hybrid=hybrid)
    if not ctx.collective:
        return part
    a = part.arrs
    S = -(-T_ // P)  # trees per rank, padded
    Tr, maxn = a.feature.shape
    K = a.stats.shape[2]
    dev = ctx.device if ctx.backend == "nccl" else torch.device("cpu")

    def words(t: torch.Tensor) -> torch.Tensor:  # [Tr, ...] -> [Tr, w] int32 words
        t = t.to(dev).contiguous()
        n = int(np.prod(t.shape[1:])) if t.dim() > 1 else 1
        return (t.view(torch.int32) if t.dtype in (torch.int32, torch.float32) else t.to(torch.int32)).reshape(Tr, n)

    gain = a.gain if a.gain is not None else torch.zeros(Tr, maxn, device=a.feature.device)
    nn = torch.as_tensor(np.asarray(a.n_nodes), dtype=torch.int32)
    depth = torch.full((Tr, 1), int(a.max_depth), dtype=torch.int32)
    cols = [words(a.feature), words(a.threshold), words(a.left), words(a.right), words(a.stats), words(gain),
            words(nn.view(-1, 1)), words(depth)]
    w = sum(c.shape[1] for c in cols)
    buf = torch.zeros(S, w, dtype=torch.int32, device=dev)
    if Tr:
        buf[:Tr] = torch.cat(cols, dim=1)
    out = torch.empty(P * S, w, dtype=torch.int32, device=dev)
    comm.all_gather_into_tensor(out, buf, group=ctx.group)
    if stats is not None:
        stats["all_gather"] = stats.get("all_gather", 0) + 1
        stats["bytes"] = stats.get("bytes", 0) + out.numel() * 4
    keep = torch.cat([torch.arange(q * S, q * S + (T_ * (q + 1)) // P - (T_ * q) // P) for q in range(P)])
    full = out[keep.to(out.device)].to(a.feature.device)
    o = 0

    def take(n: int, dtype, shape):
        nonlocal o
        v = full[:, o:o + n].contiguous()
        o += n
        v = v.view(torch.float32) if dtype == torch.float32 else v
        return v.reshape((T_,) + shape)

    feature = take(maxn, torch.int32, (maxn,))
    threshold = take(maxn, torch.float32, (maxn,))
    left = take(maxn, torch.int32, (maxn,))
    right = take(maxn, torch.int32, (maxn,))
    st = take(maxn * K, torch.float32, (maxn, K))
    g = take(maxn, torch.float32, (maxn,))
    n_nodes = take(1, torch.int32, (1,)).view(-1).cpu().numpy().astype(np.int64)
    max_depth = int(take(1, torch.int32, (1,)).max())
    arrs = ForestArrays(feature, threshold, left, right, st, n_nodes, max_depth, g if a.gain is not None else None)
    return RandomForestClassificationModel(arrs, X.shape[1], num_classes, uid=estimator.uid, device=X.device)


def fit_mlp_dp(estimator, X_shard, y_shard, ctx: DistContext, num_classes: Optional[int] = None):
    return estimator.fit_tensors(X_shard, y_shard, process_group=ctx.group, rank=ctx.rank,
                                 world_size=ctx.world_size, num_classes=num_classes)
