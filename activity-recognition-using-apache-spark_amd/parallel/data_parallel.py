"""Data-parallel training over one process per GPU.

The reference's only parallelism is Spark's implicit row partitioning with
``treeAggregate`` / ``reduceByKey`` combines.  Here each
rank owns a contiguous shard of the windows (global row ids are preserved so
every Philox draw — split, folds, bootstrap — is shard-independent) and the
combines are RCCL collectives over xGMI:

* LogisticRegression: one flat ``all_reduce`` of [loss | dW | db] per objective
  evaluation (~75 KB per model: latency-bound, so one bucket, never per tensor);
* RandomForest: per level, the (tree, node, feature, bin, class) histograms are
  summed with one ``all_reduce`` and every rank selects the same splits
  (``reduce_scatter`` by node owner + ``all_gather`` of the winners is the
  bandwidth-optimal variant for very large forests);
* MLP: fp32 gradient buckets (>= 64 KB, contiguous layer ranges of the flat buffer) all-reduced
  asynchronously while backward continues (``MLPEngine.train_step_overlapped``).

``gloo`` runs the identical code on CPU for the multi-process tests.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from ..ops import tree as T
from .dist import DistContext, shard_range


def allreduce_sum(ctx: Optional[DistContext]):
    if ctx is None or not ctx.is_distributed:
        return None

    def _ar(t: torch.Tensor):
        if t.is_cuda or ctx.backend != "nccl":
            dist.all_reduce(t, group=ctx.group)
        else:  # host tensor under RCCL: stage through the device
            d = t.to(ctx.device)
            dist.all_reduce(d, group=ctx.group)
            t.copy_(d.cpu())
    return _ar


def shard(X: torch.Tensor, y: torch.Tensor, ctx: DistContext):
    """This rank's contiguous row shard and its global row offset."""
    lo, hi = shard_range(X.shape[0], ctx.rank, ctx.world_size)
    return X[lo:hi], y[lo:hi], lo


def fit_logreg_dp(estimator, X_shard, y_shard, specs, num_classes, ctx: DistContext):
    return estimator.fit_many(X_shard, y_shard, specs, num_classes, allreduce=allreduce_sum(ctx))


def global_thresholds(X_shard: torch.Tensor, max_bins: int, ctx: DistContext, sample_rows: int = 10000,
                      seed: int = 0):
    """findSplits over a sample gathered from every rank (Spark samples the whole
    RDD); rank 0 computes, everybody receives the same thresholds."""
    Xh = X_shard.detach().float().cpu().numpy()
    if not ctx.is_distributed:
        return T.find_thresholds(Xh, max_bins, sample_rows, seed)
    per = max(1, sample_rows // ctx.world_size)
    rs = np.random.default_rng(seed + ctx.rank)
    take = Xh[np.sort(rs.choice(Xh.shape[0], size=min(per, Xh.shape[0]), replace=False))]
    parts = [None] * ctx.world_size
    dist.all_gather_object(parts, take, group=ctx.group)
    out = [None]
    if ctx.rank == 0:
        out[0] = T.find_thresholds(np.concatenate(parts, 0), max_bins, sample_rows, seed)
    dist.broadcast_object_list(out, src=0, group=ctx.group)
    return out[0]


def fit_forest_dp(estimator, X_shard, y_shard, num_classes: int, row_offset: int, ctx: DistContext):
    thr = global_thresholds(X_shard, estimator.maxBins, ctx, seed=estimator.seed)
    return estimator.fit_tensors(X_shard, y_shard, num_classes, allreduce=allreduce_sum(ctx), row_offset=row_offset,
                                 thresholds=thr)


def fit_mlp_dp(estimator, X_shard, y_shard, ctx: DistContext, num_classes: Optional[int] = None):
    return estimator.fit_tensors(X_shard, y_shard, process_group=ctx.group, rank=ctx.rank,
                                 world_size=ctx.world_size, num_classes=num_classes)
