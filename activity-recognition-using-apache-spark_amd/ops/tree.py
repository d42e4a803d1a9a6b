"""Tree-learning device ops.

* ``find_thresholds``  — per-feature candidate thresholds (Spark ``findSplits``):
  sorted distinct values -> midpoints when there are few, quantile cut points
  otherwise; at most ``max_bins - 1`` per feature.
* ``bin_features``     — fp32 -> uint8 bin ids, stored feature-major [F, N].
* ``hist_split``       — the level step: for every active (tree, node) build the
  weighted per-(feature, bin, class) histogram of its rows over its sampled
  features and pick the best (feature, bin) by impurity gain.  GPU: one fused
  HIP kernel (``har_tree_hist_split``) — an LDS-privatized histogram per
  (node, feature-chunk) workgroup, then a wave-parallel prefix scan over bins +
  gain + argmax, so histograms never touch HBM.  CPU: the same math with
  ``bincount`` (the oracle).
* ``forest_predict``   — traverse all trees for every row and accumulate the
  (normalized) leaf statistics; GPU: ``har_forest_predict``.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import _native, rng

GINI, ENTROPY = 0, 1
LDS_BUDGET = 96 * 1024  # bytes of LDS histogram per workgroup


def threshold_sample_weights(n_total: int, max_bins: int, sample_rows: int = 10000):
    """Bernoulli weights [keep, drop] of the findSplits row sample (None = every row).  Like
    Spark's ``findSplits`` (``input.sample(false, fraction)``, fraction = max(maxBins^2,
    10000) / N) the sample is a Bernoulli draw per row — here Philox keyed by (seed, global
    row id), so the sample is the same for any sharding of the rows."""
    if n_total <= sample_rows:
        return None
    frac = min(1.0, max(sample_rows, max_bins * max_bins) / float(n_total))
    return [frac, 1.0 - frac]


def threshold_sample_mask(N: int, max_bins: int, sample_rows: int = 10000, seed: int = 0, row_offset: int = 0,
                          n_total: int = None, device=None):
    """Rows [row_offset, row_offset + N) of an ``n_total``-row table kept by the findSplits
    sample: bool numpy [N] (device=None) or a device bool tensor (HIP Philox kernel)."""
    w = threshold_sample_weights(N if n_total is None else n_total, max_bins, sample_rows)
    if w is None:
        return None
    if device is not None and torch.device(device).type == "cuda":
        return rng.device_buckets(seed, rng.STREAM_FINDSPLITS, row_offset, N, w, device) == 0
    rows = np.arange(row_offset, row_offset + N, dtype=np.uint64)
    m = rng.assign_buckets(seed, rng.STREAM_FINDSPLITS, rows, w) == 0
    return m if device is None else torch.from_numpy(m).to(device)


class ThresholdTable:
    """Per-feature split thresholds as ONE padded matrix: ``mat`` [F, W] float32 (+inf after row f's
    ``counts[f]`` ascending thresholds).  Indexing / iteration give the per-feature arrays (the list
    form of ``find_thresholds``); the forest builder and the binning kernel take the matrix as is —
    no per-feature host loop, which at the reference's 3100 one-hot features cost milliseconds per
    fit."""

    def __init__(self, mat: np.ndarray, counts: np.ndarray):
        self.mat = np.ascontiguousarray(mat, dtype=np.float32)
        self.counts = np.asarray(counts, dtype=np.int64)

    @classmethod
    def from_any(cls, thresholds) -> "ThresholdTable":
        if isinstance(thresholds, ThresholdTable):
            return thresholds
        counts = np.array([len(t) for t in thresholds], dtype=np.int64)
        mat = np.full((len(counts), max(1, int(counts.max(initial=0)))), np.inf, dtype=np.float32)
        for f, t in enumerate(thresholds):
            mat[f, : len(t)] = t
        return cls(mat, counts)

    def __len__(self):
        return len(self.counts)

    def __getitem__(self, f):
        return self.mat[f, : self.counts[f]]

    def __iter__(self):
        return (self[f] for f in range(len(self)))

    def padded(self, width: int) -> np.ndarray:
        """[F, width] (+inf padding; width >= every count)."""
        out = np.full((len(self), width), np.inf, dtype=np.float32)
        w = min(width, self.mat.shape[1])
        out[:, :w] = self.mat[:, :w]
        return out


def find_thresholds(X: np.ndarray, max_bins: int, sample_rows: int = 10000, seed: int = 0, row_offset: int = 0,
                    n_total: int = None):
    """List of float32 threshold arrays (``x <= thr[b]`` goes left at split b).  NumPy
    oracle of ``find_thresholds_device``."""
    N, F = X.shape
    keep = threshold_sample_mask(N, max_bins, sample_rows, seed, row_offset, n_total)
    if keep is not None:
        X = X[keep]
    out = []
    n_splits = max_bins - 1
    for f in range(F):
        v = X[:, f]
        v = v[~np.isnan(v)]
        u, cnt = np.unique(v, return_counts=True)
        if len(u) <= 1:
            out.append(np.zeros(0, dtype=np.float32))
            continue
        if len(u) - 1 <= n_splits:
            thr = (u[:-1] + u[1:]) / 2.0
        else:
            # quantile cut points on the (weighted) distinct values
            cum = np.cumsum(cnt)
            total = cum[-1]
            targets = total * np.arange(1, n_splits + 1) / (n_splits + 1)
            idx = np.searchsorted(cum, targets, side="left")
            idx = np.unique(np.clip(idx, 0, len(u) - 2))
            thr = (u[idx] + u[idx + 1]) / 2.0
        out.append(thr.astype(np.float32))
    return out


def find_thresholds_device(X: torch.Tensor, max_bins: int, sample_rows: int = 10000, seed: int = 0,
                           row_offset: int = 0, n_total: int = None):
    """``find_thresholds`` on the tensor's device, threshold for threshold identical to the
    NumPy version (same Philox row sample, same fp32 midpoints, same fp64 quantile targets).

    The sampled rows are compacted (one size sync); one sort of their columns [F, n] puts
    NaN last, distinct values are the run starts, and the quantile target t of
    the host version (first distinct value whose cumulative count reaches t) is the distinct
    value at sorted position ceil(t) - 1.  Every feature's thresholds come back in ONE
    [F, max_bins - 1] device -> host copy."""
    N, F = X.shape
    Xs = X.float()
    keep_rows = threshold_sample_mask(N, max_bins, sample_rows, seed, row_offset, n_total, device=X.device)
    if keep_rows is not None:  # compact the ~10k sampled rows (one size sync) before the sort
        Xs = Xs[keep_rows]
    n = Xs.shape[0]
    ns = max_bins - 1
    if n == 0 or ns <= 0:
        return [np.zeros(0, dtype=np.float32) for _ in range(F)]
    if X.is_cuda and n <= 16384 and ns <= 63:
        # tree.hip: one LDS bitonic sort per feature column (NaN last), then find_splits_post_sort:
        # distinct ranks, quantile cut points, dedup — two kernels
        Xc = Xs.contiguous()
        s = torch.empty(F, n, dtype=torch.float32, device=X.device)
        _native.kernels().sort_columns(Xc.data_ptr(), n, F, F, s.data_ptr(), _native.stream_ptr())
        out = torch.empty(F, ns + 1, dtype=torch.float32, device=X.device)
        _native.kernels().find_splits_post_sort(s.data_ptr(), F, n, ns, out.data_ptr(), _native.stream_ptr())
        h = out.cpu().numpy()  # the one device -> host copy
        cnt = h[:, ns].astype(np.int64)
        return ThresholdTable(np.where(np.arange(ns)[None, :] < cnt[:, None], h[:, :ns], np.float32(np.inf)), cnt)
    s = torch.sort(Xs.t().contiguous(), dim=1).values  # [F, n], NaN sorted last
    nvalid = (~torch.isnan(s)).sum(1)  # [F]
    pos = torch.arange(n, device=X.device)
    valid = pos.view(1, n) < nvalid.view(F, 1)
    newd = torch.ones_like(valid)
    newd[:, 1:] = s[:, 1:] != s[:, :-1]
    newd &= valid
    drank = torch.cumsum(newd.to(torch.int64), 1) - 1  # distinct index of every sorted position
    ndist = newd.sum(1)  # [F]
    U = torch.zeros(F, n + 1, dtype=s.dtype, device=X.device)  # distinct values, compacted
    U.scatter_(1, torch.where(newd, drank, torch.full_like(drank, n)), s)
    k = torch.arange(ns, device=X.device)
    # few distinct values: every midpoint (j = 0 .. ndist - 2)
    few = (ndist - 1) <= ns
    # quantile cut points: t = total * (k + 1) / (ns + 1) (fp64, as in NumPy), j = distinct index
    # of sorted position ceil(t) - 1, clipped to [0, ndist - 2]
    t = nvalid.double().view(F, 1) * (k + 1).double().view(1, ns) / (ns + 1)
    q = (torch.ceil(t).to(torch.int64) - 1).clamp(0, n - 1)
    jq = torch.gather(drank, 1, q)
    jq = torch.minimum(jq, (ndist - 2).clamp_min(0).view(F, 1)).clamp_min(0)
    J = torch.where(few.view(F, 1), k.view(1, ns).expand(F, ns), jq)
    keep = torch.where(few.view(F, 1), k.view(1, ns) < (ndist - 1).view(F, 1),
                       torch.ones(F, ns, dtype=torch.bool, device=X.device))
    keep[:, 1:] &= few.view(F, 1) | (J[:, 1:] != J[:, :-1])  # np.unique of the (sorted) cut indices
    keep &= (ndist > 1).view(F, 1)
    thr = (torch.gather(U, 1, J) + torch.gather(U, 1, J + 1)) / 2.0
    packed = torch.cat([thr, keep.to(thr.dtype)], 1).cpu().numpy()  # the one device -> host copy
    thr_h, keep_h = packed[:, :ns], packed[:, ns:] > 0.5
    return [thr_h[f][keep_h[f]].astype(np.float32) for f in range(F)]


def thresholds_for(X: torch.Tensor, max_bins: int, sample_rows: int = 10000, seed: int = 0):
    """findSplits where the data lives: the device version for GPU tensors, NumPy otherwise."""
    if X.is_cuda:
        return find_thresholds_device(X.detach(), max_bins, sample_rows, seed)
    return find_thresholds(X.detach().float().cpu().numpy(), max_bins, sample_rows, seed)


def bin_features(X: np.ndarray, thresholds) -> np.ndarray:
    """uint8 bins, feature-major [F, N]: bin = #thresholds strictly below x."""
    N, F = X.shape
    bins = np.empty((F, N), dtype=np.uint8)
    for f in range(F):
        bins[f] = np.searchsorted(thresholds[f], X[:, f], side="left").astype(np.uint8)
    return bins


# ---------------------------------------------------------------------------------------------------
# One-hot-aware findSplits / binning / histograms for hybrid matrices (features.hybrid.HybridMatrix:
# the reference encoding — three one-hot blocks of 934 + 1401 + 755 binary columns beside 10 numeric
# ones, Main/main.py:51-66).  Spark grows its trees on these columns as categorical features of arity 2
# (the OneHotEncoder's attribute metadata: SURVEY.md N8, §3.4), so a one-hot column's only split is
# 0 | 1 — threshold 0.5 here, the midpoint find_thresholds takes for the two distinct values.  Nothing
# needs a sort for them: a column has its split iff the sampled rows hold both values (0 < ones < n).
# The forest is bit-identical to the dense path's (tests/test_gpu_tree_sparse.py).
SPARSE_TREES = os.environ.get("HAR_TREE_SPARSE", "1") != "0"
SPARSE_MAX_NCAT = 4  # tree.hip SP_NCAT


@dataclass
class SparseTreeInput:
    """What the one-hot-aware level kernels read beside the bins: the rows' one-hot entries and the
    one-hot column flags."""
    cat: torch.Tensor     # [N, ncat] int32 global column of each row's 1 per block (-1 none)
    onehot: torch.Tensor  # [F] uint8, 1 = one-hot column
    n_features: int


def sparse_args(sparse: Optional[SparseTreeInput]):
    if sparse is None:
        return (0, 0, 0)
    return (sparse.cat.data_ptr(), int(sparse.cat.shape[1]), sparse.onehot.data_ptr())


def hybrid_tree_ok(hm) -> bool:
    """A hybrid matrix the one-hot-aware tree path takes: on a GPU, 1..SPARSE_MAX_NCAT one-hot blocks."""
    return (SPARSE_TREES and hm is not None and hm.device.type == "cuda"
            and 0 < int(hm.cat.shape[1]) <= SPARSE_MAX_NCAT and hm.n_features <= 32767)


def find_thresholds_hybrid(hm, max_bins: int, sample_rows: int = 10000, seed: int = 0, row_offset: int = 0,
                           n_total: int = None) -> "ThresholdTable":
    """``find_thresholds`` of ``hm.to_dense()`` without densifying: the same Philox row sample, the
    device findSplits of the numeric block alone, and for every one-hot column the 0 | 1 split when
    the sampled rows hold both values (ones counted from the rows' one-hot entries)."""
    N, F = hm.n_rows, hm.n_features
    dev = hm.device
    ns = max_bins - 1
    keep = threshold_sample_mask(N, max_bins, sample_rows, seed, row_offset, n_total, device=dev)
    dense = hm.dense if keep is None else hm.dense[keep]
    cat = hm.cat if keep is None else hm.cat[keep]
    n = int(cat.shape[0])
    counts = np.zeros(F, dtype=np.int64)
    mat = np.full((F, max(1, ns)), np.inf, dtype=np.float32)
    if n == 0 or ns <= 0:
        return ThresholdTable(mat, counts)
    cv = cat.reshape(-1)
    ones = torch.bincount(cv[cv >= 0].long(), minlength=F)[:F]
    has = ((ones > 0) & (ones < n)).cpu().numpy()
    counts[has] = 1
    mat[has, 0] = np.float32(0.5)
    dcols = hm.dense_cols.cpu().numpy().astype(np.int64)
    if len(dcols):
        # the numeric block's findSplits on the rows already sampled (no second draw)
        td = ThresholdTable.from_any(find_thresholds_device(dense.contiguous(), max_bins, sample_rows=max(sample_rows, n),
                                                            seed=seed))
        w = td.mat.shape[1]
        counts[dcols] = td.counts
        mat[dcols, :min(w, mat.shape[1])] = td.mat[:, :mat.shape[1]]
    return ThresholdTable(mat, counts)


@dataclass
class DeviceThresholds:
    """findSplits' result kept on the device: ``thr_mat`` [F, W] fp32 (+inf padded) and ``nbins`` [F]
    int32 (thresholds + 1) — what the forest builder uploads from a ThresholdTable, without the host
    round trip."""
    thr_mat: torch.Tensor
    nbins: torch.Tensor

    def to_table(self) -> "ThresholdTable":
        cnt = (self.nbins.cpu().numpy() - 1).astype(np.int64)
        return ThresholdTable(self.thr_mat.cpu().numpy(), cnt)


def _hybrid_static(hm):
    """Per-matrix device constants of the one-hot-aware path (memoized on the immutable matrix): the
    int32 one-hot entries, the one-hot column flags and the column -> numeric index map."""
    memo = hm.__dict__.setdefault("_tree_static", {})
    if not memo:
        F = hm.n_features
        onehot = torch.zeros(F, dtype=torch.uint8, device=hm.device)
        for off, w in hm.blocks:
            onehot[off:off + w] = 1
        colmap = hm.col_map()[:F].contiguous()
        memo.update(cat=hm.cat.to(torch.int32).contiguous(), onehot=onehot, colmap=colmap,
                    dcols=hm.dense_cols.to(device=hm.device, dtype=torch.int32).contiguous(),
                    dense=hm.dense.float().contiguous())
    return memo


def thresholds_hybrid_device(hm, max_bins: int, sample_rows: int = 10000, seed: int = 0, row_offset: int = 0,
                             n_total: int = None) -> Optional[DeviceThresholds]:
    """``find_thresholds_hybrid`` left on the device (no host read unless the rows are sampled, whose
    compaction needs the sample size): the numeric block's LDS sort + post-sort kernels, then one
    kernel for the one-hot ones and one for the padded threshold matrix.  None when the shape needs
    the host version (sample > 16,384 rows, maxBins > 64)."""
    ns = max_bins - 1
    if ns <= 0 or ns > 63:
        return None
    st = _hybrid_static(hm)
    N, F = hm.n_rows, hm.n_features
    keep = threshold_sample_mask(N, max_bins, sample_rows, seed, row_offset, n_total, device=hm.device)
    dense, cat = (st["dense"], st["cat"]) if keep is None else (st["dense"][keep].contiguous(), st["cat"][keep].contiguous())
    n = int(cat.shape[0])
    if n == 0 or n > 16384:
        return None
    mod, stp = _native.kernels(), _native.stream_ptr()
    Fd = int(dense.shape[1])
    dthr = torch.empty(max(Fd, 1), ns + 1, dtype=torch.float32, device=hm.device)
    if Fd:
        srt = torch.empty(Fd, n, dtype=torch.float32, device=hm.device)
        mod.sort_columns(dense.data_ptr(), n, Fd, Fd, srt.data_ptr(), stp)
        mod.find_splits_post_sort(srt.data_ptr(), Fd, n, ns, dthr.data_ptr(), stp)
    ones = torch.empty(F, dtype=torch.int32, device=hm.device)
    thr_mat = torch.empty(F, max_bins, dtype=torch.float32, device=hm.device)
    nbins = torch.empty(F, dtype=torch.int32, device=hm.device)
    mod.tree_thresholds_hybrid(cat.data_ptr(), n, int(cat.shape[1]), F, st["colmap"].data_ptr(), dthr.data_ptr(), ns,
                               max_bins, ones.data_ptr(), thr_mat.data_ptr(), nbins.data_ptr(), stp)
    return DeviceThresholds(thr_mat, nbins)


def bins_hybrid(hm, thr_mat: torch.Tensor, nbins: torch.Tensor) -> torch.Tensor:
    """uint8 bins [F, N] of ``hm`` (= bin_features of its dense form) from its parts (tree.hip)."""
    N, F = hm.n_rows, hm.n_features
    out = torch.empty(F, N, dtype=torch.uint8, device=hm.device)
    st = _hybrid_static(hm)
    dense, cat, dcols = st["dense"], st["cat"], st["dcols"]
    _native.kernels().tree_bins_hybrid(dense.data_ptr(), N, int(dense.shape[1]), dcols.data_ptr(), cat.data_ptr(),
                                       int(cat.shape[1]), F, thr_mat.data_ptr(), int(thr_mat.shape[1]),
                                       nbins.data_ptr(), out.data_ptr(), _native.stream_ptr())
    return out


def sparse_tree_input(hm) -> SparseTreeInput:
    st = _hybrid_static(hm)
    return SparseTreeInput(st["cat"], st["onehot"], hm.n_features)


# rows per work item of a one-hot-aware level: a node's row pass is a few loads per row, so a node is
# chunked (and its chunks merged + searched in a second pass) only when far bigger than PLAN_ROWS
SPARSE_PLAN_ROWS = 16384  # 8 x PLAN_ROWS


@dataclass
class LevelResult:
    gain: torch.Tensor      # [A] best gain (-inf if no valid split)
    feat: torch.Tensor      # [A] best global feature id
    bin: torch.Tensor       # [A] best bin (rows with bin <= b go left)
    left: torch.Tensor      # [A, K] weighted class counts of the left child
    total: torch.Tensor     # [A, K] weighted class counts of the node


def _impurity(c: torch.Tensor, w: torch.Tensor, kind: int) -> torch.Tensor:
    p = c / w.clamp_min(1e-30).unsqueeze(-1)
    if kind == GINI:
        return 1.0 - (p * p).sum(-1)
    lp = torch.where(p > 0, torch.log2(p.clamp_min(1e-30)), torch.zeros_like(p))
    return -(p * lp).sum(-1)


def level_histogram(bins, label, rows, row_w, key, n_nodes, feats, K, max_bins) -> torch.Tensor:
    """Weighted histograms [A, m, max_bins, K] of the (row, weight, node) pairs over each
    node's sampled features ``feats`` [A, m] (torch; any device).  fp64 accumulation."""
    A, m = feats.shape
    dev = bins.device
    hist = torch.zeros(A * m * max_bins * K, dtype=torch.float64, device=dev)
    P = rows.shape[0]
    step = max(1, (1 << 24) // max(m, 1))  # bound the [P, m] temporaries
    for p0 in range(0, P, step):
        r = rows[p0:p0 + step].long()
        kk = key[p0:p0 + step].long()
        fe = feats[kk].long()                                    # [p, m]
        bv = bins[fe, r.unsqueeze(1)].long()                     # [p, m]
        y = label[r].long()
        idx = ((kk.unsqueeze(1) * m + torch.arange(m, device=dev)) * max_bins + bv) * K + y.unsqueeze(1)
        w = row_w[p0:p0 + step].double().unsqueeze(1).expand(-1, m)
        hist.index_add_(0, idx.reshape(-1), w.reshape(-1))
    return hist.view(A, m, max_bins, K)


def hist_split_torch(bins, nbins_feat, label, rows, row_w, key, n_nodes, feats, K, max_bins, min_instances,
                     min_info_gain, impurity) -> LevelResult:
    """CPU/oracle implementation of ``hist_split_native``."""
    hist = level_histogram(bins, label, rows, row_w, key, n_nodes, feats, K, max_bins)
    return split_from_hist(hist, feats, nbins_feat, min_instances, min_info_gain, impurity)


def split_from_hist(hist, feats, nbins_feat, min_instances, min_info_gain, impurity) -> LevelResult:
    A, m, nb, K = hist.shape
    left = hist.cumsum(dim=2)                        # bins <= b go left
    total = left[:, 0, -1, :]                        # [A, K]
    right = total[:, None, None, :] - left
    wl, wr = left.sum(-1), right.sum(-1)
    wt = total.sum(-1)
    imp_p = _impurity(total, wt, impurity)
    gain = imp_p[:, None, None] - (wl / wt.clamp_min(1e-30)[:, None, None]) * _impurity(left, wl, impurity) \
        - (wr / wt.clamp_min(1e-30)[:, None, None]) * _impurity(right, wr, impurity)
    nbf = nbins_feat[feats.long()].long()            # [A, m]
    valid = torch.arange(nb, device=hist.device)[None, None, :] < (nbf - 1)[:, :, None]
    valid &= (wl >= min_instances) & (wr >= min_instances)
    gain = torch.where(valid, gain, torch.full_like(gain, -float("inf")))
    flat = gain.reshape(A, -1)
    best = torch.argmax(flat, dim=1)
    bg = flat.gather(1, best[:, None]).squeeze(1)
    slot, b = best // nb, best % nb
    bf = feats.long().gather(1, slot[:, None]).squeeze(1)
    bl = left[torch.arange(A, device=hist.device), slot, b]
    ok = torch.isfinite(bg) & (bg >= min_info_gain)
    bg = torch.where(ok, bg, torch.full_like(bg, -float("inf")))
    return LevelResult(gain=bg.float(), feat=bf.int(), bin=b.int(), left=bl.float(), total=total.float())


def pack_level(res: LevelResult) -> torch.Tensor:
    """[A, 3 + 2K] fp32 rows (gain, feature, bin, left, total) — feature/bin ids are exact
    in fp32 (< 2^24); one tensor so the winners travel in ONE all-gather."""
    return torch.cat([res.gain[:, None].float(), res.feat[:, None].float(), res.bin[:, None].float(),
                      res.left.float(), res.total.float()], 1)


def unpack_level(t: torch.Tensor, K: int) -> LevelResult:
    return LevelResult(gain=t[:, 0].contiguous(), feat=t[:, 1].to(torch.int32), bin=t[:, 2].to(torch.int32),
                       left=t[:, 3:3 + K].contiguous(), total=t[:, 3 + K:3 + 2 * K].contiguous())


def split_owner(hist: torch.Tensor, feats: torch.Tensor, K: int, owner, split_fn) -> LevelResult:
    """Owner-computes split search (data parallel): ``owner.reduce_scatter``
    sums the per-node histograms across ranks and leaves each rank the node slice
    ``[a0, a1)`` it owns; the rank searches splits for those nodes only
    (``split_fn(local_hist, a0, a1)``) and ``owner.all_gather`` gives every rank all the
    winners.  Traffic per rank: (P-1)/P x histogram + a few bytes per node, vs.
    2 (P-1)/P x histogram for the all-reduce variant, and the split search is not
    repeated on every rank.  Spark's equivalent is ``reduceByKey(node)`` followed by
    ``collectAsMap`` (``Main/main.py:300,481``)."""
    A = hist.shape[0]
    local, a0, a1 = owner.reduce_scatter(hist)
    if a1 > a0:
        packed = pack_level(split_fn(local[: a1 - a0], a0, a1))
    else:
        packed = torch.zeros(0, 3 + 2 * K, dtype=torch.float32, device=hist.device)
    return unpack_level(owner.all_gather(packed, A), K)


def hist_split_native(bins, nbins_feat, label, rows, row_w, node_start, node_count, feats, K, max_bins,
                      min_instances, min_info_gain, impurity, allreduce=None, owner=None, max_rows=None,
                      check_labels: bool = True, bins_rm=None, sparse=None) -> LevelResult:
    """Fused LDS histogram + split on one device; in data parallel the kernel runs twice:
    histogram-only into a [A, m, bins, K] buffer, then either one RCCL all-reduce of it and
    split search for every node (``allreduce``), or a reduce-scatter by node owner, split
    search for the owned nodes and an all-gather of the winners (``owner``)."""
    A, m = feats.shape
    F, N = bins.shape
    fc = max(1, min(m, LDS_BUDGET // (max_bins * K * 4)))
    chunks = (m + fc - 1) // fc
    dev = bins.device
    gain = torch.empty(A * chunks, dtype=torch.float32, device=dev)
    feat = torch.empty(A * chunks, dtype=torch.int32, device=dev)
    bin_ = torch.empty(A * chunks, dtype=torch.int32, device=dev)
    left = torch.empty(A * chunks, K, dtype=torch.float32, device=dev)
    total = torch.empty(A, K, dtype=torch.float32, device=dev)
    # (host syncs) the forest builder checks the labels once per fit and passes a row-count hint
    if check_labels and label.numel() and (int(label.max()) >= K or int(label.min()) < 0):
        raise ValueError("labels out of range")
    mod = _native.kernels()
    # bins_rm: optional row-major [N, F] copy of the bins (one row's features in one or two lines)
    bptr, row_major = (bins_rm.data_ptr(), 1) if bins_rm is not None else (bins.data_ptr(), 0)
    args = [bptr, N, F, row_major, nbins_feat.data_ptr(), rows.data_ptr(), row_w.data_ptr(), node_start.data_ptr(),
            node_count.data_ptr(), A, feats.data_ptr(), m, fc, label.data_ptr(), K, max_bins, float(min_instances),
            float(min_info_gain), impurity, gain.data_ptr(), feat.data_ptr(), bin_.data_ptr(), left.data_ptr(),
            total.data_ptr()]
    # few large nodes (the top levels): split every node's rows over several workgroups so the
    # launch still fills 256 CUs; their LDS histograms merge into a global one
    blocks = A * chunks
    if max_rows is None:
        max_rows = int(node_count.max()) if A else 0
    row_chunks = 1
    if blocks < 1024 and max_rows > 4096:
        row_chunks = int(min((1024 + blocks - 1) // blocks, (max_rows + 2047) // 2048))
    st = _native.stream_ptr()
    sp = sparse_args(sparse)
    if owner is not None:
        ghist = (torch.zeros if row_chunks > 1 else torch.empty)(A, m, max_bins, K, dtype=torch.float32, device=dev)
        mod.tree_hist_split(*args, 1, ghist.data_ptr(), row_chunks, *sp, st)

        def split_slice(local, a0, a1):
            n = a1 - a0
            g = torch.empty(n * chunks, dtype=torch.float32, device=dev)
            f = torch.empty(n * chunks, dtype=torch.int32, device=dev)
            b = torch.empty(n * chunks, dtype=torch.int32, device=dev)
            lf = torch.empty(n * chunks, K, dtype=torch.float32, device=dev)
            tot = torch.empty(n, K, dtype=torch.float32, device=dev)
            loc = local.contiguous()
            sl = [bptr, N, F, row_major, nbins_feat.data_ptr(), rows.data_ptr(), row_w.data_ptr(),
                  node_start.data_ptr() + 4 * a0, node_count.data_ptr() + 4 * a0, n, feats.data_ptr() + 4 * a0 * m,
                  m, fc, label.data_ptr(), K, max_bins, float(min_instances), float(min_info_gain), impurity,
                  g.data_ptr(), f.data_ptr(), b.data_ptr(), lf.data_ptr(), tot.data_ptr()]
            mod.tree_hist_split(*sl, 2, loc.data_ptr(), 1, *sp, st)
            return _best_chunk(g, f, b, lf, tot, n, chunks, K)

        return split_owner(ghist, feats, K, owner, split_slice)
    if allreduce is None and row_chunks == 1:
        mod.tree_hist_split(*args, 0, 0, 1, *sp, st)
    else:
        ghist = (torch.zeros if row_chunks > 1 else torch.empty)(A, m, max_bins, K, dtype=torch.float32, device=dev)
        mod.tree_hist_split(*args, 1, ghist.data_ptr(), row_chunks, *sp, st)
        if allreduce is not None:
            allreduce(ghist)
        mod.tree_hist_split(*args, 2, ghist.data_ptr(), 1, *sp, st)
    return _best_chunk(gain, feat, bin_, left, total, A, chunks, K)


PLAN_ROWS = 2048  # rows per work item of a load-balanced level (larger nodes are chunked)


def hist_split_planned(bins, nbins_feat, label, rows, row_w, node_start, node_count, feats, K, max_bins,
                       min_instances, min_info_gain, impurity, rows_bound: int, bins_rm=None,
                       prows: int = PLAN_ROWS, a_dev: int = 0, store=None, hprev=None, derive_from=None,
                       parent_of=None, sparse=None) -> LevelResult:
    """Load-balanced fused histogram + split for one level on one device (no host sync).

    Work is split by ROWS, not by node: a node of <= ``prows`` rows is one work item (fused LDS
    histogram + split, as ``hist_split_native``); a bigger node becomes ceil(rows / prows) chunk
    items whose LDS histograms are added into the node's merged slot (integer-valued weights:
    exact in any order), followed by one split-search pass over the merged big nodes.  Without it a
    level's time is its largest node's: the deep levels of a forest keep a few nodes of tens of
    thousands of rows beside thousands of small ones.  ``rows_bound`` bounds the level's total
    rows (grid sizes are upper bounds; surplus workgroups exit on the device-side counts).
    ``a_dev`` (a device pointer, 0 = none) holds the level's real node count; ``feats.shape[0]``
    is then only a bound, so the level needs no host-known node count at all.

    Sibling subtraction: with ``store`` (a [A, m, max_bins, K] fp32 buffer) every node's histogram
    is kept there for the next level; with ``derive_from`` / ``parent_of`` (the previous level's
    frontier output) and ``hprev`` (the previous level's store) the nodes marked
    ``derive_from[a] >= 0`` — the heavier of two candidate siblings, whose rows the grouping skipped —
    take parent - sibling instead of a pass over their rows (exact: integer-valued weights)."""
    A, m = feats.shape
    F, N = bins.shape
    fc = max(1, min(m, LDS_BUDGET // (max_bins * K * 4)))
    chunks = (m + fc - 1) // fc
    dev = bins.device
    gain = torch.empty(A * chunks, dtype=torch.float32, device=dev)
    feat = torch.empty(A * chunks, dtype=torch.int32, device=dev)
    bin_ = torch.empty(A * chunks, dtype=torch.int32, device=dev)
    left = torch.empty(A * chunks, K, dtype=torch.float32, device=dev)
    total = torch.empty(A, K, dtype=torch.float32, device=dev)
    items_ub = A + rows_bound // prows
    max_big = max(1, min(A, rows_bound // (prows + 1)))
    plan = torch.empty(4 + (A + 1) + 3 * A + items_ub, dtype=torch.int32, device=dev)
    slot = m * max_bins * K
    by_node = store is not None
    ghist = store if by_node else torch.empty(max_big * slot, dtype=torch.float32, device=dev)
    mod, st = _native.kernels(), _native.stream_ptr()
    mod.tree_plan(node_count.data_ptr(), A, prows, plan.data_ptr(), slot, ghist.data_ptr(), max_big, int(by_node),
                  a_dev, st)
    bptr, row_major = (bins_rm.data_ptr(), 1) if bins_rm is not None else (bins.data_ptr(), 0)
    args = [bptr, N, F, row_major, nbins_feat.data_ptr(), rows.data_ptr(), row_w.data_ptr(), node_start.data_ptr(),
            node_count.data_ptr(), A, feats.data_ptr(), m, fc, label.data_ptr(), K, max_bins, float(min_instances),
            float(min_info_gain), impurity, gain.data_ptr(), feat.data_ptr(), bin_.data_ptr(), left.data_ptr(),
            total.data_ptr()]
    dptr = derive_from.data_ptr() if derive_from is not None else 0
    sp = sparse_args(sparse)
    mod.tree_hist_split_planned(*args, 3, ghist.data_ptr(), plan.data_ptr(), prows, items_ub, int(by_node), 0, dptr,
                                0, *sp, st)
    mod.tree_hist_split_planned(*args, 4, ghist.data_ptr(), plan.data_ptr(), prows, max_big, int(by_node), 0, 0, 0,
                                *sp, st)
    if derive_from is not None:
        mod.tree_hist_split_planned(*args, 5, ghist.data_ptr(), plan.data_ptr(), prows, A, 1, hprev.data_ptr(), dptr,
                                    parent_of.data_ptr(), *sp, st)
    return _best_chunk(gain, feat, bin_, left, total, A, chunks, K)


# integer-valued histogram counts up to this are exact in fp16 (DP wire format of small levels)
FP16_EXACT_MAX = 2048.0


# DP wire format of the per-node histograms (HAR_TREE_DP_WIRE): "packed" = present classes only, each
# count in an 8 / 16 / 32-bit field of int32 words by its node's total weight (tree_dp.hip); "fp16" =
# the dense store, fp16 when every count is < 2048, else fp32
DP_WIRE = os.environ.get("HAR_TREE_DP_WIRE", "packed")


def dp_wire_plan(node_cc: torch.Tensor, mb: int, P: int):
    """The packed wire layout of one DP level from the candidates' GLOBAL class counts ``node_cc``
    [A, K] (identical on every rank): per node the present classes ``cls`` [A, K] (ascending, first
    ``kp`` valid), the field width ``bw`` in bytes (1 / 2 / 4: the node's total weight < 2^8 / 2^16 /
    else) and its words; nodes go to owner ranks in contiguous word-balanced ranges.  Returns
    (cls, kp, bw, woff, bounds, wmax): ``woff`` [A] int64 = the node's word offset in the [P, wmax]
    send buffer, ``bounds`` (host list, P + 1) = rank r owns nodes bounds[r] .. bounds[r + 1] - 1.
    One small device -> host read (the bounds and the widest rank's words)."""
    A, K = node_cc.shape
    dev = node_cc.device
    present = node_cc > 0
    kp = present.sum(1).to(torch.int32)
    w = node_cc.sum(1)
    bw = torch.where(w < 256, 1, torch.where(w < 65536, 2, 4)).to(torch.int32)
    per = (4 // bw).long()
    words = (mb * kp.long() + per - 1) // per
    ar = torch.arange(K, device=dev)
    cls = (torch.sort(torch.where(present, ar, ar + K), dim=1).values % K).to(torch.int32).contiguous()
    incl = torch.cumsum(words, 0)
    excl = incl - words
    total = incl[-1:].clamp_min(1)
    own = torch.minimum(excl * P // total, torch.tensor(P - 1, device=dev))
    bounds_d = torch.searchsorted(own, torch.arange(P + 1, device=dev))
    bounds_d[-1] = A
    start = torch.cat([excl, incl[-1:]])[bounds_d]          # first word of each rank's range
    seg = start[1:] - start[:-1]
    hdr = torch.cat([bounds_d, seg]).cpu().tolist()
    bounds, wmax = [int(v) for v in hdr[:P + 1]], max(1, max(int(v) for v in hdr[P + 1:]))
    woff = (own * wmax + excl - start[own]).contiguous()
    return cls, kp, bw, woff, bounds, wmax


def hist_split_planned_dp(bins, nbins_feat, label, rows, row_w, node_start, node_count, feats, K, max_bins,
                          min_instances, min_info_gain, impurity, rows_bound: int, a_dev: int, allreduce=None,
                          owner=None, bins_rm=None, prows: int = PLAN_ROWS, max_weight: float = -1.0,
                          node_cc: Optional[torch.Tensor] = None, sparse=None) -> LevelResult:
    """The data-parallel level on the planned path.  ``feats.shape[0]`` = A is the level's node count:
    EXACT when ``a_dev`` is 0 (the level loop read its 16-byte count record back), else a bound shared
    by every rank with ``a_dev`` pointing at the device count.

    1. the row-balanced work items of ``hist_split_planned`` write this rank's per-node histograms
       into the store [A, m, bins, K] (kernel mode 6: a node of one work item stores its slot, the
       chunks of a big node add into their slot, zeroed by the plan — no fill of the whole store);
    2. the store is summed across ranks — ``allreduce`` (every rank then searches every node) or
       ``owner.reduce_scatter_store`` (rank r receives the summed slice of nodes [a0, a1)), straight
       from the store (allocated with the owner padding; no staging copy on RCCL).  With the exact
       count every collective carries real nodes only, and when ``max_weight`` (the largest candidate
       node's weight, known with the count) is <= 2048 the counts travel as fp16 — integer-valued
       (bootstrap x fold weights), so exact — halving the wire bytes again;
    3. split search from the (slice of the) reduced store (mode 7);
    4. owner: the slice's winners, packed [n, 3 + 2K] (``pack_level``), travel in ONE all-gather.

    With ``node_cc`` (the candidates' global class counts, exact level, integer weights) the owner
    reduction ships the PACKED wire format instead (``dp_wire_plan`` / tree_dp.hip): present classes
    only, 8 / 16 / 32-bit integer fields by node weight, one int32 reduce-scatter of word-balanced
    rank rows; the owner unpacks its summed row into the fp32 store the split kernel reads."""
    A, m = feats.shape
    F, N = bins.shape
    fc = max(1, min(m, LDS_BUDGET // (max_bins * K * 4)))
    chunks = (m + fc - 1) // fc
    dev = bins.device
    exact = a_dev == 0
    items_ub = A + rows_bound // prows
    plan = torch.empty(4 + (A + 1) + 3 * A + items_ub, dtype=torch.int32, device=dev)
    slot = m * max_bins * K
    P = owner.ctx.world_size if owner is not None else 1
    S = max(1, -(-A // P))
    if exact:  # every slot is written by its node's items: no zero fill (owner padding never read)
        store = torch.empty((P * S if owner is not None else A) * slot, dtype=torch.float32, device=dev)
    else:      # bound: the surplus slots past the device count must sum to zero
        store = torch.zeros(A * slot, dtype=torch.float32, device=dev)
    mod, st = _native.kernels(), _native.stream_ptr()
    mod.tree_plan(node_count.data_ptr(), A, prows, plan.data_ptr(), slot, store.data_ptr(), max(1, A), 1, a_dev, st)
    bptr, row_major = (bins_rm.data_ptr(), 1) if bins_rm is not None else (bins.data_ptr(), 0)
    sp = sparse_args(sparse)

    def launch(mode, n, a0, hist_ptr, fptr, outs, bound):
        g, f, b, lf, tot = outs
        mod.tree_hist_split_planned(bptr, N, F, row_major, nbins_feat.data_ptr(), rows.data_ptr(), row_w.data_ptr(),
                                    node_start.data_ptr(), node_count.data_ptr(), n, fptr, m, fc, label.data_ptr(),
                                    K, max_bins, float(min_instances), float(min_info_gain), impurity, g.data_ptr(),
                                    f.data_ptr(), b.data_ptr(), lf.data_ptr(), tot.data_ptr(), mode, hist_ptr,
                                    plan.data_ptr(), a0 if mode == 7 else prows, bound, 1, 0, 0, 0, *sp, st)

    def outs(n):
        return (torch.empty(n * chunks, dtype=torch.float32, device=dev),
                torch.empty(n * chunks, dtype=torch.int32, device=dev),
                torch.empty(n * chunks, dtype=torch.int32, device=dev),
                torch.empty(n * chunks, K, dtype=torch.float32, device=dev),
                torch.empty(n, K, dtype=torch.float32, device=dev))

    full = outs(A)
    launch(6, A, 0, store.data_ptr(), feats.data_ptr(), full, items_ub)
    narrow = exact and 0 <= max_weight <= FP16_EXACT_MAX
    if owner is None:
        if allreduce is not None:
            if narrow:
                h = store.to(torch.float16)
                allreduce(h)
                store.copy_(h)
            else:
                allreduce(store)
        launch(7, A, 0, store.data_ptr(), feats.data_ptr(), full, A)
        return _best_chunk(*full, A, chunks, K)
    if exact and node_cc is not None and DP_WIRE == "packed" and P > 1:
        mb = m * max_bins
        cls, kp, bw, woff, bounds, wmax = dp_wire_plan(node_cc[:A].contiguous(), mb, P)
        send = owner.words_buffer(P * wmax, dev)
        mod.tree_dp_pack(store.data_ptr(), A, slot, mb, K, cls.data_ptr(), kp.data_ptr(), bw.data_ptr(),
                         woff.data_ptr(), send.data_ptr(), st)
        recv = owner.reduce_scatter_words(send, wmax, dev)
        r = owner.ctx.rank
        a0, a1 = bounds[r], bounds[r + 1]
        n = a1 - a0
        if n > 0:
            loc = torch.empty(n * slot, dtype=torch.float32, device=dev)
            mod.tree_dp_unpack(recv.data_ptr(), a0, n, slot, mb, K, cls.data_ptr(), kp.data_ptr(), bw.data_ptr(),
                               woff.data_ptr(), r * wmax, loc.data_ptr(), st)
            part = outs(n)
            launch(7, n, a0, loc.data_ptr(), feats.data_ptr() + 4 * a0 * m, part, n)
            packed = pack_level(_best_chunk(*part, n, chunks, K))
        else:
            packed = torch.zeros(0, 3 + 2 * K, dtype=torch.float32, device=dev)
        return unpack_level(owner.all_gather_ranges(packed, bounds), K)
    if exact:
        local, a0, a1 = owner.reduce_scatter_store(store.view(P * S, slot), A, narrow)
    else:
        local, a0, a1 = owner.reduce_scatter(store.view(A, slot))
    n = a1 - a0
    if n > 0:
        loc = local[:n].contiguous()
        part = outs(n)
        launch(7, n, a0, loc.data_ptr(), feats.data_ptr() + 4 * a0 * m, part, n)
        packed = pack_level(_best_chunk(*part, n, chunks, K))
    else:
        packed = torch.zeros(0, 3 + 2 * K, dtype=torch.float32, device=dev)
    return unpack_level(owner.all_gather(packed, A), K)


def _best_chunk(gain, feat, bin_, left, total, A, chunks, K) -> LevelResult:
    if chunks == 1:  # every sampled feature in one workgroup: the kernel's winner is the node's
        return LevelResult(gain=gain, feat=feat, bin=bin_, left=left.view(A, K), total=total)
    gain, feat, bin_, left = gain.view(A, chunks), feat.view(A, chunks), bin_.view(A, chunks), left.view(A, chunks, K)
    best = torch.argmax(gain, dim=1)  # first max -> lowest chunk (lowest feature slot) on ties
    ar = torch.arange(A, device=gain.device)
    return LevelResult(gain=gain[ar, best], feat=feat[ar, best], bin=bin_[ar, best], left=left[ar, best],
                       total=total)


def forest_predict_torch(X, feature, threshold, left, right, leaf_stats, max_depth, normalize=True):
    """X [N, F]; trees SoA [T, maxNodes]; returns summed (normalized) leaf stats [N, K]."""
    T = feature.shape[0]
    N = X.shape[0]
    node = torch.zeros(T, N, dtype=torch.long, device=X.device)
    tix = torch.arange(T, device=X.device)[:, None].expand(T, N)
    for _ in range(max_depth + 1):
        f = feature[tix, node].long()
        is_leaf = f < 0
        xv = X[torch.arange(N, device=X.device)[None, :].expand(T, N), f.clamp_min(0)]
        go_left = xv <= threshold[tix, node]
        nxt = torch.where(go_left, left[tix, node], right[tix, node]).long()
        node = torch.where(is_leaf, node, nxt)
    st = leaf_stats[tix, node]                      # [T, N, K]
    if normalize:
        st = st / st.sum(-1, keepdim=True).clamp_min(1e-30)
    return st.sum(0)


def forest_predict_native(X, feature, threshold, left, right, leaf_stats, max_depth, normalize=True):
    T, maxn = feature.shape
    N, F = X.shape
    K = leaf_stats.shape[-1]
    out = torch.zeros(N, K, dtype=torch.float32, device=X.device)
    _native.kernels().forest_predict(X.contiguous().data_ptr(), N, F, X.stride(0), feature.data_ptr(),
                                     threshold.data_ptr(), left.data_ptr(), right.data_ptr(), leaf_stats.data_ptr(),
                                     T, maxn, K, max_depth, int(normalize), out.data_ptr(), _native.stream_ptr())
    return out
