"""DecisionTreeClassifier / RandomForestClassifier — level-wise forest builder.

Reference: ``DecisionTreeClassifier(maxDepth=3)`` (``Main/main.py:297``) and
``RandomForestClassifier(numTrees=100, maxDepth=4, maxBins=32)`` (``Main/main.py:478``);
Spark ``RandomForest.run`` semantics:

* ``findSplits``: at most ``maxBins - 1`` thresholds per feature (midpoints of the
  distinct values, or quantile cut points); a binary one-hot feature gets the
  single split 0 | 1, which is Spark's 2-category split;
* bagging: RandomForest with ``numTrees > 1`` draws Poisson(subsamplingRate) per (tree, row)
  (with replacement), a single tree Bernoulli(subsamplingRate) (without; every row once at 1);
* ``featureSubsetStrategy``: ``auto`` = ``sqrt`` for a forest, ``all`` for one
  tree; the subset is re-drawn at every node;
* impurity gini (or entropy); a node splits only when its best gain is > 0 and
  >= ``minInfoGain`` and both children have >= ``minInstancesPerNode`` weight;
* prediction: a tree's ``rawPrediction`` is its leaf's class counts; a forest
  sums each tree's *normalized* leaf distribution (soft vote,
  ``result.txt:282-286``); probability = normalized raw.

Engine: every tree of the forest grows in lock step, one level at a time.  Per
level the rows of all active (tree, node) pairs are grouped on the device, one
fused HIP kernel builds the LDS histograms and picks every node's best split
(``har_tree_hist_split``), and a vectorized partition step moves rows to the
children.  Bootstrap weights are Philox(seed, tree, global row) so forests are
identical for any sharding.  In data-parallel mode (``parallel.data_parallel``:
``fit_forest_dp`` / ``NodeOwner``) the per-rank histograms are reduce-scattered by node
owner (packed integer wire format) or all-reduced before split selection;
``fit_forest_tree_parallel`` grows disjoint tree slices per rank instead.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from ..data.table import Table
from ..ops import _native, rng
from ..ops import tree as T
from .base import ClassificationModel, ClassifierParams, Estimator, dp_allreduce, dp_context, dp_owner, dp_rows, \
    features_tensor, labels_tensor, new_uid, num_label_classes, resolve_device


@dataclass
class ForestArrays:
    feature: torch.Tensor    # [T, maxn] int32, -1 = leaf
    threshold: torch.Tensor  # [T, maxn] float32 (x <= thr goes left)
    left: torch.Tensor       # [T, maxn] int32
    right: torch.Tensor      # [T, maxn] int32
    stats: torch.Tensor      # [T, maxn, K] float32 weighted class counts
    n_nodes: np.ndarray      # [T] nodes per tree
    max_depth: int
    gain: Optional[torch.Tensor] = None  # [T, maxn] split gains (feature importances)

    def to(self, device):
        return ForestArrays(self.feature.to(device), self.threshold.to(device), self.left.to(device),
                            self.right.to(device), self.stats.to(device), self.n_nodes, self.max_depth,
                            None if self.gain is None else self.gain.to(device))


def subset_size(strategy, n_features: int, num_trees: int) -> int:
    s = str(strategy).lower()
    if s == "auto":
        s = "all" if num_trees == 1 else "sqrt"
    if s == "all":
        return n_features
    if s == "sqrt":
        return int(math.ceil(math.sqrt(n_features)))
    if s == "log2":
        return max(1, int(math.ceil(math.log2(n_features))))
    if s == "onethird":
        return max(1, int(math.ceil(n_features / 3.0)))
    v = float(s)
    if v >= 1.0 and v == int(v):
        return min(n_features, int(v))
    return max(1, int(math.ceil(v * n_features)))


class ForestBuilder:
    """Builds ``num_trees`` trees level-synchronously on one device (or one DP rank)."""

    def __init__(self, num_classes: int, num_trees: int = 1, max_depth: int = 5, max_bins: int = 32,
                 min_instances: int = 1, min_info_gain: float = 0.0, impurity: str = "gini",
                 feature_subset: str = "auto", bootstrap: Optional[bool] = None, seed: int = 0,
                 allreduce=None, tree_offset: int = 0, owner=None, subsample: float = 1.0):
        if max_bins > 64:
            raise ValueError("maxBins <= 64 (one lane per bin in the split kernel)")
        self.K, self.T, self.D = num_classes, num_trees, max_depth
        self.max_bins, self.min_inst, self.min_gain = max_bins, float(min_instances), float(min_info_gain)
        self.impurity = T.GINI if impurity == "gini" else T.ENTROPY
        self.subset = feature_subset
        self.bootstrap = (num_trees > 1) if bootstrap is None else bootstrap
        if not 0.0 < subsample <= 1.0:
            raise ValueError("subsamplingRate must be in (0, 1]")
        self.subsample = float(subsample)
        # Spark BaggedPoint: with replacement (a forest) Poisson(rate) counts, without replacement
        # (one tree) Bernoulli(rate) at rate < 1, else every row once
        if self.bootstrap:
            self.cdf = rng.poisson_thresholds(self.subsample)
        elif self.subsample < 1.0:
            self.cdf = rng.bernoulli_thresholds(self.subsample)
        else:
            self.cdf = None
        self.seed = seed
        self.allreduce = allreduce  # optional callable(tensor) -> None (DP histogram reduction)
        self.tree_offset = tree_offset  # global id of tree 0 (bootstrap / feature-subset streams)
        # optional owner-computes communicator (reduce_scatter / all_gather / allreduce); when
        # given, level histograms are reduce-scattered by node owner instead of all-reduced
        self.owner = owner
        if owner is not None and allreduce is None:
            self.allreduce = owner.allreduce

    def prepare(self, X: torch.Tensor, thresholds=None, hybrid=None):
        from ..ops.stats import bin_features

        self.sparse = None
        if (hybrid is not None and X.is_cuda and T.hybrid_tree_ok(hybrid) and hybrid.n_rows == X.shape[0]
                and self.max_bins <= 32):
            # one-hot-aware path (ops/tree.py): findSplits sorts the numeric block only (on the device,
            # no host round trip), the bins come from the hybrid parts, the level histograms of the
            # one-hot columns run over their entries
            if thresholds is None:
                thresholds = (T.thresholds_hybrid_device(hybrid, self.max_bins, seed=self.seed)
                              or T.find_thresholds_hybrid(hybrid, self.max_bins, seed=self.seed))
            if isinstance(thresholds, T.DeviceThresholds) and thresholds.thr_mat.shape[1] == self.max_bins:
                self.thresholds = thresholds
                self.nbins, self.thr_mat = thresholds.nbins, thresholds.thr_mat
            else:
                if isinstance(thresholds, T.DeviceThresholds):
                    thresholds = thresholds.to_table()
                self.thresholds = tt = T.ThresholdTable.from_any(thresholds)
                self.nbins = torch.from_numpy((tt.counts + 1).astype(np.int32)).to(X.device)
                self.thr_mat = torch.from_numpy(tt.padded(self.max_bins)).to(X.device)
            self.bins = T.bins_hybrid(hybrid, self.thr_mat, self.nbins)
            self.sparse = T.sparse_tree_input(hybrid)
            return
        if isinstance(thresholds, T.DeviceThresholds):
            thresholds = thresholds.to_table()
        if thresholds is None:
            # GPU: device findSplits (one sort, one small copy back; the same thresholds)
            thresholds = T.thresholds_for(X, self.max_bins, seed=self.seed)
        self.thresholds = tt = T.ThresholdTable.from_any(thresholds)  # one padded matrix, no per-feature loop
        self.nbins = torch.from_numpy((tt.counts + 1).astype(np.int32)).to(X.device)
        self.thr_mat = torch.from_numpy(tt.padded(self.max_bins)).to(X.device)
        self.bins = bin_features(X, tt).to(X.device).contiguous()  # [F, N] uint8 (HIP on the GPU)

    def bootstrap_weights(self, N: int, device, row_offset: int = 0) -> torch.Tensor:
        """Host oracle of the device tree_init draws (same Philox keys, same CDF table)."""
        if self.cdf is None:
            return torch.ones(self.T, N, dtype=torch.float32, device=device)
        return torch.from_numpy(rng.bootstrap_weights(self.seed, range(self.tree_offset, self.tree_offset + self.T),
                                                      N, row_offset, self.cdf)).float().to(device)

    def fit(self, X: torch.Tensor, y: torch.Tensor, row_offset: int = 0, thresholds=None,
            row_weight: Optional[torch.Tensor] = None, hybrid=None) -> ForestArrays:
        """``row_weight`` [T, N] multiplies the bootstrap weights (0 = row not seen by that
        tree): the cross-validation folds of several forests grow in one lock-step build.
        ``hybrid`` (features.hybrid.HybridMatrix of the same rows as X): the one-hot-aware path."""
        dev = X.device
        N, F = X.shape
        self.prepare(X, thresholds, hybrid)
        Tn, K, D = self.T, self.K, self.D
        m = subset_size(self.subset, F, Tn)
        y32 = y.to(torch.int32).contiguous()
        n_all = N
        if self.allreduce is not None:  # data parallel: the node capacity must agree across ranks
            nt = torch.tensor([float(N)], dtype=torch.float64, device=dev)
            self.allreduce(nt)
            n_all = int(nt.item())
        maxn = int(min(2 ** (D + 1) - 1, 2 * max(n_all, 1) + 1))
        feature = torch.full((Tn, maxn), -1, dtype=torch.int32, device=dev)
        thresh = torch.zeros(Tn, maxn, dtype=torch.float32, device=dev)
        left = torch.zeros(Tn, maxn, dtype=torch.int32, device=dev)
        right = torch.zeros(Tn, maxn, dtype=torch.int32, device=dev)
        stats = torch.zeros(Tn, maxn, K, dtype=torch.float32, device=dev)
        gains = torch.zeros(Tn, maxn, dtype=torch.float32, device=dev)
        n_nodes = np.ones(Tn, dtype=np.int64)
        if dev.type == "cuda":
            rw = None if row_weight is None else row_weight.to(device=dev, dtype=torch.float32).contiguous()
            return _fit_device(self, y32, rw, row_offset, N, F, m, maxn, n_all)
        # ---- CPU builder (PyTorch; the oracle of the device loop) ----
        W = self.bootstrap_weights(N, dev, row_offset)        # [T, N]
        if row_weight is not None:
            W = W * row_weight.to(device=dev, dtype=W.dtype)
        # [T, N] x one-hot [N, K]: exact (integer weights)
        root = W @ torch.nn.functional.one_hot(y.long(), K).to(W.dtype)
        if self.allreduce is not None:
            self.allreduce(root)
        stats[:, 0] = root
        node_of = torch.zeros(Tn, N, dtype=torch.int32, device=dev)   # node id per (tree,row); -1 = done
        node_of[W == 0] = -1
        front_t = np.arange(Tn, dtype=np.int64)   # frontier: (tree, node)
        front_n = np.zeros(Tn, dtype=np.int64)
        for depth in range(D):
            if len(front_t) == 0:
                break
            st = stats[torch.as_tensor(front_t, device=dev), torch.as_tensor(front_n, device=dev)]  # [A0, K]
            w_tot = st.sum(1)
            imp = T._impurity(st.double(), w_tot.double(), self.impurity)
            cand = ((imp > 1e-12) & (w_tot >= 2 * self.min_inst)).cpu().numpy()
            ct, cn = front_t[cand], front_n[cand]
            A = len(ct)
            if A == 0:
                break
            # ---- group the rows of every candidate node ----
            cand_idx = torch.full((Tn, maxn), -1, dtype=torch.int64, device=dev)
            cand_idx[torch.as_tensor(ct, device=dev), torch.as_tensor(cn, device=dev)] = torch.arange(A, device=dev)
            valid = node_of >= 0
            key = torch.where(valid, cand_idx.gather(1, node_of.clamp_min(0).long()),
                              torch.full_like(node_of, -1, dtype=torch.int64))
            sel = key >= 0
            tt, rr = torch.nonzero(sel, as_tuple=True)
            kk = key[tt, rr]
            order = torch.argsort(kk, stable=True)
            rows = rr[order].to(torch.int32).contiguous()
            keys = kk[order]
            row_w = W[tt[order], rr[order]].contiguous()
            feats = torch.from_numpy(rng.feature_subsets(self.seed, ct + self.tree_offset, cn, F, m)).to(dev)
            # ---- histogram + best split ----
            hist = T.level_histogram(self.bins, y32, rows, row_w, keys, A, feats, K, self.max_bins)
            if self.owner is not None:
                res = T.split_owner(hist, feats, K, self.owner, lambda h, a0, a1: T.split_from_hist(
                    h, feats[a0:a1], self.nbins, self.min_inst, self.min_gain, self.impurity))
            else:
                if self.allreduce is not None:
                    self.allreduce(hist)
                res = T.split_from_hist(hist, feats, self.nbins, self.min_inst, self.min_gain, self.impurity)
            do_split = (res.gain > 0) & torch.isfinite(res.gain)
            ds = do_split.cpu().numpy()
            if not ds.any():
                break
            st_t, st_n = ct[ds], cn[ds]
            # allocate children: per tree, consecutive ids (the frontier stays grouped by tree,
            # so a node's rank inside its tree is its offset from the tree's first entry)
            rank_in_tree = np.arange(len(st_t)) - np.searchsorted(st_t, st_t, side="left")
            child_l = n_nodes[st_t] + 2 * rank_in_tree
            n_nodes += 2 * np.bincount(st_t, minlength=Tn)
            ti = torch.as_tensor(st_t, device=dev)
            ni = torch.as_tensor(st_n, device=dev)
            cl = torch.as_tensor(child_l, device=dev)
            dsi = torch.as_tensor(np.nonzero(ds)[0], device=dev)
            bf = res.feat[dsi].long()
            bb = res.bin[dsi].long()
            feature[ti, ni] = bf.to(torch.int32)
            thresh[ti, ni] = self.thr_mat[bf, bb]
            left[ti, ni] = cl.to(torch.int32)
            right[ti, ni] = (cl + 1).to(torch.int32)
            gains[ti, ni] = res.gain[dsi] * res.total[dsi].sum(1)
            lstat = res.left[dsi]
            stats[ti, cl] = lstat
            stats[ti, cl + 1] = res.total[dsi] - lstat
            # ---- partition: rows of the nodes split at THIS level move to a child, all others finish ----
            lvl_feat = torch.full((Tn, maxn), -1, dtype=torch.int64, device=dev)
            lvl_bin = torch.zeros(Tn, maxn, dtype=torch.int64, device=dev)
            lvl_left = torch.zeros(Tn, maxn, dtype=torch.int64, device=dev)
            lvl_feat[ti, ni] = bf
            lvl_bin[ti, ni] = bb
            lvl_left[ti, ni] = cl
            idx = node_of.clamp_min(0).long()
            f_of = lvl_feat.gather(1, idx)
            moved = (node_of >= 0) & (f_of >= 0)
            b_of = self.bins[f_of.clamp_min(0), torch.arange(N, device=dev).view(1, -1).expand(Tn, -1)].long()
            go_left = b_of <= lvl_bin.gather(1, idx)
            nxt = lvl_left.gather(1, idx) + (~go_left).long()
            node_of = torch.where(moved, nxt, torch.full_like(nxt, -1)).to(torch.int32)
            front_t = np.repeat(st_t, 2)
            front_n = np.stack([child_l, child_l + 1], 1).reshape(-1)
        return ForestArrays(feature, thresh, left, right, stats, n_nodes, D, gains)


GROUP_MAX_NT = 4096  # tree_level.hip: per-tree candidates a level grouping keeps in LDS
# Bounds of a level enqueued without reading its counts back (the kernels read the real counts from
# the device; arrays and grids are sized by these bounds): node-count bound, and the bound times
# the grouping's row chunks (its count workspace).
ASYNC_MAX_NODES = 1 << 22
ASYNC_MAX_COUNT_WS = 1 << 27
# Sibling subtraction (trees that search every feature at every node: DecisionTree, featureSubset
# "all"): per-level histogram store cap in bytes; a level whose store would exceed it histograms
# every node directly.  With per-node random feature subsets (RandomForest sqrt / log2 / onethird)
# a child's features are not its parent's, so there is no parent histogram to subtract from.
SUBTRACT_MAX_BYTES = 4 << 30
SIBLING_SUBTRACTION = True
# ... and only for fits of at least this many (tree, row) pairs: below it a level is launch-bound and
# the store writes + derive pass cost more than the halved histogram work saves (bench --config dt:
# 60k rows 2.71 ms with, 2.57 ms without)
SUBTRACT_MIN_PAIRS = 1 << 20


# Test hook: when True the level loop groups rows with the stable radix sort of the level keys
# instead of the counting-sort kernel (the two must grow bit-identical forests).
FORCE_SORT_GROUPING = False
# Test hook: when True a single-device level runs one workgroup per node (hist_split_native)
# instead of the row-balanced plan (hist_split_planned); both grow the same forest.
FORCE_NODE_BLOCKS = False
# Test hook: when True every level reads its counts back (one 16-byte D2H per level) instead of
# running on device-side counts; both grow the same forest.
FORCE_LEVEL_SYNC = False
# host timestamps of the last device level loop: (start, every level enqueued, node counts read back)
LAST_LEVEL_TIMES = (0.0, 0.0, 0.0)
# device -> host count reads the level loops have made (0 per fit when every level runs on the device
# counts; a data-parallel fit reads one 16-byte record per level: tests/test_gpu_distributed.py)
LEVEL_SYNCS = 0
# data parallel: read each level's node count (16 bytes) so the histogram collectives carry the real
# nodes only, in fp16 when exact; False = the r3 behaviour (collectives sized by the host bound
# min(2^depth x trees, trees x rows), no reads) — kept for the byte comparison (HAR_TREE_DP_BOUND=1)
DP_COUNT_READS = os.environ.get("HAR_TREE_DP_BOUND", "0") != "1"


def _levels_device_frontier(b: "ForestBuilder", y32, W, N: int, F: int, m: int, maxn: int, stats, feature, thresh,
                            left, right, gains, node_of, n_all: Optional[int] = None):
    """Device level loop with the frontier resident on the GPU; returns the per-tree node counts
    (a device tensor: the caller reads them back once).

    The root frontier (candidate roots: impurity > 1e-12 in fp64 and weight >= 2 minInstances, the
    decision kernel's rule) is built on the device from the root class counts (tree_root_frontier).

    Per level (tree_level.hip unless noted): stable counting-sort grouping of the (tree, row)
    pairs by candidate node; Floyd feature subsets; the fused histogram + split kernel
    (tree.hip); the split / child-candidacy decision; the frontier update (split slots by a
    scan, child ids per tree, next candidates by a second scan, their cand_idx entries and tree
    starts); the commit of every split and both children's stats; the row partition.

    Counts on the device: the frontier kernel writes each level's [splits, next candidates, max
    candidates per tree, max candidate weight] into its own row of ``scal_all``; the next level's
    kernels read the candidate count from there (``a_dev``) while the host sizes grids and arrays
    by a bound (next candidates <= 2 x this level's, per tree <= 2 x the per-tree maximum).  On one
    device the whole fit is therefore enqueued with no device -> host read until the final node
    counts.  A level whose bound would exceed ``ASYNC_MAX_NODES`` / ``ASYNC_MAX_COUNT_WS`` or the
    grouping's LDS (``GROUP_MAX_NT`` per tree) first reads the previous level's 16 bytes back — the
    kernels then get the exact counts.  Both modes grow the same forest node for node.

    Data parallel (``b.allreduce`` / ``b.owner``) runs this same loop: the same grouping, plan and
    work items, with the level's histograms kept per node (``ops.tree.hist_split_planned_dp``) and
    summed across ranks before the split search.  Every collective is sized by the host bound of
    the level's node count, which all ranks share (the bounds use the global row count ``n_all``),
    so a DP level reads nothing back either; the frontier is replicated (every rank applies the
    same winners).  Sibling subtraction stays single-device (a derived node would need its
    parent's summed histogram on the rank that owns it)."""
    dp = b.owner is not None or b.allreduce is not None
    n_all = N if n_all is None else n_all
    dev = W.device
    Tn, K, D = b.T, b.K, b.D
    mod = _native.kernels()
    st = _native.stream_ptr()
    i32 = dict(dtype=torch.int32, device=dev)
    Wf = W.reshape(-1).contiguous()
    sparse = getattr(b, "sparse", None)
    # [N, F] for the histogram gathers (partition keeps [F, N]); the one-hot-aware kernel gathers only
    # the numeric columns' bytes and reads the feature-major bins
    bins_rm = b.bins.t().contiguous() if sparse is None else None
    nch = mod.tree_level_group_chunks(N)
    nch_g = mod.tree_level_group_chunks(n_all)  # rank-independent bound checks (DP: every rank decides alike)
    planned = not FORCE_NODE_BLOCKS
    # data parallel: ONE 16-byte count read per level, so every collective is sized by the level's
    # real node count (not the bound 2^depth x trees) and may travel as fp16 (DP_COUNT_READS)
    async_ok = planned and not FORCE_SORT_GROUPING and not FORCE_LEVEL_SYNC and not (dp and DP_COUNT_READS)
    slot_bytes = 4 * F * b.max_bins * K
    subtract = planned and not dp and m >= F and SIBLING_SUBTRACTION and Tn * N >= SUBTRACT_MIN_PAIRS
    hprev = parent_of = derive_from = None  # the previous level's store and this level's derive info

    # root frontier on the device: scal_all row 0 = [0, root candidates, 1, max root weight bits]
    A, nt_max = Tn, 1  # bounds (exact = False: the kernels read the root candidate count from row 0)
    exact = False
    ct, cn, tlo = torch.empty(A, **i32), torch.empty(A, **i32), torch.empty(Tn + 1, **i32)
    cand_idx = torch.full((Tn, maxn), -1, **i32)  # stale entries name nodes no row sits in any more
    scal_all = torch.zeros(4 * (D + 1), **i32)
    mod.tree_root_frontier(stats.data_ptr(), Tn, K, maxn * K, b.impurity, float(2 * b.min_inst), maxn,
                           ct.data_ptr(), cn.data_ptr(), tlo.data_ptr(), cand_idx.data_ptr(), scal_all.data_ptr(), st)
    nn = torch.ones(Tn, **i32)
    nn_next = torch.empty_like(nn)
    split_bin = torch.zeros(Tn, maxn, **i32)
    rows_buf = torch.empty(Tn * N, **i32)
    roww_buf = torch.empty(Tn * N, dtype=torch.float32, device=dev)
    tlo_next = torch.empty(Tn + 1, **i32)
    scal_h = None
    max_w = 0.0
    global LEVEL_SYNCS
    if not async_ok:  # exact counts from the start (test hooks): read row 0 back
        scal_h = torch.empty(4, dtype=torch.int32).pin_memory()
        scal_h.copy_(scal_all[:4])
        LEVEL_SYNCS += 1
        A, wbits = int(scal_h[1]), int(scal_h[3])
        max_w = float(np.array([wbits], dtype=np.int32).view(np.float32)[0])
        exact = True
        if A == 0:
            return nn
        ct, cn = ct[:A], cn[:A]
    cnt_ws = None
    t_start = time.perf_counter()
    for depth in range(D):
        a_dev = 0 if exact else scal_all.data_ptr() + 4 * (4 * depth + 1)
        scal = scal_all[4 * (depth + 1):4 * (depth + 2)]
        if cnt_ws is None or cnt_ws.numel() < nch * A:
            cnt_ws = torch.empty(nch * max(A, 2 * Tn), **i32)
        counts, starts = torch.empty(A, **i32), torch.empty(A, **i32)
        if nt_max <= GROUP_MAX_NT and not FORCE_SORT_GROUPING:
            mod.tree_level_group(node_of.data_ptr(), cand_idx.data_ptr(), tlo.data_ptr(), Wf.data_ptr(), Tn, N,
                                 maxn, A, nt_max, cnt_ws.data_ptr(), counts.data_ptr(), starts.data_ptr(),
                                 rows_buf.data_ptr(), roww_buf.data_ptr(), a_dev, st)
            rows, row_w = rows_buf, roww_buf
        else:  # a tree with > GROUP_MAX_NT candidates (exact level): a stable radix sort of the keys
            key = torch.empty(Tn * N, **i32)
            mod.tree_level_keys(node_of.data_ptr(), cand_idx.data_ptr(), Tn, N, maxn, key.data_ptr(), st)
            keys, order = torch.sort(key, stable=True)
            rows, row_w = (order % N).to(torch.int32), Wf[order]
            bounds = torch.searchsorted(keys, torch.arange(A + 1, **i32))
            counts = (bounds[1:] - bounds[:-1]).to(torch.int32)
            starts = bounds[:-1].to(torch.int32)
        if m >= F:
            feats = torch.arange(F, **i32).repeat(A, 1)
        else:
            feats = torch.empty(A, m, **i32)
            tr = ct + b.tree_offset if b.tree_offset else ct
            mod.tree_feature_subsets(b.seed, tr.data_ptr(), cn.data_ptr(), A, F, m, feats.data_ptr(), a_dev, st)
        store = None
        if subtract and A * slot_bytes <= SUBTRACT_MAX_BYTES:
            store = torch.empty(A * slot_bytes // 4, dtype=torch.float32, device=dev)
        if planned and dp:
            # data parallel: the same work items, histograms summed across ranks by the bound A
            # the candidates' global class counts (replicated stats): the packed wire format's layout
            node_cc = (stats.view(Tn * maxn, K)[ct[:A].long() * maxn + cn[:A].long()]
                       if exact and b.owner is not None and getattr(b, "int_weights", False) else None)
            res = T.hist_split_planned_dp(b.bins, b.nbins, y32, rows, row_w, starts, counts, feats, K, b.max_bins,
                                          b.min_inst, b.min_gain, b.impurity, rows_bound=Tn * N, a_dev=a_dev,
                                          allreduce=None if b.owner is not None else b.allreduce, owner=b.owner,
                                          bins_rm=bins_rm,
                                          # fp16 transport only for integer counts (exact below 2048)
                                          max_weight=max_w if exact and getattr(b, "int_weights", False) else -1.0,
                                          node_cc=node_cc, sparse=sparse)
        elif planned:
            # one device: work items by rows (big nodes chunked), no host sync (ops/tree.py)
            res = T.hist_split_planned(b.bins, b.nbins, y32, rows, row_w, starts, counts, feats, K, b.max_bins,
                                       b.min_inst, b.min_gain, b.impurity, rows_bound=Tn * N, bins_rm=bins_rm,
                                       prows=T.PLAN_ROWS if sparse is None else T.SPARSE_PLAN_ROWS,
                                       a_dev=a_dev, store=store, hprev=hprev, derive_from=derive_from,
                                       parent_of=parent_of, sparse=sparse)
        else:
            res = T.hist_split_native(b.bins, b.nbins, y32, rows, row_w, starts, counts, feats, K, b.max_bins,
                                      b.min_inst, b.min_gain, b.impurity,
                                      allreduce=None if b.owner is not None else b.allreduce, owner=b.owner,
                                      max_rows=int(max_w), check_labels=False, bins_rm=bins_rm, sparse=sparse)
        res = T.LevelResult(gain=res.gain.contiguous(), feat=res.feat.contiguous(), bin=res.bin.contiguous(),
                            left=res.left.contiguous(), total=res.total.contiguous())
        dec = torch.empty(5, A, dtype=torch.float32, device=dev)
        mod.tree_level_decide(A, res.gain.data_ptr(), res.left.data_ptr(), res.total.data_ptr(), K, b.impurity,
                              float(2 * b.min_inst), dec.data_ptr(), a_dev, st)
        pos = torch.empty(A + 1, **i32)
        ti, ni, cl, dsi = (torch.empty(A, dtype=torch.int64, device=dev) for _ in range(4))
        front = torch.empty(2 * A, dtype=torch.float32, device=dev)
        q = torch.empty(2 * A + 1, **i32)
        ct_next, cn_next = torch.empty(2 * A, **i32), torch.empty(2 * A, **i32)
        A_b = min(2 * A, Tn * n_all)
        # the next level derives siblings when this level kept its histograms and the next one can
        derive = store is not None and A_b * slot_bytes <= SUBTRACT_MAX_BYTES
        par_n = torch.empty(2 * A, **i32) if derive else None
        der_n = torch.empty(2 * A, **i32) if derive else None
        mod.tree_frontier(A, Tn, maxn, ct.data_ptr(), cn.data_ptr(), tlo.data_ptr(), dec.data_ptr(), nn.data_ptr(),
                          nn_next.data_ptr(), pos.data_ptr(), ti.data_ptr(), ni.data_ptr(), cl.data_ptr(),
                          dsi.data_ptr(), front.data_ptr(), q.data_ptr(), ct_next.data_ptr(), cn_next.data_ptr(),
                          tlo_next.data_ptr(), cand_idx.data_ptr(), scal.data_ptr(), a_dev,
                          par_n.data_ptr() if derive else 0, der_n.data_ptr() if derive else 0, st)
        # the last level commits on the device count too (nothing after it needs the host)
        bounds_ok = A_b <= ASYNC_MAX_NODES and nch_g * A_b <= ASYNC_MAX_COUNT_WS and 2 * nt_max <= GROUP_MAX_NT
        stay_async = async_ok and (depth + 1 == D or bounds_ok)
        if stay_async:  # the next level runs on the device counts in scal
            S, s_dev, A_next, nt_next = A, scal.data_ptr(), A_b, 2 * nt_max
        else:
            if scal_h is None:
                scal_h = torch.empty(4, dtype=torch.int32).pin_memory()
            scal_h.copy_(scal)  # this level's one sync
            LEVEL_SYNCS += 1
            S, A_next, nt_next, wbits = (int(v) for v in scal_h.tolist())
            s_dev = 0
            max_w = float(np.array([wbits], dtype=np.int32).view(np.float32)[0])
            if S == 0:
                break
        mod.tree_commit_level(S, ti.data_ptr(), ni.data_ptr(), cl.data_ptr(), dsi.data_ptr(), res.feat.data_ptr(),
                              res.bin.data_ptr(), res.gain.data_ptr(), res.left.data_ptr(), res.total.data_ptr(), K,
                              b.thr_mat.data_ptr(), b.thr_mat.shape[1], maxn, feature.data_ptr(),
                              split_bin.data_ptr(), thresh.data_ptr(), left.data_ptr(), right.data_ptr(),
                              gains.data_ptr(), stats.data_ptr(), s_dev, st)
        mod.tree_partition_split(node_of.data_ptr(), feature.data_ptr(), split_bin.data_ptr(), left.data_ptr(),
                                 b.bins.data_ptr(), Tn, N, maxn, st)
        nn, nn_next = nn_next, nn
        ct, cn, A = ct_next[:A_next], cn_next[:A_next], A_next
        tlo, tlo_next = tlo_next, tlo
        nt_max = max(nt_next, 1)
        exact = not stay_async
        hprev, parent_of, derive_from = (store, par_n, der_n) if derive else (None, None, None)
        if A == 0:
            break
    global LAST_LEVEL_TIMES
    LAST_LEVEL_TIMES = (t_start, time.perf_counter(), 0.0)
    return nn


def levels_all_async(b: "ForestBuilder", N: int, F: int, m: int, n_all: Optional[int] = None) -> bool:
    """True when every level of this fit runs on device-side counts (no host read inside the
    loop): the condition for capturing the fit in a HIP graph.  The loop's decisions depend only
    on the bounds, so this replays them."""
    if FORCE_NODE_BLOCKS or FORCE_SORT_GROUPING or FORCE_LEVEL_SYNC:
        return False
    n_all = N if n_all is None else n_all
    nch = _native.kernels().tree_level_group_chunks(n_all)
    A, nt = b.T, 1
    for depth in range(b.D - 1):
        A_b = min(2 * A, b.T * n_all)
        if A_b > ASYNC_MAX_NODES or nch * A_b > ASYNC_MAX_COUNT_WS or 2 * nt > GROUP_MAX_NT:
            return False
        A, nt = A_b, 2 * nt
    return True


# HIP graphs of whole device fits (tree_init + root frontier + every level), keyed by everything
# the launches bake in; a signature is captured the second time it is fitted (a one-off fit stays
# eager: capture costs about one eager fit) and replayed from then on, after its inputs are
# copied into the graph's static buffers.  HAR_TREE_GRAPH=0 disables it.
FIT_GRAPHS = os.environ.get("HAR_TREE_GRAPH", "1") != "0"
FIT_GRAPH_MAX = 8
# how the last device fit ran: "eager" (launched from Python), "capture" (launched while recorded
# into a HIP graph) or "replay" (the graph of an earlier fit of the same signature)
LAST_FIT_KIND = "eager"
_fit_graph_seen: dict = {}
_fit_graphs: dict = {}


class _FitGraph:
    def __init__(self, b: "ForestBuilder", y32, rw, N: int, F: int, maxn: int):
        dev = y32.device
        Tn, K = b.T, b.K
        self.bins = torch.empty_like(b.bins)
        self.nbins = torch.empty_like(b.nbins)
        self.thr_mat = torch.empty_like(b.thr_mat)
        self.y32 = torch.empty_like(y32)
        self.rw = None if rw is None else torch.empty_like(rw)
        sp = getattr(b, "sparse", None)
        # the one-hot-aware kernels' inputs are baked into the graph too: static copies
        self.sparse = None if sp is None else T.SparseTreeInput(torch.empty_like(sp.cat), torch.empty_like(sp.onehot),
                                                                 sp.n_features)
        self.bufs = _alloc_fit_buffers(Tn, N, K, maxn, dev)
        self.graph = None
        self.maxn = maxn

    def load(self, b: "ForestBuilder", y32, rw):
        self.bins.copy_(b.bins)
        self.nbins.copy_(b.nbins)
        self.thr_mat.copy_(b.thr_mat)
        self.y32.copy_(y32)
        if rw is not None:
            self.rw.copy_(rw)
        if self.sparse is not None:
            self.sparse.cat.copy_(b.sparse.cat)
            self.sparse.onehot.copy_(b.sparse.onehot)


_OUT_ARRAYS = (("feature", torch.int32, False), ("thresh", torch.float32, False), ("left", torch.int32, False),
               ("right", torch.int32, False), ("stats", torch.float32, True), ("gains", torch.float32, False))


def _alloc_fit_buffers(Tn: int, N: int, K: int, maxn: int, dev) -> dict:
    """Work arrays of one device fit; the six output arrays are views of ONE flat 32-bit buffer
    (``out``), so a fit's result is one clone, not six."""
    per = Tn * maxn
    sizes = [per * K if wide else per for _, _, wide in _OUT_ARRAYS]
    flat = torch.empty(sum(sizes), dtype=torch.int32, device=dev)
    bufs = dict(W=torch.empty(Tn, N, dtype=torch.float32, device=dev),
                node_of=torch.empty(Tn, N, dtype=torch.int32, device=dev),
                bad=torch.empty(1, dtype=torch.int32, device=dev), out=flat)
    bufs.update(_out_views(flat, Tn, maxn, K))
    return bufs


def _out_views(flat: torch.Tensor, Tn: int, maxn: int, K: int) -> dict:
    views, o = {}, 0
    for (name, dt, wide) in _OUT_ARRAYS:
        n = Tn * maxn * (K if wide else 1)
        v = flat[o:o + n]
        v = v.view(torch.float32) if dt == torch.float32 else v
        views[name] = v.view(Tn, maxn, K) if wide else v.view(Tn, maxn)
        o += n
    return views


def _enqueue_fit(b: "ForestBuilder", bufs: dict, y32, rw, row_offset: int, N: int, F: int, m: int, maxn: int,
                 n_all: Optional[int] = None):
    """Every launch of one device fit into ``bufs`` (no host read on one device): initial node
    arrays, tree_init (bootstrap weights x row weights, node ids, root class counts, label check), the
    DP all-reduce of the root counts, the level loop.  Returns the node-count tensor."""
    Tn, K = b.T, b.K
    bufs["out"].zero_()  # (thresh / left / right / stats / gains; one fill)
    bufs["feature"].fill_(-1)
    bufs["bad"].zero_()
    cdf = [] if b.cdf is None else [int(v) for v in b.cdf]
    _native.kernels().tree_init(b.seed, b.tree_offset, Tn, row_offset, N, cdf, 0 if rw is None else rw.data_ptr(),
                                y32.data_ptr(), K, bufs["W"].data_ptr(), bufs["node_of"].data_ptr(),
                                bufs["stats"].data_ptr(), maxn * K, bufs["bad"].data_ptr(), _native.stream_ptr())
    if b.allreduce is not None:
        # integer row weights (bootstrap counts x 0/1 folds): histogram counts are integers, so the DP
        # levels may ship them as packed integer fields (ops.tree.dp_wire_plan) or as fp16.  Every rank
        # must take the SAME wire path (mismatched collectives hang or corrupt the sums), so the
        # shard-local "some weight is fractional" flag rides in the root-count all-reduce: integer
        # only when no rank has a fractional weight
        nonint = (torch.zeros(1, device=y32.device) if rw is None
                  else (rw != torch.round(rw)).any().float().reshape(1))
        root = torch.cat([bufs["stats"][:, 0].reshape(-1), nonint])
        b.allreduce(root)
        bufs["stats"][:, 0] = root[:-1].view(Tn, K)
        b.int_weights = bool(root[-1].item() == 0)
    return _levels_device_frontier(b, y32, bufs["W"], N, F, m, maxn, bufs["stats"], bufs["feature"], bufs["thresh"],
                                   bufs["left"], bufs["right"], bufs["gains"], bufs["node_of"], n_all=n_all)


def _finish_fit(b: "ForestBuilder", bufs: dict, nn, clone: bool) -> ForestArrays:
    h = torch.cat([nn, bufs["bad"]]).cpu().numpy()  # the fit's one device -> host read
    if h[-1] != 0:
        raise ValueError("labels out of range")
    Tn, maxn = bufs["feature"].shape
    o = _out_views(bufs["out"].clone(), Tn, maxn, b.K) if clone else bufs
    return ForestArrays(o["feature"], o["thresh"], o["left"], o["right"], o["stats"], h[:-1].astype(np.int64), b.D,
                        o["gains"])


def _fit_device(b: "ForestBuilder", y32, rw, row_offset: int, N: int, F: int, m: int, maxn: int,
                n_all: Optional[int] = None) -> ForestArrays:
    global LAST_FIT_KIND
    dev = y32.device
    n_all = N if n_all is None else n_all
    key = None
    if FIT_GRAPHS and not (b.allreduce or b.owner) and levels_all_async(b, N, F, m, n_all):
        key = (dev.index, b.T, b.K, b.D, N, F, m, maxn, b.max_bins, b.impurity, b.min_inst, b.min_gain, b.seed,
               b.tree_offset, None if b.cdf is None else tuple(int(v) for v in b.cdf), rw is not None, row_offset,
               SIBLING_SUBTRACTION, SUBTRACT_MIN_PAIRS, SUBTRACT_MAX_BYTES, ASYNC_MAX_NODES, ASYNC_MAX_COUNT_WS,
               b.bins.shape, tuple(b.thr_mat.shape),
               None if getattr(b, "sparse", None) is None else tuple(b.sparse.cat.shape))
    ent = _fit_graphs.get(key) if key is not None else None
    if ent is None and key is not None and _fit_graph_seen.get(key, 0) >= 1 and len(_fit_graphs) < FIT_GRAPH_MAX:
        # second fit of this signature: capture it (the first, eager fit warmed every kernel up)
        ent = _FitGraph(b, y32, rw, N, F, maxn)
        ent.load(b, y32, rw)
        own = (b.bins, b.nbins, b.thr_mat, getattr(b, "sparse", None))
        b.bins, b.nbins, b.thr_mat, b.sparse = ent.bins, ent.nbins, ent.thr_mat, ent.sparse
        try:
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                ent.nn = _enqueue_fit(b, ent.bufs, ent.y32, ent.rw, row_offset, N, F, m, maxn, n_all)
            ent.graph = g
        finally:
            b.bins, b.nbins, b.thr_mat, b.sparse = own
        _fit_graphs[key] = ent
        LAST_FIT_KIND = "capture"
    elif ent is not None:
        LAST_FIT_KIND = "replay"
    else:
        LAST_FIT_KIND = "eager"
    if ent is not None:
        ent.load(b, y32, rw)
        ent.graph.replay()
        return _finish_fit(b, ent.bufs, ent.nn, clone=True)
    if key is not None:
        _fit_graph_seen[key] = _fit_graph_seen.get(key, 0) + 1
    bufs = _alloc_fit_buffers(b.T, N, b.K, maxn, dev)
    nn = _enqueue_fit(b, bufs, y32, rw, row_offset, N, F, m, maxn, n_all)
    return _finish_fit(b, bufs, nn, clone=False)


def predict_forest(arrs: ForestArrays, X: torch.Tensor, normalize: bool) -> torch.Tensor:
    a = arrs if arrs.feature.device == X.device else arrs.to(X.device)
    if X.is_cuda:
        return T.forest_predict_native(X.float(), a.feature, a.threshold, a.left, a.right, a.stats, a.max_depth,
                                       normalize)
    return T.forest_predict_torch(X.float(), a.feature, a.threshold, a.left, a.right, a.stats, a.max_depth,
                                  normalize)


def _tree_depth(arrs: ForestArrays, t: int) -> int:
    feat = arrs.feature[t].cpu().numpy()
    left = arrs.left[t].cpu().numpy()
    right = arrs.right[t].cpu().numpy()
    best, stack = 0, [(0, 0)]
    while stack:
        n, d = stack.pop()
        best = max(best, d)
        if feat[n] >= 0:
            stack += [(int(left[n]), d + 1), (int(right[n]), d + 1)]
    return best


class DecisionTreeClassificationModel(ClassificationModel):
    def __init__(self, arrs: ForestArrays, num_features: int, num_classes: int, uid=None, device=None):
        super().__init__(uid or new_uid("DecisionTreeClassifier"))
        self.arrs = arrs
        self.num_features, self.num_classes = num_features, num_classes
        self.device = device or arrs.feature.device

    @property
    def depth(self) -> int:
        return _tree_depth(self.arrs, 0)

    @property
    def numNodes(self) -> int:
        return int(self.arrs.n_nodes[0])

    def predict_raw(self, X):
        return predict_forest(self.arrs, X.to(self.device), normalize=False)

    @property
    def featureImportances(self) -> torch.Tensor:
        return _importances(self.arrs, self.num_features)

    def __str__(self):
        return (f"DecisionTreeClassificationModel (uid={self.uid}) of depth {self.depth} "
                f"with {self.numNodes} nodes")

    def state(self):
        a = self.arrs
        return {"feature": a.feature.cpu(), "threshold": a.threshold.cpu(), "left": a.left.cpu(),
                "right": a.right.cpu(), "stats": a.stats.cpu(), "n_nodes": torch.as_tensor(a.n_nodes),
                "max_depth": a.max_depth}


class RandomForestClassificationModel(DecisionTreeClassificationModel):
    def __init__(self, arrs: ForestArrays, num_features: int, num_classes: int, uid=None, device=None):
        super().__init__(arrs, num_features, num_classes, uid or new_uid("RandomForestClassifier"), device)

    @property
    def getNumTrees(self) -> int:
        return int(self.arrs.feature.shape[0])

    @property
    def totalNumNodes(self) -> int:
        return int(self.arrs.n_nodes.sum())

    def predict_raw(self, X):
        return predict_forest(self.arrs, X.to(self.device), normalize=True)

    def __str__(self):
        return f"RandomForestClassificationModel (uid={self.uid}) with {self.getNumTrees} trees"


def _importances(arrs: ForestArrays, F: int) -> torch.Tensor:
    """Spark-style importances: per tree, gain-weighted split counts normalized, averaged, normalized."""
    imp = torch.zeros(F, dtype=torch.float64)
    feat = arrs.feature.cpu()
    g = arrs.gain.cpu().double() if arrs.gain is not None else torch.ones_like(feat, dtype=torch.float64)
    for t in range(feat.shape[0]):
        m = feat[t] >= 0
        it = torch.zeros(F, dtype=torch.float64)
        it.index_add_(0, feat[t][m].long(), g[t][m])
        s = it.sum()
        if s > 0:
            imp += it / s
    s = imp.sum()
    return imp / s if s > 0 else imp


class _TreeEstimatorBase(Estimator, ClassifierParams):
    _param_names = ("maxDepth", "maxBins", "minInstancesPerNode", "minInfoGain", "impurity", "seed",
                    "featuresCol", "labelCol", "device")

    def _prep(self, table: Table):
        dev = resolve_device(self.device)
        X = features_tensor(table, self.featuresCol, dev)
        y = labels_tensor(table, self.labelCol, dev)
        K = num_label_classes(table, self.labelCol, dev)
        return X, y, K

    def _hybrid(self, table: Table, device):
        """The column's one-hot index + numeric layout when it has one-hot blocks (the reference
        encoding) and the one-hot-aware tree path takes it, else None (features.hybrid)."""
        from ..features.hybrid import tree_hybrid

        hm = tree_hybrid(table, self.featuresCol, device)
        return hm if T.hybrid_tree_ok(hm) else None

    def _thresholds(self, X, hybrid):
        if hybrid is not None:
            return (T.thresholds_hybrid_device(hybrid, self.maxBins, seed=self.seed)
                    or T.find_thresholds_hybrid(hybrid, self.maxBins, seed=self.seed))
        return T.thresholds_for(X, self.maxBins, seed=self.seed)


class DecisionTreeClassifier(_TreeEstimatorBase):
    def __init__(self, featuresCol="features", labelCol="label", maxDepth: int = 5, maxBins: int = 32,
                 minInstancesPerNode: int = 1, minInfoGain: float = 0.0, impurity: str = "gini", seed: int = 0,
                 device=None):
        super().__init__(new_uid("DecisionTreeClassifier"))
        self.featuresCol, self.labelCol = featuresCol, labelCol
        self.maxDepth, self.maxBins, self.minInstancesPerNode = maxDepth, maxBins, minInstancesPerNode
        self.minInfoGain, self.impurity, self.seed, self.device = minInfoGain, impurity, seed, device

    def fit(self, table: Table) -> DecisionTreeClassificationModel:
        X, y, K = self._prep(table)
        hm = self._hybrid(table, X.device)
        if dp_context() is None:
            return self.fit_tensors(X, y, K, hybrid=hm)
        thr = self._thresholds(X, hm)
        lo, hi = dp_rows(X.shape[0])
        return self.fit_tensors(X[lo:hi], y[lo:hi], K, thresholds=thr, owner=dp_owner(), row_offset=lo,
                                hybrid=None if hm is None else hm.rows(lo, hi))

    def fit_tensors(self, X, y, K, thresholds=None, allreduce=None, owner=None,
                    row_offset: int = 0, hybrid=None) -> DecisionTreeClassificationModel:
        b = ForestBuilder(K, 1, self.maxDepth, self.maxBins, self.minInstancesPerNode, self.minInfoGain,
                          self.impurity, "all", bootstrap=False, seed=self.seed, allreduce=allreduce, owner=owner)
        return DecisionTreeClassificationModel(b.fit(X, y, row_offset=row_offset, thresholds=thresholds, hybrid=hybrid),
                                               X.shape[1], K, uid=self.uid, device=X.device)

    def fit_folds(self, X, y, K, masks: torch.Tensor, hybrid=None) -> List["DecisionTreeClassificationModel"]:
        """One tree per fold (``masks`` [k, N]: 1 = training row of fold f), all grown together
        (data parallel inside ``data_parallel``: row shards, owner-computes splits)."""
        b = ForestBuilder(K, masks.shape[0], self.maxDepth, self.maxBins, self.minInstancesPerNode, self.minInfoGain,
                          self.impurity, "all", bootstrap=False, seed=self.seed, owner=dp_owner())
        arrs = _fit_sharded(b, X, y, masks, self.maxBins, self.seed, hybrid)
        return [DecisionTreeClassificationModel(_slice_arrays(arrs, f, f + 1), X.shape[1], K, uid=self.uid,
                                                device=X.device) for f in range(masks.shape[0])]



# (tree, row) slots of one lock-step forest build: row lists, counts and scans in tree_level.hip
# are int32, so one build never holds more slots than this (bigger forests grow in tree waves)
LOCKSTEP_SLOT_LIMIT = 2 ** 31 - 1


def max_lockstep_trees(n_rows: int) -> int:
    """Most trees one lock-step build may grow over ``n_rows`` rows (>= 1)."""
    return max(1, LOCKSTEP_SLOT_LIMIT // max(1, n_rows))


# "auto" tree parallelism while the replicated fp32 feature matrix stays below this (every rank holds it)
TREE_PARALLEL_MAX_BYTES = 16 << 30


class RandomForestClassifier(_TreeEstimatorBase):
    _param_names = _TreeEstimatorBase._param_names + ("numTrees", "featureSubsetStrategy", "subsamplingRate",
                                                      "parallelism")

    def __init__(self, featuresCol="features", labelCol="label", numTrees: int = 20, maxDepth: int = 5,
                 maxBins: int = 32, minInstancesPerNode: int = 1, minInfoGain: float = 0.0, impurity: str = "gini",
                 featureSubsetStrategy: str = "auto", subsamplingRate: float = 1.0, seed: int = 0, device=None,
                 parallelism: str = "auto"):
        super().__init__(new_uid("RandomForestClassifier"))
        self.featuresCol, self.labelCol = featuresCol, labelCol
        self.numTrees, self.maxDepth, self.maxBins = numTrees, maxDepth, maxBins
        self.minInstancesPerNode, self.minInfoGain, self.impurity = minInstancesPerNode, minInfoGain, impurity
        self.featureSubsetStrategy, self.subsamplingRate = featureSubsetStrategy, subsamplingRate
        self.seed, self.device = seed, device
        # multi-GPU strategy under data_parallel: "data" = row shards + per-level owner reduction,
        # "tree" = every rank all rows, numTrees / P trees, one all-gather; "auto" = tree when the
        # replicated feature matrix is small (TREE_PARALLEL_MAX_BYTES) and there are >= P trees
        self.parallelism = parallelism

    def resolve_parallelism(self, n_rows: int, n_features: int, world: int) -> str:
        p = str(self.parallelism).lower()
        if p not in ("auto", "data", "tree"):
            raise ValueError(f"parallelism must be auto, data or tree, got {self.parallelism!r}")
        if p != "auto":
            return p
        fits = n_rows * n_features * 4 <= TREE_PARALLEL_MAX_BYTES
        return "tree" if (fits and self.numTrees >= world) else "data"

    def fit(self, table: Table) -> RandomForestClassificationModel:
        X, y, K = self._prep(table)
        hm = self._hybrid(table, X.device)
        ctx = dp_context()
        if ctx is None:
            return self.fit_tensors(X, y, K, hybrid=hm)
        thr = self._thresholds(X, hm)
        if self.resolve_parallelism(X.shape[0], X.shape[1], ctx.world_size) == "tree":
            from ..parallel.data_parallel import fit_forest_tree_parallel

            return fit_forest_tree_parallel(self, X, y, K, ctx, thresholds=thr, hybrid=hm)
        lo, hi = dp_rows(X.shape[0])
        return self.fit_tensors(X[lo:hi], y[lo:hi], K, row_offset=lo, thresholds=thr, owner=dp_owner(),
                                hybrid=None if hm is None else hm.rows(lo, hi))

    def fit_tensors(self, X, y, K, allreduce=None, row_offset: int = 0, thresholds=None,
                    tree_wave: int = 0, checkpoint_dir: Optional[str] = None, rank: int = 0, owner=None,
                    tree_offset: int = 0, num_trees: Optional[int] = None, hybrid=None):
        """Grow the forest (all trees in lock step, or in waves of ``tree_wave`` trees —
        each wave checkpointed under ``checkpoint_dir`` and skipped on resume).  Trees
        are keyed by their global id, so a waved forest equals the one-shot forest.
        ``hybrid``: the one-hot-aware path (same forest)."""
        strategy = self.featureSubsetStrategy
        if str(strategy).lower() == "auto":
            strategy = "all" if self.numTrees == 1 else "sqrt"
        if hybrid is not None and not (X.is_cuda and T.hybrid_tree_ok(hybrid)):
            hybrid = None
        if thresholds is None:
            thresholds = self._thresholds(X, hybrid)
        # tree-parallel mode grows trees [tree_offset, tree_offset + num_trees) of the forest: global tree
        # ids key the bootstrap and feature-subset streams, so the slices concatenate into the forest
        total = self.numTrees if num_trees is None else int(num_trees)
        wave = tree_wave if tree_wave and tree_wave < total else total
        # (tree, row) slots of one lock-step build are int32-indexed on the device
        # (tree_level.hip row lists / scans): cap a wave at LOCKSTEP_SLOT_LIMIT slots
        max_wave = max_lockstep_trees(int(X.shape[0]))
        if wave > max_wave:
            wave = max_wave
        ckpt = None
        parts: List[ForestArrays] = []
        fp = {"numTrees": total, "tree_offset": tree_offset, "seed": self.seed, "maxDepth": self.maxDepth,
              "maxBins": self.maxBins, "minInstancesPerNode": self.minInstancesPerNode,
              "minInfoGain": self.minInfoGain, "impurity": self.impurity, "strategy": str(strategy),
              "subsamplingRate": self.subsamplingRate, "rows": int(X.shape[0]), "features": int(X.shape[1]),
              "classes": int(K), "row_offset": int(row_offset)}
        if checkpoint_dir:
            from ..utils.checkpoint import Checkpointer

            ckpt = Checkpointer(checkpoint_dir, rank=rank)
            last = ckpt.latest(fingerprint=fp)
            if last is not None:
                prev = _arrays_from_state(last[0])
                parts.append(_slice_arrays(prev, 0, min(total, prev.feature.shape[0])))
        from ..utils.checkpoint import maybe_inject_fault

        done = sum(p.feature.shape[0] for p in parts)
        if total <= 0:  # a tree-parallel rank with an empty slice (more ranks than trees)
            D = self.maxDepth
            maxn = int(min(2 ** (D + 1) - 1, 2 * max(int(X.shape[0]), 1) + 1))
            dev = X.device
            parts.append(ForestArrays(torch.full((0, maxn), -1, dtype=torch.int32, device=dev),
                                      torch.zeros(0, maxn, device=dev), torch.zeros(0, maxn, dtype=torch.int32, device=dev),
                                      torch.zeros(0, maxn, dtype=torch.int32, device=dev),
                                      torch.zeros(0, maxn, K, device=dev), np.zeros(0, dtype=np.int64), D,
                                      torch.zeros(0, maxn, device=dev)))
        while done < total:
            maybe_inject_fault(done, rank)
            nt = min(wave, total - done)
            b = ForestBuilder(K, nt, self.maxDepth, self.maxBins, self.minInstancesPerNode, self.minInfoGain,
                              self.impurity, strategy, bootstrap=self.numTrees > 1, seed=self.seed,
                              allreduce=allreduce, tree_offset=tree_offset + done, owner=owner,
                              subsample=self.subsamplingRate)
            parts.append(b.fit(X, y, row_offset=row_offset, thresholds=thresholds, hybrid=hybrid))
            done += nt
            if ckpt is not None and done < total:
                merged = _concat_arrays(parts)
                parts = [merged]
                ckpt.save(done, _arrays_state(merged), {"trees": done}, fingerprint=fp)
        arrs = _concat_arrays(parts) if len(parts) > 1 else parts[0]
        return RandomForestClassificationModel(arrs.to(X.device), X.shape[1], K, uid=self.uid, device=X.device)

    def fit_folds(self, X, y, K, masks: torch.Tensor, hybrid=None) -> List["RandomForestClassificationModel"]:
        """k forests of numTrees trees (fold f: trees f*T .. f*T+T-1, its own bootstrap / feature
        streams) grown as ONE level-synchronous build of k*T trees over the shared binned matrix."""
        T_, k = self.numTrees, masks.shape[0]
        strategy = self.featureSubsetStrategy
        if str(strategy).lower() == "auto":
            strategy = "all" if T_ == 1 else "sqrt"
        b = ForestBuilder(K, k * T_, self.maxDepth, self.maxBins, self.minInstancesPerNode, self.minInfoGain,
                          self.impurity, strategy, bootstrap=T_ > 1, seed=self.seed, owner=dp_owner(),
                          subsample=self.subsamplingRate)
        arrs = _fit_sharded(b, X, y, masks.repeat_interleave(T_, dim=0), self.maxBins, self.seed, hybrid)
        return [RandomForestClassificationModel(_slice_arrays(arrs, f * T_, (f + 1) * T_), X.shape[1], K, uid=self.uid,
                                                device=X.device) for f in range(k)]


def _fit_sharded(b: "ForestBuilder", X, y, row_weight, max_bins: int, seed: int, hybrid=None) -> ForestArrays:
    """``b.fit`` over the whole matrix, or — inside ``data_parallel`` — over this rank's
    row shard (thresholds from the whole matrix, so every rank bins identically)."""
    if hybrid is not None and not (X.is_cuda and T.hybrid_tree_ok(hybrid)):
        hybrid = None
    if dp_context() is None:
        return b.fit(X, y, row_weight=row_weight, hybrid=hybrid)
    thr = ((T.thresholds_hybrid_device(hybrid, max_bins, seed=seed) or T.find_thresholds_hybrid(hybrid, max_bins,
                                                                                                seed=seed))
           if hybrid is not None else T.thresholds_for(X, max_bins, seed=seed))
    lo, hi = dp_rows(X.shape[0])
    return b.fit(X[lo:hi], y[lo:hi], row_offset=lo, thresholds=thr, row_weight=row_weight[:, lo:hi],
                 hybrid=None if hybrid is None else hybrid.rows(lo, hi))


def _slice_arrays(a: ForestArrays, lo: int, hi: int) -> ForestArrays:
    return ForestArrays(a.feature[lo:hi], a.threshold[lo:hi], a.left[lo:hi], a.right[lo:hi], a.stats[lo:hi],
                        a.n_nodes[lo:hi], a.max_depth, None if a.gain is None else a.gain[lo:hi])


def _concat_arrays(parts: List[ForestArrays]) -> ForestArrays:
    maxn = max(p.feature.shape[1] for p in parts)

    def pad(t, fill):
        if t.shape[1] == maxn:
            return t
        shape = (t.shape[0], maxn - t.shape[1]) + tuple(t.shape[2:])
        return torch.cat([t, torch.full(shape, fill, dtype=t.dtype, device=t.device)], dim=1)

    dev = parts[0].feature.device
    return ForestArrays(torch.cat([pad(p.feature.to(dev), -1) for p in parts]),
                        torch.cat([pad(p.threshold.to(dev), 0) for p in parts]),
                        torch.cat([pad(p.left.to(dev), 0) for p in parts]),
                        torch.cat([pad(p.right.to(dev), 0) for p in parts]),
                        torch.cat([pad(p.stats.to(dev), 0) for p in parts]),
                        np.concatenate([p.n_nodes for p in parts]), max(p.max_depth for p in parts),
                        torch.cat([pad(p.gain.to(dev), 0) for p in parts]) if all(p.gain is not None for p in parts)
                        else None)


def _arrays_state(a: ForestArrays):
    st = {"feature": a.feature, "threshold": a.threshold, "left": a.left, "right": a.right, "stats": a.stats,
          "n_nodes": torch.as_tensor(a.n_nodes), "max_depth": torch.tensor([a.max_depth])}
    if a.gain is not None:
        st["gain"] = a.gain
    return st


def _arrays_from_state(st) -> ForestArrays:
    return ForestArrays(st["feature"], st["threshold"], st["left"], st["right"], st["stats"], st["n_nodes"].numpy(),
                        int(st["max_depth"][0]), st.get("gain"))


__all__ = ["DecisionTreeClassifier", "RandomForestClassifier", "DecisionTreeClassificationModel",
           "RandomForestClassificationModel", "ForestBuilder", "ForestArrays"]
