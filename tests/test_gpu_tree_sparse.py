"""One-hot-aware trees on the reference encoding.

The reference grows DecisionTree(depth 3) / RandomForest(100 x depth 4) on a 3,100-wide vector of
three one-hot blocks (934 + 1,401 + 755 binary columns) and 10 numeric columns (``Main/main.py:51-66,
297,478``).  The one-hot-aware path (``ops/tree.py`` find_thresholds_hybrid / bins_hybrid, tree.hip
SPARSE) takes the one-hot columns' 0 | 1 split from their entries instead of a sort, bins from the
hybrid parts and histograms a one-hot column over its nonzeros only (bin 0 = node totals - bin 1).
Every test pins it to the dense path of the same fit: thresholds, bins and whole forests bit for bit.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wisdm_ref(cuda, wisdm_csv):
    from har.suite import load_wisdm

    train, test, _ = load_wisdm(wisdm_csv, "reference", 2018, device=cuda)
    return train, test


def _dense_path(fn):
    from har.ops import tree as T

    old = T.SPARSE_TREES
    T.SPARSE_TREES = False
    try:
        return fn()
    finally:
        T.SPARSE_TREES = old


def _same_arrays(a, b):
    for k in ("feature", "threshold", "left", "right", "stats", "gain"):
        x, y = getattr(a, k), getattr(b, k)
        assert torch.equal(x, y), k
    assert np.array_equal(a.n_nodes, b.n_nodes)


def _synthetic_hybrid(cuda, N=24000, widths=(40, 7, 3), Fd=5, seed=0, all_ones_block=False):
    """A hybrid matrix with some one-hot columns absent (no 1 in any row), the last category dropped
    (-1 rows) and, optionally, a block whose first column is set in every row (no split)."""
    from har.features.hybrid import HybridMatrix

    g = torch.Generator().manual_seed(seed)
    blocks, off, cats = [], 0, []
    for i, w in enumerate(widths):
        c = torch.randint(-1, w - 2, (N,), generator=g)  # columns w-2, w-1 never set
        if all_ones_block and i == len(widths) - 1:
            c = torch.zeros(N, dtype=torch.int64)
        cats.append(torch.where(c >= 0, c + off, c).to(torch.int32))
        blocks.append((off, w))
        off += w
    dense = torch.randn(N, Fd, generator=g)
    dense[:, 0] = torch.randint(0, 4, (N,), generator=g).float()  # few distinct values: midpoints
    dense[::97, 1] = float("nan")
    dense_cols = torch.arange(off, off + Fd, dtype=torch.int32)
    hm = HybridMatrix(dense.to(cuda), dense_cols.to(cuda), torch.stack(cats, 1).contiguous().to(cuda), blocks, off + Fd)
    y = (cats[0] % 3 + (dense[:, 2] > 0).to(torch.int32)).long().clamp_max(3).to(cuda)
    return hm, y


@pytest.mark.parametrize("n,sample", [(3853, False), (24000, True)])
def test_hybrid_thresholds_and_bins_equal_dense(cuda, n, sample):
    from har.ops import tree as T
    from har.ops.stats import bin_features

    hm, _ = _synthetic_hybrid(cuda, N=n, seed=n)
    X = hm.to_dense()
    assert (T.threshold_sample_weights(n, 32) is not None) == sample
    for mb in (32, 2, 5):
        a = T.find_thresholds_hybrid(hm, mb, seed=7)
        b = T.ThresholdTable.from_any(T.find_thresholds_device(X, mb, seed=7))
        assert np.array_equal(a.counts, b.counts)
        w = max(a.mat.shape[1], b.mat.shape[1])
        assert np.array_equal(a.padded(w), b.padded(w))
        nb = torch.from_numpy((a.counts + 1).astype(np.int32)).to(cuda)
        thr = torch.from_numpy(a.padded(mb)).to(cuda)
        assert torch.equal(T.bins_hybrid(hm, thr, nb), bin_features(X, a))
        # the device-resident version (no host round trip): the same padded matrix and bin counts
        d = T.thresholds_hybrid_device(hm, mb, seed=7)
        assert d is not None
        assert torch.equal(d.nbins, nb) and torch.equal(d.thr_mat, thr)


def test_hybrid_all_ones_column_has_no_split(cuda):
    from har.ops import tree as T

    hm, _ = _synthetic_hybrid(cuda, N=3000, all_ones_block=True)
    tt = T.find_thresholds_hybrid(hm, 32)
    off, w = hm.blocks[-1]
    assert tt.counts[off] == 0  # every row holds it: one distinct value
    assert (tt.counts[off + w - 2:off + w] == 0).all()  # never set
    ref = T.ThresholdTable.from_any(T.find_thresholds_device(hm.to_dense(), 32))
    assert np.array_equal(tt.counts, ref.counts)


@pytest.mark.parametrize("kind", ["dt", "dt7", "rf", "rf_sub"])
def test_sparse_forest_equals_dense_synthetic(cuda, kind):
    from har.models.tree import DecisionTreeClassifier, RandomForestClassifier

    hm, y = _synthetic_hybrid(cuda, N=12000, seed=3)
    X = hm.to_dense()
    est = {"dt": lambda: DecisionTreeClassifier(maxDepth=3),
           "dt7": lambda: DecisionTreeClassifier(maxDepth=7, minInstancesPerNode=3),
           "rf": lambda: RandomForestClassifier(numTrees=20, maxDepth=5, seed=11),
           "rf_sub": lambda: RandomForestClassifier(numTrees=8, maxDepth=6, seed=2, subsamplingRate=0.6,
                                                    featureSubsetStrategy="onethird")}[kind]
    m = est().fit_tensors(X, y, 4, hybrid=hm)
    r = _dense_path(lambda: est().fit_tensors(X, y, 4))
    _same_arrays(m.arrs, r.arrs)


def test_sparse_reference_suite_fits_equal_dense(wisdm_ref):
    """The reference's DecisionTree(depth 3) and RandomForest(100 x depth 4) on WISDM: the
    one-hot-aware fits (eager, graph capture, graph replay) grow the dense path's forests."""
    from har.models import tree as tr
    from har.models.tree import DecisionTreeClassifier, RandomForestClassifier

    train, test = wisdm_ref
    tr._fit_graphs.clear()  # (a full graph cache would keep the capture from happening)
    tr._fit_graph_seen.clear()
    for make in (lambda: DecisionTreeClassifier(featuresCol="features", labelCol="label", maxDepth=3, maxBins=32),
                 lambda: RandomForestClassifier(featuresCol="features", labelCol="label", numTrees=100, maxDepth=4,
                                                maxBins=32, seed=2018)):
        ref = _dense_path(lambda: make().fit(train))
        est = make()
        assert est._hybrid(train, ref.device) is not None, "the reference encoding must take the sparse path"
        kinds = []
        for _ in range(3):  # eager, capture, replay
            m = est.fit(train)
            kinds.append(tr.LAST_FIT_KIND)
            _same_arrays(m.arrs, ref.arrs)
        assert kinds == ["eager", "capture", "replay"], kinds
        Xt = m.features_input(test)
        assert torch.equal(m.predict(Xt), ref.predict(Xt))


def test_sparse_tree_cross_validation_equals_dense(wisdm_ref):
    """DT-CV / RF-CV (fit_folds: every fold's trees in one build) on the reference encoding."""
    from har.evaluation.evaluators import MulticlassClassificationEvaluator
    from har.models.tree import DecisionTreeClassifier, RandomForestClassifier
    from har.tuning.crossval import CrossValidator, ParamGridBuilder

    train, _ = wisdm_ref
    for base, grid in ((DecisionTreeClassifier(maxDepth=3), ParamGridBuilder().addGrid("maxDepth", [2, 3]).build()),
                       (RandomForestClassifier(numTrees=10, maxDepth=3, seed=5),
                        ParamGridBuilder().addGrid("numTrees", [5, 10]).build())):
        def cv():
            return CrossValidator(estimator=base, estimatorParamMaps=grid,
                                  evaluator=MulticlassClassificationEvaluator(metricName="accuracy"),
                                  numFolds=3, seed=7).fit(train)

        a = cv()
        b = _dense_path(cv)
        assert a.avgMetrics == b.avgMetrics
        _same_arrays(a.bestModel.arrs, b.bestModel.arrs)
