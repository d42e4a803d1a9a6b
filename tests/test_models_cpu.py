"""Estimators on the CPU path (the oracles of the GPU paths) + golden accuracy
floors on WISDM from SURVEY.md §4 (LR >= 0.61, DT >= 0.73, RF >= 0.63, LR-CV >= 0.71)."""
import numpy as np
import pytest
import torch

from har.data.csv_io import read_csv
from har.data.split import random_split
from har.evaluation.evaluators import MulticlassClassificationEvaluator, evaluate_all
from har.features import wisdm
from har.models.logreg import FitSpec, LogisticRegression
from har.models.mlp import MLPEngine, MultilayerPerceptronClassifier
from har.models.naive_bayes import NaiveBayes
from har.models.tree import DecisionTreeClassifier, RandomForestClassifier
from har.ops import tree as T
from har.ops.logreg import logreg_loss_grad_torch
from har.optim import lbfgs
from har.tuning.crossval import CrossValidator, ParamGridBuilder


@pytest.fixture(scope="module")
def wisdm_split(wisdm_csv):
    torch.set_num_threads(8)
    _, _, df = wisdm.prepare(read_csv(wisdm_csv), "reference")
    return random_split(df, [0.7, 0.3], 2018)


def _acc(model, table):
    out = model.transform(table)
    return float((out["prediction"].data == out["label"].data).mean())


def _blobs(n=1500, f=8, k=4, seed=0):
    g = torch.Generator().manual_seed(seed)
    mu = torch.randn(k, f, generator=g) * 2
    y = torch.randint(0, k, (n,), generator=g)
    return mu[y] + torch.randn(n, f, generator=g), y


def test_logreg_grad_matches_autograd():
    g = torch.Generator().manual_seed(0)
    N, F, B, K = 200, 7, 3, 5
    X = torch.randn(N, F, dtype=torch.float64, generator=g)
    y = torch.randint(0, K, (N,), generator=g)
    W = torch.randn(B, K, F, dtype=torch.float64, generator=g, requires_grad=True)
    b = torch.randn(B, K, dtype=torch.float64, generator=g, requires_grad=True)
    rw = (torch.rand(B, N, generator=g) > 0.3).double()
    inv = 1 / rw.sum(1)
    loss, gW, gb = logreg_loss_grad_torch(X, y, W.detach(), b.detach(), rw, inv)
    Z = torch.einsum("nf,bkf->nbk", X, W) + b
    ce = torch.logsumexp(Z, 2) - Z.gather(2, y.view(-1, 1, 1).expand(-1, B, 1)).squeeze(2)
    ref = (ce * rw.T * inv).sum(0)
    gWr, gbr = torch.autograd.grad(ref.sum(), (W, b))
    torch.testing.assert_close(loss, ref.detach())
    torch.testing.assert_close(gW, gWr)
    torch.testing.assert_close(gb, gbr)


def test_lbfgs_quadratic_and_owlqn_sparsity():
    A = torch.diag(torch.tensor([1.0, 10.0, 100.0], dtype=torch.float64))
    c = torch.tensor([1.0, -2.0, 3.0], dtype=torch.float64)

    def f(x):  # two identical problems in a batch
        v = 0.5 * (x @ A * x).sum(1) - x @ c
        return v, x @ A - c
    r = lbfgs.minimize(f, torch.zeros(2, 3, dtype=torch.float64), max_iter=50, tol=1e-12)
    torch.testing.assert_close(r.x[0], torch.linalg.solve(A, c), rtol=1e-6, atol=1e-8)
    l1 = torch.tensor([[0.0, 0.0, 0.0], [5.0, 5.0, 5.0]], dtype=torch.float64)
    r = lbfgs.minimize(f, torch.zeros(2, 3, dtype=torch.float64), max_iter=100, tol=1e-12, l1=l1)
    # with a strong L1 term the first two coordinates are exactly zero (soft threshold)
    assert r.x[1, 0] == 0 and r.x[1, 1] == 0 and abs(float(r.x[1, 2]) - (3 - 5) / 100) < 1e-6 or \
        float(r.x[1, 2]) == 0.0


def test_logreg_wisdm_reference(wisdm_split):
    tr, te = wisdm_split
    m = LogisticRegression(maxIter=20, regParam=0.3, elasticNetParam=0).fit(tr)
    assert _acc(m, te) >= 0.61
    assert m.coefficientMatrix.shape == (6, 3100)
    assert abs(float(m.interceptVector.sum())) < 1e-5  # centered intercepts (multinomial)
    assert float(m.coefficientMatrix[:, 3090].abs().max()) == 0.0  # XAVG has std 0 -> zero coefficient


def test_logreg_binomial():
    x, y = _blobs(1000, 5, 2)
    m = LogisticRegression(maxIter=100, regParam=0.01).fit_many(x, y, [FitSpec(None, 0.01, 0.0)], 2)[0]
    assert m.binomial and m.coefficientMatrix.shape == (1, 5)
    assert float((m.predict(x) == y).float().mean()) > 0.9
    p = m.predict_all(x)[1]
    torch.testing.assert_close(p.sum(1), torch.ones(1000))


def test_crossvalidator_lr_batched(wisdm_split):
    tr, te = wisdm_split
    lr = LogisticRegression(maxIter=20)
    grid = ParamGridBuilder().addGrid("regParam", [0.1, 0.3, 0.5]).addGrid("elasticNetParam", [0.0, 0.1, 0.2]).build()
    assert len(grid) == 9
    cv = CrossValidator(estimator=lr, estimatorParamMaps=grid,
                        evaluator=MulticlassClassificationEvaluator(metricName="accuracy"), numFolds=5, seed=2018)
    m = cv.fit(tr)
    assert len(m.avgMetrics) == 9
    assert _acc(m, te) >= 0.70


def test_decision_tree_wisdm(wisdm_split):
    tr, te = wisdm_split
    m = DecisionTreeClassifier(maxDepth=3).fit(tr)
    assert m.numNodes == 15 and m.depth == 3  # result.txt:231
    assert _acc(m, te) >= 0.72
    imp = m.featureImportances
    assert abs(float(imp.sum()) - 1.0) < 1e-9


def test_random_forest_wisdm(wisdm_split):
    tr, te = wisdm_split
    m = RandomForestClassifier(numTrees=100, maxDepth=4, maxBins=32, seed=2018).fit(tr)
    assert m.getNumTrees == 100
    assert _acc(m, te) >= 0.62
    raw = m.predict_raw(torch.as_tensor(te["features"].data[:10]))
    torch.testing.assert_close(raw.sum(1), torch.full((10,), 100.0))  # soft vote of normalized leaves


def test_split_from_hist_bruteforce():
    g = torch.Generator().manual_seed(0)
    hist = torch.randint(0, 5, (2, 3, 8, 3), generator=g).double()
    feats = torch.tensor([[0, 1, 2], [3, 4, 5]], dtype=torch.int32)
    nb = torch.tensor([8, 5, 2, 8, 8, 1], dtype=torch.int32)
    res = T.split_from_hist(hist, feats, nb, 1.0, 0.0, T.GINI)
    for a in range(2):
        best = (-1e9, None)
        tot = hist[a, 0].sum(0)
        for s in range(3):
            for b in range(int(nb[feats[a, s]]) - 1):
                L = hist[a, s, : b + 1].sum(0)
                R = tot - L
                if L.sum() < 1 or R.sum() < 1:
                    continue
                gi = lambda c: 1 - ((c / c.sum()) ** 2).sum()  # noqa: E731
                gain = gi(tot) - L.sum() / tot.sum() * gi(L) - R.sum() / tot.sum() * gi(R)
                if gain > best[0] + 1e-12:
                    best = (float(gain), (int(feats[a, s]), b))
        assert (int(res.feat[a]), int(res.bin[a])) == best[1]
        assert abs(float(res.gain[a]) - best[0]) < 1e-6


def test_naive_bayes_vs_sklearn():
    from sklearn.naive_bayes import GaussianNB, MultinomialNB

    x, y = _blobs(800, 6, 3, seed=1)
    g = NaiveBayes(modelType="gaussian").fit_tensors(x, y, 3)
    sk = GaussianNB(var_smoothing=1e-9).fit(x.numpy(), y.numpy())
    agree = (g.predict(x).numpy() == sk.predict(x.numpy())).mean()
    assert agree > 0.99
    xa = x.abs()
    m = NaiveBayes(modelType="multinomial", smoothing=1.0).fit_tensors(xa, y, 3)
    skm = MultinomialNB(alpha=1.0).fit(xa.numpy(), y.numpy())
    np.testing.assert_allclose(m.theta.numpy(), skm.feature_log_prob_, rtol=1e-4)
    with pytest.raises(ValueError):
        NaiveBayes(modelType="multinomial").fit_tensors(x, y, 3)  # negative features


def test_naive_bayes_gaussian_large_mean_variance():
    """Two-pass variance: a feature offset by 1e4 (fp32 E[x^2]-mu^2 would lose ~all digits)."""
    x, y = _blobs(600, 4, 3, seed=3)
    g0 = NaiveBayes(modelType="gaussian").fit_tensors(x, y, 3)
    g1 = NaiveBayes(modelType="gaussian").fit_tensors(x + 1.0e4, y, 3)
    np.testing.assert_allclose(g1.sigma.numpy(), g0.sigma.numpy(), rtol=2e-3)


def test_mlp_cpu_trains():
    x, y = _blobs(2048, 43, 6, seed=2)
    m = MultilayerPerceptronClassifier(layers=[43, 64, 64, 6], maxIter=15, blockSize=256, stepSize=3e-3,
                                       device="cpu").fit_tensors(x, y)
    assert float((m.predict(x) == y).float().mean()) > 0.95


def test_mlp_flat_layout():
    eng = MLPEngine([43, 64, 96, 6], 128, "cpu")
    L = eng.layout
    assert L.in_pad == 64 and L.view(eng.P, "W0").shape == (64, 64) and L.view(eng.P, "Wout").shape == (32, 96)
    assert float(L.view(eng.P, "W0")[:, 43:].abs().max()) == 0.0
    assert float(L.view(eng.P, "Wout")[6:].abs().max()) == 0.0
    assert all(s.offset % 64 == 0 for s in L.segments)


def test_tree_cv_folds_batched_equal_per_fold():
    """The fold-batched build (fold masks x bootstrap weights, one lock-step forest) gives, for
    a decision tree, exactly the tree fitted on that fold's rows with the same split candidates."""
    from har.data.split import kfold_ids

    X, y = _blobs(900, 8, 3, seed=4)
    fold = torch.as_tensor(kfold_ids(900, 3, 7))
    masks = torch.stack([(fold != f).float() for f in range(3)])
    thr = T.find_thresholds(X.numpy(), 32)
    dt = DecisionTreeClassifier(maxDepth=4, device="cpu")
    batched = dt.fit_folds(X, y, 3, masks)
    for f in range(3):
        keep = fold != f
        single = dt.fit_tensors(X[keep], y[keep], 3, thresholds=thr)
        assert torch.equal(batched[f].arrs.feature, single.arrs.feature)
        torch.testing.assert_close(batched[f].predict_raw(X), single.predict_raw(X))
    rfs = RandomForestClassifier(numTrees=6, maxDepth=4, seed=1, device="cpu").fit_folds(X, y, 3, masks)
    assert len(rfs) == 3 and all(m.arrs.feature.shape[0] == 6 for m in rfs)
    assert all(float((m.predict(X) == y).float().mean()) > 0.8 for m in rfs)


def test_crossvalidator_trees(wisdm_split):
    train, test = wisdm_split
    ev = MulticlassClassificationEvaluator(metricName="accuracy")
    cv = CrossValidator(estimator=DecisionTreeClassifier(maxDepth=3, device="cpu"),
                        estimatorParamMaps=ParamGridBuilder().addGrid("maxDepth", [2, 3]).build(), evaluator=ev,
                        numFolds=5, seed=3).fit(train)
    assert len(cv.avgMetrics) == 2 and cv.bestIndex == 1 and cv.avgMetrics[1] > 0.6
    assert _acc(cv, test) > 0.6


def test_find_thresholds_device_equals_numpy():
    """Device findSplits (one sort of the sampled columns) == the NumPy oracle, threshold for
    threshold: ties, NaNs, constant columns, few / many distinct values, sampled and not."""
    rng = np.random.default_rng(0)
    for trial in range(24):
        N, F = int(rng.integers(1, 25000)), int(rng.integers(1, 10))
        X = rng.normal(size=(N, F)).astype(np.float32)
        for f in range(F):
            if trial % 4 == 1:
                X[:, f] = np.round(X[:, f] * rng.integers(1, 20))
            if trial % 4 == 2:
                X[rng.random(N) < 0.3, f] = np.nan
            if trial % 4 == 3 and f == 0:
                X[:, f] = 1.0
        mb = int(rng.choice([2, 4, 16, 32, 64]))
        a = T.find_thresholds(X, mb, 10000, seed=trial)
        b = T.find_thresholds_device(torch.from_numpy(X), mb, 10000, seed=trial)
        for f in range(F):
            assert b[f].dtype == np.float32 and np.array_equal(a[f], b[f]), (trial, f)


def test_threshold_sample_is_shard_invariant():
    """The findSplits row sample is keyed by global row id: the shards' samples concatenate
    into the single-process sample, and its size is close to max(maxBins^2, 10000)."""
    N = 60000
    full = T.threshold_sample_mask(N, 32, 10000, seed=7)
    bounds = [0, 7001, 30000, 45555, N]
    parts = [T.threshold_sample_mask(b - a, 32, 10000, seed=7, row_offset=a, n_total=N)
             for a, b in zip(bounds[:-1], bounds[1:])]
    assert np.array_equal(full, np.concatenate(parts))
    assert 9500 < full.sum() < 10500
    assert T.threshold_sample_mask(9000, 32, 10000) is None


def test_random_forest_subsampling_rate():
    """subsamplingRate (Spark BaggedPoint): a forest draws Poisson(rate) counts per (tree, row),
    one tree Bernoulli(rate); the draws come from one CDF table shared with the device kernel."""
    import numpy as np

    from har.models.tree import ForestBuilder, RandomForestClassifier
    from har.ops import rng

    b = ForestBuilder(3, num_trees=40, subsample=0.5, seed=3)
    w = b.bootstrap_weights(20000, torch.device("cpu")).numpy()
    assert abs(w.mean() - 0.5) < 0.01 and abs(w.var() - 0.5) < 0.02  # Poisson(0.5): mean = var = 0.5
    one = ForestBuilder(3, num_trees=1, subsample=0.3, seed=3).bootstrap_weights(20000, torch.device("cpu")).numpy()
    assert set(np.unique(one)) <= {0, 1} and abs(one.mean() - 0.3) < 0.01
    assert np.array_equal(ForestBuilder(3, num_trees=5, seed=3).cdf, rng.POISSON1_THR)  # rate 1 unchanged
    g = torch.Generator().manual_seed(1)
    X = torch.randn(600, 6, generator=g)
    y = (X[:, 0] > 0).long() + (X[:, 1] > 0.5).long()
    m = RandomForestClassifier(numTrees=10, maxDepth=4, subsamplingRate=0.6, seed=2).fit_tensors(X, y, 3)
    assert float((m.predict(X) == y).float().mean()) > 0.8
    with pytest.raises(ValueError):
        ForestBuilder(3, num_trees=2, subsample=1.5)


def test_classification_thresholds():
    """Spark thresholds: argmax of p / t; a zero threshold wins wherever its probability is > 0;
    binary LogisticRegression(threshold=t) == thresholds [1 - t, t]."""
    from har.models.logreg import LogisticRegression

    g = torch.Generator().manual_seed(0)
    X = torch.randn(800, 4, generator=g)
    y = (X[:, 0] + 0.3 * torch.randn(800, generator=g) > 0).long()
    base = LogisticRegression(maxIter=30, device="cpu").fit_many(X, y, [FitSpec(None, 0.0, 0.0)], 2)[0]
    raw, prob, pred = base.predict_all(X)
    assert torch.equal(pred, torch.argmax(prob, 1))
    strict = LogisticRegression(maxIter=30, device="cpu", threshold=0.9)
    m = strict._apply_thresholds(base)
    _, prob2, pred2 = m.predict_all(X)
    assert torch.equal(pred2, (prob2[:, 1] > 0.9).long())
    assert int(pred2.sum()) < int(pred.sum())
    m.setThresholds([0.0, 1.0])  # class 0 wins wherever p0 > 0
    _, p3, pred3 = m.predict_all(X)
    assert int(pred3[p3[:, 0] > 0].sum()) == 0 and bool((pred3[p3[:, 0] == 0] == 1).all())
    with pytest.raises(ValueError):
        m.setThresholds([0.0, 0.0])


def test_logreg_checkpoint_resume(tmp_path, monkeypatch):
    """A finished LR fit batch is checkpointed under its fingerprint; a rerun (restarted job)
    loads it without solving and returns the same models; other parameters refit."""
    from har.models import logreg as lr_mod
    from har.models.logreg import FitSpec, LogisticRegression

    g = torch.Generator().manual_seed(4)
    X = torch.randn(500, 5, generator=g)
    y = torch.randint(0, 3, (500,), generator=g)
    specs = [FitSpec(None, 0.1, 0.0), FitSpec(None, 0.05, 0.5)]
    ck = str(tmp_path / "lr")
    a = LogisticRegression(maxIter=20, device="cpu", checkpointDir=ck).fit_many(X, y, specs, 3)

    def boom(*args, **kw):
        raise AssertionError("resumed fit must not solve again")

    monkeypatch.setattr(lr_mod.LogisticRegression, "_setup", boom)
    b = LogisticRegression(maxIter=20, device="cpu", checkpointDir=ck).fit_many(X, y, specs, 3)
    for ma, mb in zip(a, b):
        assert torch.equal(ma.coefficientMatrix, mb.coefficientMatrix)
        assert torch.equal(ma.interceptVector, mb.interceptVector)
        assert mb.summary["resumed"] and mb.summary["iterations"] == ma.summary["iterations"]
    with pytest.raises(AssertionError):  # a different fit (maxIter) is not resumed from the stale checkpoint
        LogisticRegression(maxIter=21, device="cpu", checkpointDir=ck).fit_many(X, y, specs, 3)


def test_crossvalidator_scores_with_thresholds():
    """CV folds are scored as model.transform would predict them: a LogisticRegression(threshold=t)
    inside CrossValidator is scored at t, not at 0.5 (Spark scores folds through transform)."""
    from har.data.table import Column, Table
    from har.tuning.crossval import _batched_predictions

    g = torch.Generator().manual_seed(3)
    X = torch.randn(900, 3, generator=g)
    y = (X[:, 0] + 0.8 * torch.randn(900, generator=g) > 0).long()
    lr = LogisticRegression(maxIter=25, device="cpu", threshold=0.85)
    models = lr.fit_many(X, y, [FitSpec(None, 0.0, 0.0), FitSpec(None, 0.1, 0.0)], 2)
    raw = torch.stack([m.predict_raw(X) for m in models])
    pred = _batched_predictions(models, raw)
    for m, p in zip(models, pred):
        assert torch.equal(p, m.predict(X))
    assert int(pred.sum()) < int(torch.argmax(raw, 2).sum())  # the threshold moved predictions
    t = Table([Column("features", "vector", X.numpy().astype(np.float64)),
               Column("label", "double", y.numpy().astype(np.float64))])
    ev = MulticlassClassificationEvaluator(metricName="accuracy")
    plain = CrossValidator(estimator=LogisticRegression(maxIter=25, device="cpu"), evaluator=ev, numFolds=3,
                           seed=1).fit(t)
    strict = CrossValidator(estimator=lr, evaluator=ev, numFolds=3, seed=1).fit(t)
    assert strict.avgMetrics[0] < plain.avgMetrics[0]


def test_logreg_checkpoint_keys_on_content(tmp_path):
    """The LR checkpoint fingerprint carries the data content and the fold masks: a rerun on other
    data of the same shape / label sum, or with other fold masks, does not resume a stale fit; fits
    with different fingerprints in one directory do not overwrite each other."""
    g = torch.Generator().manual_seed(5)
    X = torch.randn(400, 4, generator=g)
    y = torch.randint(0, 3, (400,), generator=g)
    ck = str(tmp_path / "lr")
    w1 = (torch.arange(400) % 5 != 0).float()
    w2 = (torch.arange(400) % 5 != 1).float()
    lr = LogisticRegression(maxIter=15, device="cpu", checkpointDir=ck)
    a = lr.fit_many(X, y, [FitSpec(w1, 0.1, 0.0)], 3)[0]
    b = lr.fit_many(X, y, [FitSpec(w2, 0.1, 0.0)], 3)[0]      # other fold mask: solved, not resumed
    assert not b.summary.get("resumed")
    X2 = X.clone()
    X2[0, 0] += 1.0                                            # same shape and labels, other content
    c = lr.fit_many(X2, y, [FitSpec(w1, 0.1, 0.0)], 3)[0]
    assert not c.summary.get("resumed")
    a2 = lr.fit_many(X, y, [FitSpec(w1, 0.1, 0.0)], 3)[0]     # the first fit is still there
    assert a2.summary.get("resumed") and torch.equal(a2.coefficientMatrix, a.coefficientMatrix)
    with pytest.raises(ValueError):
        LogisticRegression(lineSearchTrials=5)


def test_crossvalidator_batched_refit_matches_plain_fit():
    """The CrossValidator's best model comes from the batched solve (the 9 candidates' full-data
    refits ride along with the 45 fold fits).  Its fp summation order differs from a separate
    ``est.copy(best_map).fit(table)``, so the two agree within tolerance, not bitwise: the same
    objective to 1e-4 relative and > 99% identical predictions."""
    from har.data.table import Column, Table

    x, y = _blobs(1200, 10, 4, seed=5)
    t = Table([Column("features", "vector", x.numpy().astype(np.float32)),
               Column("label", "double", y.numpy().astype(np.float64))])
    lr = LogisticRegression(maxIter=30)
    grid = ParamGridBuilder().addGrid("regParam", [0.05, 0.2]).addGrid("elasticNetParam", [0.0, 0.1]).build()
    cv = CrossValidator(estimator=lr, estimatorParamMaps=grid,
                        evaluator=MulticlassClassificationEvaluator(metricName="accuracy"), numFolds=3, seed=1)
    m = cv.fit(t)
    plain = lr.copy(grid[m.bestIndex]).fit(t)
    fa, fb = m.bestModel.summary["objective"], plain.summary["objective"]
    assert abs(fa - fb) / abs(fb) < 1e-4, (fa, fb)
    agree = float((m.bestModel.predict(x) == plain.predict(x)).float().mean())
    assert agree > 0.99, agree


def test_logreg_per_model_objective_history():
    """Every model of a batched fit reports its own objective trajectory (not the batch mean)."""
    x, y = _blobs(600, 6, 3, seed=2)
    specs = [FitSpec(None, 0.01, 0.0), FitSpec(None, 1.0, 0.0)]
    ms = LogisticRegression(maxIter=15).fit_many(x, y, specs, 3)
    h0, h1 = ms[0].summary["objectiveHistory"], ms[1].summary["objectiveHistory"]
    assert len(h0) >= 2 and h0 != h1
    assert abs(h0[-1] - ms[0].summary["objective"]) < 1e-6 * max(1.0, abs(h0[-1]))
    assert abs(h1[-1] - ms[1].summary["objective"]) < 1e-6 * max(1.0, abs(h1[-1]))
    assert all(b <= a + 1e-9 for a, b in zip(h0, h0[1:]))  # monotone (Armijo steps only)


def test_logreg_many_classes_cpu():
    """More classes than the device kernels' 16 class rows: the same estimator fits them."""
    x, y = _blobs(2000, 12, 18, seed=3)
    m = LogisticRegression(maxIter=60, regParam=0.001).fit_many(x, y, [FitSpec(None, 0.001, 0.0)], 18)[0]
    assert m.coefficientMatrix.shape == (18, 12)
    assert float((m.predict(x) == y).float().mean()) > 0.8


@pytest.mark.parametrize("model_type", ["multinomial", "gaussian"])
def test_naive_bayes_crossvalidator_fold_masks_match_row_subsets(model_type):
    """CrossValidator over NaiveBayes fits every fold from the full matrix with the fold mask as row
    weights (``NaiveBayes.fit_folds``) and scores the folds in one batched pass; the metrics equal the
    per-fold row-subset fits (``take_rows``) of the generic loop."""
    from har.data.split import kfold_ids
    from har.data.table import Column, Table
    from har.tuning.crossval import CrossValidator, ParamGridBuilder

    x, y = _blobs(900, 8, 3, seed=4)
    x = x.abs() if model_type == "multinomial" else x
    t = Table([Column("features", "vector", x.numpy().astype(np.float32)),
               Column("label", "double", y.numpy().astype(np.float64))])
    nb = NaiveBayes(modelType=model_type)
    grid = ParamGridBuilder().addGrid("smoothing", [0.5, 1.0]).build()
    ev = MulticlassClassificationEvaluator(metricName="accuracy")
    cv = CrossValidator(estimator=nb, estimatorParamMaps=grid, evaluator=ev, numFolds=3, seed=2).fit(t)
    fold = kfold_ids(t.count(), 3, 2)
    want = []
    for pm in grid:
        vals = []
        for f in range(3):
            tr, va = t.take_rows(np.nonzero(fold != f)[0]), t.take_rows(np.nonzero(fold == f)[0])
            vals.append(ev.evaluate(nb.copy(pm).fit(tr).transform(va)))
        want.append(float(np.mean(vals)))
    np.testing.assert_allclose(cv.avgMetrics, want, rtol=0, atol=1e-9)


def test_mlp_crossvalidator_device_fold_rows_match_row_subsets():
    """CrossValidator over the MLP gathers each fold's training rows on the device
    (``fit_folds``) instead of building host row subsets; same rows, same order, same model."""
    from har.data.split import kfold_ids
    from har.data.table import Column, Table

    x, y = _blobs(600, 8, 3, seed=5)
    t = Table([Column("features", "vector", x.numpy().astype(np.float32)),
               Column("label", "double", y.numpy().astype(np.float64))])
    mlp = MultilayerPerceptronClassifier(layers=[8, 32, 3], maxIter=3, blockSize=64, stepSize=1e-2, device="cpu")
    grid = ParamGridBuilder().addGrid("stepSize", [1e-2, 3e-2]).build()
    ev = MulticlassClassificationEvaluator(metricName="f1")
    cv = CrossValidator(estimator=mlp, estimatorParamMaps=grid, evaluator=ev, numFolds=3, seed=1).fit(t)
    fold = kfold_ids(t.count(), 3, 1)
    want = []
    for pm in grid:
        vals = [ev.evaluate(mlp.copy(pm).fit(t.take_rows(np.nonzero(fold != f)[0]))
                            .transform(t.take_rows(np.nonzero(fold == f)[0]))) for f in range(3)]
        want.append(float(np.mean(vals)))
    np.testing.assert_allclose(cv.avgMetrics, want, rtol=0, atol=1e-6)


def test_native_solver_histories_equal_per_model_history():
    """DeviceLogregSolver.histories (one host conversion for every model) == history(b) per model:
    trailing repeats of the final value dropped, interior repeats (a rejected line-search round) kept."""
    from types import SimpleNamespace

    from har.ops.logreg import DeviceLogregSolver

    hist = torch.tensor([[5.0, 4.0, 9.0], [3.0, 4.0, 8.0], [3.0, 2.0, 8.0], [2.0, 2.0, 8.0], [2.0, 2.0, 8.0]],
                        dtype=torch.float64)
    ns = SimpleNamespace(hist=hist, hist_rows=4)
    many = DeviceLogregSolver.histories(ns, hist)
    assert many == [DeviceLogregSolver.history(ns, b, hist) for b in range(3)]
    assert many == [[5.0, 3.0, 3.0, 2.0], [4.0, 4.0, 2.0], [9.0, 8.0]]
