"""Philox oracle + metric definitions vs scikit-learn."""
import numpy as np
import pytest
import torch

from har.evaluation import metrics as M
from har.evaluation.evaluators import evaluate_all
from har.ops import rng


def _philox_raw(ctr, key):
    M0, M1 = 0xD2511F53, 0xCD9E8D57
    c = list(ctr)
    k0, k1 = key
    for r in range(10):
        if r:
            k0, k1 = (k0 + 0x9E3779B9) & 0xFFFFFFFF, (k1 + 0xBB67AE85) & 0xFFFFFFFF
        p0, p1 = M0 * c[0], M1 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & 0xFFFFFFFF, p1 & 0xFFFFFFFF, ((p0 >> 32) ^ c[3] ^ k1) & 0xFFFFFFFF,
             p0 & 0xFFFFFFFF]
    return c


def test_philox_known_answer():
    # Random123 KAT for philox4x32-10: ctr = key = 0
    assert _philox_raw((0, 0, 0, 0), (0, 0)) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    idx = np.array([0, 1, 2 ** 33 + 5], dtype=np.uint64)
    out = rng.philox4x32(0x1234_5678_9ABC, 7, idx)
    for i, x in enumerate(idx):
        ref = _philox_raw((int(x) & 0xFFFFFFFF, int(x) >> 32, 7, rng.TAG), (0x5678_9ABC, 0x1234))
        assert list(map(int, out[i])) == ref


def test_poisson_and_subsets():
    w = rng.poisson1_weights(3, range(4), 50000)
    assert abs(w.mean() - 1.0) < 0.02 and abs(w.var() - 1.0) < 0.05
    s = rng.feature_subsets(9, [0, 0, 1], [0, 5, 0], 3100, 56)
    assert s.shape == (3, 56)
    for row in s:
        assert len(set(row.tolist())) == 56 and (np.diff(row) > 0).all() and row.max() < 3100
    np.testing.assert_array_equal(s, rng.feature_subsets(9, [0, 0, 1], [0, 5, 0], 3100, 56))


def test_multiclass_vs_sklearn():
    from sklearn.metrics import accuracy_score, f1_score, precision_score, recall_score

    g = np.random.default_rng(0)
    y = g.integers(0, 6, 2000)
    p = np.where(g.random(2000) < 0.6, y, g.integers(0, 4, 2000))
    m = M.multiclass_metrics(y, p, 6)
    assert abs(m["accuracy"] - accuracy_score(y, p)) < 1e-12
    assert abs(m["f1"] - f1_score(y, p, average="weighted")) < 1e-12
    assert abs(m["weightedPrecision"] - precision_score(y, p, average="weighted", zero_division=0)) < 1e-12
    assert abs(m["weightedRecall"] - recall_score(y, p, average="weighted")) < 1e-12
    assert m["weightedRecall"] == pytest.approx(m["accuracy"])  # result.txt:166-167 identity


def test_binary_vs_sklearn():
    from sklearn.metrics import auc, precision_recall_curve, roc_auc_score

    g = np.random.default_rng(1)
    lab = g.integers(0, 6, 3000).astype(float)
    score = g.normal(size=3000) + (lab > 0.5) * 0.7
    score = np.round(score, 1)  # ties
    b = M.binary_metrics(score, lab)
    assert abs(b["areaUnderROC"] - roc_auc_score(lab > 0.5, score)) < 1e-9
    prec, rec, _ = precision_recall_curve(lab > 0.5, score)
    assert abs(b["areaUnderPR"] - auc(rec, prec)) < 5e-3  # Spark adds (0, p_first); sklearn (0, 1)


def test_regression_metrics():
    from sklearn.metrics import mean_absolute_error, mean_squared_error, r2_score

    g = np.random.default_rng(2)
    y = g.integers(0, 6, 500).astype(float)
    p = g.integers(0, 6, 500).astype(float)
    r = M.regression_metrics(y, p)
    assert abs(r["mse"] - mean_squared_error(y, p)) < 1e-12
    assert abs(r["rmse"] - np.sqrt(mean_squared_error(y, p))) < 1e-12
    assert abs(r["mae"] - mean_absolute_error(y, p)) < 1e-12
    assert abs(r["r2"] - r2_score(y, p)) < 1e-12


def test_evaluate_all_reference_identities():
    g = np.random.default_rng(3)
    y = torch.as_tensor(g.integers(0, 6, 1625))
    raw = torch.as_tensor(g.normal(size=(1625, 6)))
    pred = raw.argmax(1)
    r = evaluate_all(y, pred, raw, 6)
    assert r.raw_prediction == r.area_under_roc  # result.txt:158,160
    assert r.correct + r.wrong == r.count_total == 1625
    assert r.ratio_correct == pytest.approx(r.accuracy)
    assert r.mse == pytest.approx(r.rmse ** 2)


@pytest.mark.parametrize("metric", ["mse", "rmse", "mae", "r2", "var"])
def test_batched_regression_metrics_match_single(metric):
    """The CrossValidator's batched regression metric (one requested metric, masked rows per model)
    equals the single-model definition on each model's rows."""
    from har.evaluation.metrics import batched_metrics, regression_metrics

    g = torch.Generator().manual_seed(3)
    N, B = 400, 4
    label = torch.randint(0, 6, (N,), generator=g)
    pred = torch.randint(0, 6, (B, N), generator=g)
    mask = torch.rand(B, N, generator=g) < 0.4
    got = batched_metrics(metric, label, pred, mask, 6)
    for b in range(B):
        rows = torch.nonzero(mask[b]).squeeze(1)
        want = regression_metrics(label[rows].numpy(), pred[b, rows].numpy())[metric]
        assert abs(got[b] - want) < 1e-9 * max(1.0, abs(want))


def test_batched_metrics_rejects_out_of_range_labels():
    import pytest

    from har.evaluation.metrics import batched_metrics

    label = torch.tensor([0, 1, 2, 6])
    pred = torch.zeros(2, 4, dtype=torch.long)
    with pytest.raises(ValueError):
        batched_metrics("accuracy", label, pred, torch.ones(2, 4), 6)
