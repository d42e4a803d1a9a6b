"""Device logistic regression (csrc/kernels/logreg_qn.hip) against its fp32/fp64 PyTorch oracles.

* the fused evaluation + gradient kernels on a HYBRID layout (one-hot index blocks + dense
  columns, per-spec row weights, several trial models) vs ``LogregDesign.eval_torch`` in fp64;
* the prediction-mode margins vs a dense fp64 product;
* the device L-BFGS / OWL-QN solver vs ``optim.lbfgs.minimize_trials`` (same algorithm in torch);
* bitwise determinism of a device fit (no atomics anywhere on the path);
* the WISDM reference-encoding fits (LR, LR CrossValidator) through the public estimators.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _hybrid_problem(dev, N=1500, seed=0, blocks=((0, 40), (40, 25)), Fd=9, K=6):
    from har.features.hybrid import from_dense

    g = torch.Generator().manual_seed(seed)
    F = sum(w for _, w in blocks) + Fd
    X = torch.zeros(N, F)
    y = torch.randint(0, K, (N,), generator=g)
    for off, w in blocks:
        idx = torch.randint(0, w + 1, (N,), generator=g)  # w == dropped last category
        idx = torch.where(torch.rand(N, generator=g) < 0.5, (y * 7) % (w + 1), idx)
        ok = idx < w
        X[torch.nonzero(ok).squeeze(1), off + idx[ok]] = 1.0
    X[:, F - Fd:] = torch.randn(N, Fd, generator=g) + y[:, None].float() * 0.3
    hm = from_dense(X.to(dev), list(blocks))
    assert hm is not None and hm.cat.shape[1] == len(blocks) and hm.dense.shape[1] == Fd
    return X, y, hm


def test_hybrid_eval_kernel_matches_fp64(cuda):
    from har.ops.logreg import DeviceLogregSolver, LogregDesign

    X, y, hm = _hybrid_problem(cuda)
    N, F = X.shape
    K, S, T = 6, 3, 2
    g = torch.Generator().manual_seed(1)
    rw = (torch.rand(S, N, generator=g) > 0.25).float().to(cuda)
    design = LogregDesign(hm, y.to(cuda), rw, K)
    inv_std = (torch.rand(S, F, generator=g) + 0.5).to(cuda)
    pmask = torch.ones(S, K, F + 1, device=cuda)
    pmask[:, :, 3] = 0  # a frozen column
    inv_wsum = 1.0 / rw.sum(1)
    D = K * (F + 1)
    solver = DeviceLogregSolver(design, S, T, 4, inv_std, pmask, inv_wsum, torch.zeros(S, D, device=cuda), None, 1,
                                1e-6)
    xt = torch.randn(S * T, K, F + 1, generator=g).to(cuda) * 0.3
    spec = torch.arange(S * T, device=cuda) // T
    W = xt[:, :, :F] * inv_std[spec][:, None, :] * pmask[spec][:, :, :F]
    solver.weff.zero_()
    solver.weff[:, :F, :K] = W.transpose(1, 2)
    solver.weff[:, F, :K] = xt[:, :, F] * pmask[spec][:, :, F]
    solver._evaluate(1)
    ref_loss, ref_G = LogregDesign(hm, y.to(cuda), rw.double(), K).eval_torch(
        xt.double(), T, inv_std.double(), pmask.double(), inv_wsum.double())
    torch.testing.assert_close(solver.loss, ref_loss, rtol=2e-5, atol=1e-6)
    torch.testing.assert_close(solver.G.double(), ref_G, rtol=2e-4, atol=2e-6)
    assert float(solver.G.view(S * T, K, F + 1)[:, :, 3].abs().max()) == 0.0


@pytest.mark.parametrize("Fd,K", [(43, 6), (70, 12), (16, 3)])
def test_wide_dense_eval_mfma_matches_fp64(cuda, Fd, K):
    """Dense designs wider than the narrow tile run the evaluation's two dense products on the matrix
    cores (fp32 MFMA: margins W^T X^T, gradient R^T X; KP = 8 and 16; one and several 32-column LDS
    chunks, a ragged last chunk): loss and gradient equal the fp64 oracle."""
    from har.ops.logreg import DeviceLogregSolver, LogregDesign

    X, y, hm = _hybrid_problem(cuda, N=1300, seed=Fd, blocks=((0, 12),), Fd=Fd, K=K)
    N, F = X.shape
    S, T = 2, 3
    g = torch.Generator().manual_seed(7)
    rw = (torch.rand(S, N, generator=g) > 0.2).float().to(cuda)
    design = LogregDesign(hm, y.to(cuda), rw, K)
    inv_std = (torch.rand(S, F, generator=g) + 0.5).to(cuda)
    pmask = torch.ones(S, K, F + 1, device=cuda)
    inv_wsum = 1.0 / rw.sum(1)
    D = K * (F + 1)
    solver = DeviceLogregSolver(design, S, T, 4, inv_std, pmask, inv_wsum, torch.zeros(S, D, device=cuda), None, 1,
                                1e-6)
    xt = torch.randn(S * T, K, F + 1, generator=g).to(cuda) * 0.2
    spec = torch.arange(S * T, device=cuda) // T
    W = xt[:, :, :F] * inv_std[spec][:, None, :] * pmask[spec][:, :, :F]
    solver.weff.zero_()
    solver.weff[:, :F, :K] = W.transpose(1, 2)
    solver.weff[:, F, :K] = xt[:, :, F] * pmask[spec][:, :, F]
    solver._evaluate(1)
    ref_loss, ref_G = LogregDesign(hm, y.to(cuda), rw.double(), K).eval_torch(
        xt.double(), T, inv_std.double(), pmask.double(), inv_wsum.double())
    torch.testing.assert_close(solver.loss, ref_loss, rtol=2e-5, atol=1e-6)
    torch.testing.assert_close(solver.G.double(), ref_G, rtol=2e-4, atol=2e-6)


def test_margins_kernel_matches_dense(cuda):
    from har.ops.logreg import logreg_margins_native

    X, y, hm = _hybrid_problem(cuda, N=700, seed=3)
    F = X.shape[1]
    g = torch.Generator().manual_seed(2)
    W = torch.randn(3, F + 1, 8, generator=g)
    W[:, :, 6:] = 0
    out = logreg_margins_native(hm, W.to(cuda), 6, 3)
    ref = torch.einsum("nf,bfk->bnk", X.double(), W[:, :F].double()) + W[:, F].double()[:, None, :]
    torch.testing.assert_close(out.double().cpu(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("alpha", [0.0, 0.4])
def test_device_solver_matches_torch_algorithm(cuda, alpha):
    """The kernels run the algorithm of minimize_trials: same objective after the fit, and the
    same predictions (fp32 differences only)."""
    from har.models.logreg import FitSpec, LogisticRegression

    X, y, hm = _hybrid_problem(cuda, N=2000, seed=5)
    est = LogisticRegression(maxIter=30, regParam=0.05)
    specs = [FitSpec(None, 0.05, alpha), FitSpec((torch.arange(2000) % 5 != 0).float(), 0.02, alpha)]
    cpu = est.fit_many(X, y, specs, 6)
    gpu = est.fit_many(hm, y.to(cuda), [FitSpec(None if s.row_weight is None else s.row_weight.to(cuda),
                                                 s.regParam, s.elasticNetParam) for s in specs], 6)
    for c, gm in zip(cpu, gpu):
        assert abs(c.summary["objective"] - gm.summary["objective"]) <= 2e-4 * max(1.0, abs(c.summary["objective"]))
        agree = (c.predict(X) == gm.predict(hm).cpu()).float().mean()
        assert agree > 0.99
        if alpha > 0:  # OWL-QN leaves exact zeros
            assert int((gm.coefficientMatrix == 0).sum()) > 0


def test_device_fit_is_bitwise_deterministic(cuda):
    from har.models.logreg import FitSpec, LogisticRegression

    _, y, hm = _hybrid_problem(cuda, N=3000, seed=6)
    est = LogisticRegression(maxIter=20, regParam=0.1)
    specs = [FitSpec(None, 0.1, 0.0), FitSpec(None, 0.3, 0.1)]
    a = est.fit_many(hm, y.to(cuda), specs, 6)
    b = est.fit_many(hm, y.to(cuda), specs, 6)
    for m1, m2 in zip(a, b):
        assert torch.equal(m1.coefficientMatrix, m2.coefficientMatrix)
        assert torch.equal(m1.interceptVector, m2.interceptVector)


def test_native_solve_plan_equals_python_loop(cuda, monkeypatch):
    """The whole-solve native call (bind.cpp logreg_solve) enqueues the launch sequence of the Python
    loop in DeviceLogregSolver.solve: bit-identical coefficients, objectives and histories."""
    from har.models.logreg import FitSpec, LogisticRegression

    _, y, hm = _hybrid_problem(cuda, N=3000, seed=8)
    est = LogisticRegression(maxIter=20, regParam=0.1)
    specs = [FitSpec(None, 0.1, 0.0), FitSpec(None, 0.3, 0.1)]
    out = []
    for flag in ("1", "0"):
        monkeypatch.setenv("HAR_LR_NATIVE_SOLVE", flag)
        out.append(est.fit_many(hm, y.to(cuda), specs, 6))
    for m1, m2 in zip(*out):
        assert torch.equal(m1.coefficientMatrix, m2.coefficientMatrix)
        assert torch.equal(m1.interceptVector, m2.interceptVector)
        assert m1.summary["objective"] == m2.summary["objective"]
        assert m1.summary["objectiveHistory"] == m2.summary["objectiveHistory"]


def test_wisdm_reference_lr_and_cv_on_device(cuda, wisdm_csv):
    from har.data.csv_io import read_csv
    from har.data.split import random_split
    from har.evaluation.evaluators import RegressionEvaluator
    from har.features import wisdm
    from har.models.base import features_tensor
    from har.models.logreg import LogisticRegression
    from har.tuning.crossval import CrossValidator, ParamGridBuilder

    _, _, df = wisdm.prepare(read_csv(wisdm_csv), "reference")
    tr, te = random_split(df, [0.7, 0.3], 2018)
    yt = torch.as_tensor(te["label"].data.astype(np.int64), device=cuda)
    lr = LogisticRegression(maxIter=20, regParam=0.3, device=cuda)
    m = lr.fit(tr)
    acc = float((m.predict(m.features_input(te)) == yt).float().mean())
    assert acc >= 0.61
    # the hybrid-layout prediction equals the dense (3100-wide MFMA GEMM) prediction
    dense = m.predict_raw(features_tensor(te, "features", cuda))
    torch.testing.assert_close(m.predict_raw(m.features_input(te)), dense, rtol=1e-4, atol=1e-4)
    grid = ParamGridBuilder().addGrid("regParam", [0.1, 0.3, 0.5]).addGrid("elasticNetParam", [0.0, 0.1, 0.2]).build()
    cv = CrossValidator(estimator=LogisticRegression(maxIter=20, device=cuda), estimatorParamMaps=grid,
                        evaluator=RegressionEvaluator(metricName="mae"), numFolds=5, seed=2018).fit(tr)
    acc_cv = float((cv.bestModel.predict(cv.bestModel.features_input(te)) == yt).float().mean())
    assert acc_cv >= 0.70 and len(cv.avgMetrics) == 9


def test_device_solver_wide_dense_165(cuda):
    """A 165-column all-dense design (the 9-axis feature width) on the device solver — no width cap,
    no host-synced fallback — against the torch algorithm (minimize_trials) on the same data."""
    from har.features.hybrid import from_dense
    from har.models.logreg import FitSpec, LogisticRegression

    g = torch.Generator().manual_seed(11)
    N, F, K = 3000, 165, 12
    mu = torch.randn(K, F, generator=g) * 0.4
    y = torch.randint(0, K, (N,), generator=g)
    X = mu[y] + torch.randn(N, F, generator=g)
    est = LogisticRegression(maxIter=25, regParam=0.01)
    specs = [FitSpec(None, 0.01, 0.0), FitSpec((torch.arange(N) % 4 != 0).float(), 0.02, 0.3)]
    cpu = est.fit_many(X, y, specs, K)
    hm = from_dense(X.to(cuda), [])
    gpu = est.fit_many(hm, y.to(cuda), [FitSpec(None if s.row_weight is None else s.row_weight.to(cuda),
                                                 s.regParam, s.elasticNetParam) for s in specs], K)
    for c, gm in zip(cpu, gpu):
        assert abs(c.summary["objective"] - gm.summary["objective"]) <= 2e-4 * max(1.0, abs(c.summary["objective"]))
        agree = (c.predict(X) == gm.predict(hm).cpu()).float().mean()
        assert agree > 0.99
        assert isinstance(gm.summary["objectiveHistory"], list) and len(gm.summary["objectiveHistory"]) >= 2


def test_device_setup_matches_torch(cuda):
    """The device summarizer + prepare kernels (logreg_setup.hip) == the torch setup: standardization,
    masks, regularization vectors and the initial point, for weighted and unweighted specs."""
    from har.models.logreg import FitSpec, LogisticRegression

    X, y, hm = _hybrid_problem(cuda, N=1800, seed=12)
    specs = [FitSpec(None, 0.1, 0.0), FitSpec((torch.arange(1800) % 3 != 0).float(), 0.3, 0.2)]
    est = LogisticRegression()
    from har.features.hybrid import from_dense

    hm_cpu = from_dense(X, list(hm.blocks))
    c = est._setup(hm_cpu, y, specs, 6, None)
    g = est._setup(hm, y.to(cuda), [FitSpec(None if s.row_weight is None else s.row_weight.to(cuda), s.regParam,
                                            s.elasticNetParam) for s in specs], 6, None)
    torch.testing.assert_close(g[0].summary().cpu()[:1].expand(2, -1) if g[0].S == 1 else g[0].summary().cpu(),
                               c[0].summary(), rtol=1e-12, atol=1e-9)
    for i in (3, 4, 5, 6, 8):  # inv_std, inv_wsum, pmask, l2v, x0
        torch.testing.assert_close(g[i].cpu().reshape(c[i].shape), c[i], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(g[7].cpu(), c[7], rtol=1e-5, atol=1e-6)  # l1v


def test_logreg_more_than_16_classes_on_gpu(cuda):
    """18 classes exceed the device kernels' 16 class rows: the GPU fit runs the torch objective on
    the device with the same L-BFGS algorithm (it used to raise), predictions through the
    dense path, for plain fits and a CrossValidator."""
    from har.data.table import Column, Table
    from har.evaluation.evaluators import MulticlassClassificationEvaluator
    from har.models.logreg import FitSpec, LogisticRegression
    from har.tuning.crossval import CrossValidator, ParamGridBuilder

    g = torch.Generator().manual_seed(4)
    K, N, F = 18, 3000, 16
    mu = torch.randn(K, F, generator=g) * 2
    y = torch.randint(0, K, (N,), generator=g)
    x = mu[y] + torch.randn(N, F, generator=g)
    spec = [FitSpec(None, 0.001, 0.0)]
    mg = LogisticRegression(maxIter=40, device=cuda).fit_many(x.to(cuda), y.to(cuda), spec, K)[0]
    mc = LogisticRegression(maxIter=40, device="cpu").fit_many(x, y, spec, K)[0]
    assert mg.coefficientMatrix.shape == (K, F)
    pg, pc = mg.predict(x.to(cuda)).cpu(), mc.predict(x)
    assert float((pg == pc).float().mean()) > 0.99
    assert float((pg == y).float().mean()) > 0.8
    assert abs(mg.summary["objective"] - mc.summary["objective"]) / abs(mc.summary["objective"]) < 1e-3
    t = Table([Column("features", "vector", x.numpy().astype(np.float32)),
               Column("label", "double", y.numpy().astype(np.float64))])
    grid = ParamGridBuilder().addGrid("regParam", [0.001, 0.01]).build()
    cv = CrossValidator(estimator=LogisticRegression(maxIter=20, device=cuda), estimatorParamMaps=grid,
                        evaluator=MulticlassClassificationEvaluator(metricName="accuracy"), numFolds=3, seed=1).fit(t)
    assert len(cv.avgMetrics) == 2 and cv.bestModel.coefficientMatrix.shape == (K, F)


def test_crossvalidator_batched_refit_matches_plain_fit_gpu(cuda):
    """GPU twin of ``test_models_cpu.py::test_crossvalidator_batched_refit_matches_plain_fit``: the best
    model of the batched device solve (its refit rides in the 54-model batch, ~9 chunks per model, a
    materialized all-ones weight row) against a separate single device fit of the winning parameters:
    the same objective within 1e-4 relative and > 99% identical predictions."""
    from har.data.table import Column, Table
    from har.evaluation.evaluators import MulticlassClassificationEvaluator
    from har.models.logreg import LogisticRegression
    from har.tuning.crossval import CrossValidator, ParamGridBuilder

    g = torch.Generator().manual_seed(5)
    K, F, N = 4, 10, 1200
    mu = torch.randn(K, F, generator=g) * 1.5
    y = torch.randint(0, K, (N,), generator=g)
    x = mu[y] + torch.randn(N, F, generator=g)
    t = Table([Column("features", "vector", x.numpy().astype(np.float32)),
               Column("label", "double", y.numpy().astype(np.float64))])
    lr = LogisticRegression(maxIter=30, device=cuda)
    grid = ParamGridBuilder().addGrid("regParam", [0.05, 0.2]).addGrid("elasticNetParam", [0.0, 0.1]).build()
    cv = CrossValidator(estimator=lr, estimatorParamMaps=grid,
                        evaluator=MulticlassClassificationEvaluator(metricName="accuracy"), numFolds=3, seed=1)
    m = cv.fit(t)
    plain = lr.copy(grid[m.bestIndex]).fit(t)
    fa, fb = m.bestModel.summary["objective"], plain.summary["objective"]
    assert abs(fa - fb) / abs(fb) < 1e-4, (fa, fb)
    xd = x.to(cuda)
    agree = float((m.bestModel.predict(xd) == plain.predict(xd)).float().mean())
    assert agree > 0.99, agree


@pytest.mark.parametrize("specs_kind", ["pair", "wisdm"])
def test_persistent_solve_equals_launch_sequence(cuda, wisdm_csv, specs_kind):
    """The whole solve as ONE cooperative launch (logreg_solve_persistent_kernel: the same phase
    bodies over virtual blocks, grid barriers for the kernel boundaries) is bitwise the launch
    sequence: coefficients, intercepts and objective histories."""
    from har.models.logreg import FitSpec, LogisticRegression
    from har.ops import _native
    from har.ops import logreg as L

    mod = _native.kernels()
    if specs_kind == "pair":
        _, y, hm = _hybrid_problem(cuda, N=3000, seed=9)
        est = LogisticRegression(maxIter=20, regParam=0.1)
        specs, K = [FitSpec(None, 0.1, 0.0), FitSpec(None, 0.3, 0.1)], 6
        y = y.to(cuda)
    else:
        from har.features.hybrid import hybrid_features
        from har.suite import load_wisdm
        from har.models.base import labels_tensor, num_label_classes

        train, _, _ = load_wisdm(wisdm_csv, "reference", 2018, device=cuda)
        hm = hybrid_features(train, "features", cuda)
        y = labels_tensor(train, "label", cuda)
        K = num_label_classes(train, "label", cuda)
        est = LogisticRegression(maxIter=20, regParam=0.3, elasticNetParam=0.8)
        specs = [FitSpec(None, 0.3, 0.8)]
    out, modes = [], []
    old = mod.logreg_set_persistent(1)
    try:
        for mode in (1, 0):
            mod.logreg_set_persistent(mode)
            out.append(est.fit_many(hm, y, specs, K))
            modes.append(L.LAST_SOLVE_MODE)
    finally:
        mod.logreg_set_persistent(old)
    assert modes == [1, 0]
    for m1, m2 in zip(*out):
        assert torch.equal(m1.coefficientMatrix, m2.coefficientMatrix)
        assert torch.equal(m1.interceptVector, m2.interceptVector)
        assert m1.summary["objectiveHistory"] == m2.summary["objectiveHistory"]


def test_persistent_solve_timeout_falls_back_to_the_sequence(cuda):
    """A grid barrier of the persistent solve that runs out of polls raises the timeout flag; the
    fit must not return the unsynchronized results: it is rerun as the launch sequence (mode 3) and
    equals a plain launch-sequence fit bit for bit (the flag was never read)."""
    import warnings

    from har.models.logreg import FitSpec, LogisticRegression
    from har.ops import _native
    from har.ops import logreg as L

    mod = _native.kernels()
    _, y, hm = _hybrid_problem(cuda, N=3000, seed=9)
    est = LogisticRegression(maxIter=20, regParam=0.1)
    specs, K = [FitSpec(None, 0.1, 0.0), FitSpec(None, 0.3, 0.1)], 6
    y = y.to(cuda)
    old, old_lim = mod.logreg_set_persistent(2), mod.logreg_set_spin_limit(1)
    try:
        L.solver_cache_clear()
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            a = est.fit_many(hm, y, specs, K)
        mode_a = L.LAST_SOLVE_MODE
        mod.logreg_set_persistent(0)
        L.solver_cache_clear()
        b = est.fit_many(hm, y, specs, K)
    finally:
        mod.logreg_set_persistent(old)
        mod.logreg_set_spin_limit(old_lim)
        L.solver_cache_clear()
    if mode_a == -1 or mode_a == 0:
        pytest.skip("the persistent solve was not co-resident on this device")
    assert mode_a == 3 and any("timed out" in str(x.message) for x in w), mode_a
    for m1, m2 in zip(a, b):
        assert torch.equal(m1.coefficientMatrix, m2.coefficientMatrix)
        assert torch.equal(m1.interceptVector, m2.interceptVector)


def test_solver_cache_refit_is_bitwise_a_fresh_fit(cuda, wisdm_csv):
    """A repeated fit on the same resident table reuses the cached solver (arena, argument blocks,
    solve plan): its model is bitwise the model of a fit with the cache cleared, and a fit with other
    hyper-parameters in between leaves it unchanged."""
    from har.models.logreg import LogisticRegression
    from har.ops import logreg as L
    from har.suite import load_wisdm

    train, _, _ = load_wisdm(wisdm_csv, "reference", 2018, device=cuda)
    est = LogisticRegression(maxIter=20, regParam=0.3, elasticNetParam=0.8)
    L.solver_cache_clear()
    a = est.fit(train)
    assert len(L._SOLVER_CACHE) == 1
    other = LogisticRegression(maxIter=20, regParam=0.05, elasticNetParam=0.5).fit(train)  # same key, new inputs
    b = est.fit(train)
    assert len(L._SOLVER_CACHE) == 1
    L.solver_cache_clear()
    c = est.fit(train)
    for m in (b, c):
        assert torch.equal(m.coefficientMatrix, a.coefficientMatrix)
        assert torch.equal(m.interceptVector, a.interceptVector)
        assert m.summary["objectiveHistory"] == a.summary["objectiveHistory"]
    assert not torch.equal(other.coefficientMatrix, a.coefficientMatrix)


def test_solver_cache_crossvalidator_repeat_is_bitwise(cuda, wisdm_csv):
    """The CrossValidator's batched weighted fit reuses its cached solver on a repeat (new fold row
    weights copied into the cached design): the same metrics and model as with the cache cleared."""
    from har.evaluation.evaluators import RegressionEvaluator
    from har.models.logreg import LogisticRegression
    from har.ops import logreg as L
    from har.suite import load_wisdm
    from har.tuning.crossval import CrossValidator, ParamGridBuilder

    train, _, _ = load_wisdm(wisdm_csv, "reference", 2018, device=cuda)
    lr = LogisticRegression(maxIter=10)
    grid = ParamGridBuilder().addGrid("regParam", [0.1, 0.3]).addGrid("elasticNetParam", [0.0, 0.5]).build()

    def run(seed):
        return CrossValidator(estimator=lr, estimatorParamMaps=grid, evaluator=RegressionEvaluator(metricName="mae"),
                              numFolds=3, seed=seed).fit(train)

    L.solver_cache_clear()
    a = run(1)
    run(5)  # other folds through the cached solver
    b = run(1)
    L.solver_cache_clear()
    c = run(1)
    for m in (b, c):
        assert m.avgMetrics == a.avgMetrics
        assert torch.equal(m.bestModel.coefficientMatrix, a.bestModel.coefficientMatrix)


@pytest.mark.parametrize("reg,alpha", [(0.3, 0.0), (0.1, 0.2)])
def test_wolfe_line_search_device_matches_cpu_oracle(cuda, wisdm_csv, reg, alpha):
    """LogisticRegression(lineSearch="wolfe") on the WISDM reference encoding: the device fit (the
    evaluation kernels at each round's trial points, DeviceLogregSolver.evaluate_at) against the CPU
    oracle (the same optim.lbfgs.minimize_wolfe with the torch objective): objective histories,
    iterations and coefficients agree to the rounding of the two objective evaluations."""
    from har.models.logreg import LogisticRegression
    from har.ops import logreg as L
    from har.suite import load_wisdm

    n = {"at": 0}
    real = L.DeviceLogregSolver.evaluate_at

    def count(self, x):
        n["at"] += 1
        return real(self, x)

    L.DeviceLogregSolver.evaluate_at = count
    try:
        trg, _, _ = load_wisdm(wisdm_csv, "reference", 2018, device=cuda)
        mg = LogisticRegression(maxIter=20, regParam=reg, elasticNetParam=alpha, lineSearch="wolfe",
                                device="cuda").fit(trg)
    finally:
        L.DeviceLogregSolver.evaluate_at = real
    assert n["at"] >= mg.summary["iterations"] + 1
    trc, _, _ = load_wisdm(wisdm_csv, "reference", 2018)
    mc = LogisticRegression(maxIter=20, regParam=reg, elasticNetParam=alpha, lineSearch="wolfe",
                            device="cpu").fit(trc)
    hg, hc = mg.summary["objectiveHistory"], mc.summary["objectiveHistory"]
    assert mg.summary["iterations"] == mc.summary["iterations"], (hg, hc)
    np.testing.assert_allclose(hg, hc, rtol=2e-5)
    torch.testing.assert_close(mg.coefficientMatrix.cpu(), mc.coefficientMatrix, rtol=2e-3, atol=2e-4)
