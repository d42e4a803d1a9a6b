"""Breeze-semantics line searches for LogisticRegression (``lineSearch="wolfe"``):
the batched strong-Wolfe L-BFGS / backtracking OWL-QN of ``optim.lbfgs.minimize_wolfe`` (the CPU
oracle of the device path: the same function, the objective from the evaluation kernels)."""
import numpy as np
import pytest
import torch

from har.optim.lbfgs import minimize_trials, minimize_wolfe

N, F, K = 1500, 10, 4


def _problem(seed=0):
    g = torch.Generator().manual_seed(seed)
    mu = torch.randn(K, F, generator=g)
    y = torch.randint(0, K, (N,), generator=g)
    X = (mu[y] + 1.5 * torch.randn(N, F, generator=g)).double()

    def data(x):  # the softmax cross entropy (mean) of B weight tables x [B, K (F + 1)] and its gradient
        B = x.shape[0]
        W = x.double().view(B, K, F + 1)
        z = torch.einsum("nf,bkf->bnk", X, W[:, :, :F]) + W[:, None, :, F]
        loss = torch.nn.functional.cross_entropy(z.reshape(-1, K), y.repeat(B), reduction="none").view(B, N).mean(1)
        p = torch.softmax(z, -1)
        p[:, torch.arange(N), y] -= 1
        p /= N
        G = torch.cat([torch.einsum("bnk,nf->bkf", p, X), p.sum(1)[:, :, None]], 2).reshape(B, -1)
        return loss, G.float()

    return data


def _reg(l2, l1):
    notb = torch.ones(K, F + 1)
    notb[:, F] = 0  # the intercept is not regularized
    l2v = (torch.tensor(l2)[:, None] * notb.reshape(1, -1)).float()
    l1v = (torch.tensor(l1)[:, None] * notb.reshape(1, -1)).float()
    return l2v, l1v


def test_wolfe_lbfgs_reaches_the_scipy_optimum():
    import scipy.optimize as so

    data = _problem()
    l2v, l1v = _reg([0.1, 0.01], [0.0, 0.0])
    r = minimize_wolfe(data, torch.zeros(2, K * (F + 1)), l2v, None, max_iter=300, tol=1e-12)
    for b in range(2):
        def fg(w):
            wt = torch.tensor(w)
            loss, G = data(wt[None])
            reg = l2v[b].double()
            return float(loss[0]) + 0.5 * float((reg * wt * wt).sum()), (G[0].double() + reg * wt).numpy()

        ref = so.minimize(fg, np.zeros(K * (F + 1)), jac=True, method="L-BFGS-B",
                          options=dict(maxiter=2000, gtol=1e-12, ftol=1e-15))
        assert abs(float(r.f[b]) - ref.fun) <= 1e-9 * max(1.0, abs(ref.fun)), (b, float(r.f[b]), ref.fun)


def test_wolfe_steps_satisfy_their_conditions_and_decrease():
    """Every accepted L-BFGS step satisfies the strong Wolfe conditions (Armijo, |phi'(t)| <= 0.9
    |phi'(0)|) and every accepted OWL-QN step Armijo + the weak curvature condition (phi'(t) >= 0.9
    phi'(0), phi' along the pseudo-gradient), on the line searches' own recorded values, which are
    tied to the path: phi(0) / phi(t) of consecutive steps are the objective history, and phi(t) is
    the objective recomputed at the accepted point.  The histories decrease; OWL-QN ends at the
    optimum a long Armijo-trial solve reaches."""
    data = _problem(1)
    l2v, l1v = _reg([0.05, 0.02], [0.0, 0.03])
    trace = []
    r = minimize_wolfe(data, torch.zeros(2, K * (F + 1)), l2v, l1v, max_iter=25, tol=1e-9, trace=trace)
    c1, c2 = 1e-4, 0.9
    for b in range(2):
        h = r.history_per_model[b]
        assert all(b2 <= a2 + 1e-12 for a2, b2 in zip(h, h[1:])), h
        steps = [s for s in trace if s["model"] == b]
        assert len(steps) == int(r.iterations[b]) >= 5, (b, len(steps))
        assert steps[0]["owl"] == (b == 1)
        for i, s in enumerate(steps):
            assert s["iter"] == i and s["t"] > 0
            assert s["d0"] < 0, s                                      # a descent direction
            assert s["ft"] <= s["f0"] + c1 * s["t"] * s["d0"], s       # Armijo (sufficient decrease)
            if b == 0:
                assert abs(s["dt"]) <= c2 * abs(s["d0"]), s           # strong curvature
            else:
                assert s["dt"] >= c2 * s["d0"], s                     # weak curvature
            assert s["f0"] == h[i] and s["ft"] == h[i + 1]           # the recorded values are the path's
    # phi(t) of the last accepted step is the objective at the solution, recomputed independently
    for b in range(2):
        loss, _ = data(r.x[b:b + 1])
        x = r.x[b].double()
        obj = float(loss[0]) + 0.5 * float((l2v[b].double() * x * x).sum()) + float((l1v[b].double() * x.abs()).sum())
        assert abs(obj - [s for s in trace if s["model"] == b][-1]["ft"]) <= 1e-9 * max(1.0, abs(obj))
    long = minimize_trials(data, torch.zeros(2, K * (F + 1)), l2v, l1v, max_iter=400, tol=1e-12)
    r2 = minimize_wolfe(data, torch.zeros(2, K * (F + 1)), l2v, l1v, max_iter=400, tol=1e-12)
    np.testing.assert_allclose(r2.f.numpy(), long.f.numpy(), rtol=1e-9)


def test_wolfe_batch_equals_single_model_solves():
    """Models advance their own line-search state machines: a batched solve of three models equals
    the three single-model solves (the same trial points, iterations and objective histories)."""
    data = _problem(2)
    l2v, l1v = _reg([0.1, 0.3, 0.05], [0.0, 0.0, 0.01])
    x0 = torch.zeros(3, K * (F + 1))
    rb = minimize_wolfe(data, x0, l2v, l1v, max_iter=20, tol=1e-6)
    for b in range(3):
        rs = minimize_wolfe(data, x0[b:b + 1], l2v[b:b + 1], l1v[b:b + 1] if l1v[b].any() else None,
                            max_iter=20, tol=1e-6)
        assert torch.equal(rs.x[0], rb.x[b]), b
        assert rs.iterations.tolist() == [int(rb.iterations[b])]
        n = len(rs.history_per_model[0])
        assert rs.history_per_model[0] == rb.history_per_model[b][:n]


def test_logistic_regression_wolfe_on_wisdm(wisdm_csv):
    """The reference's LR (maxIter 20, regParam 0.3) and an OWL-QN grid point with lineSearch="wolfe":
    accuracy at least the reference's (0.6148, result.txt:167), one objectiveHistory entry per
    iteration (+ the start), decreasing."""
    from har.data.csv_io import read_csv
    from har.data.split import random_split
    from har.features import wisdm
    from har.models.logreg import LogisticRegression

    _, _, df = wisdm.prepare(read_csv(wisdm_csv), "reference")
    train, test = random_split(df, [0.7, 0.3], 2018)
    for reg, a in ((0.3, 0.0), (0.1, 0.2)):
        m = LogisticRegression(maxIter=20, regParam=reg, elasticNetParam=a, lineSearch="wolfe").fit(train)
        s = m.summary
        h = s["objectiveHistory"]
        assert s["lineSearch"] == "wolfe" and len(h) == s["iterations"] + 1, (len(h), s["iterations"])
        assert all(b <= a2 + 1e-12 for a2, b in zip(h, h[1:]))
        assert len(s["lineSearchRounds"]) >= s["iterations"]
        out = m.transform(test)
        acc = float((out["prediction"].data == out["label"].data).mean())
        assert acc >= 0.61, (reg, a, acc)


def test_line_search_param_validated():
    from har.models.logreg import LogisticRegression

    with pytest.raises(ValueError):
        LogisticRegression(lineSearch="more-thuente")
