"""Batched, device-resident L-BFGS / OWL-QN.

Replaces Breeze's ``LBFGS`` (elasticNetParam = 0) and ``OWLQN`` (elasticNetParam
> 0) that Spark's ``LogisticRegression.train`` drives on the JVM driver, with a
``treeAggregate`` of the loss/gradient over the executors per evaluation
(``Main/main.py:117`` single fit, ``:215`` the 45 CrossValidator fits; SURVEY.md
N7/K10, §3.3).

Here B independent problems (e.g. 5 folds x 9 grid points) advance in lock
step: the objective is evaluated for all of them in ONE fused forward/backward
launch sequence, and the two-loop recursion, the orthant projection and the
Armijo backtracking are batched tensor ops over the model dimension — the
driver never round-trips per model.  With ``l1 == 0`` OWL-QN reduces exactly to
L-BFGS, so one code path serves the whole elastic-net grid.

Convergence (per model, like Breeze's FirstOrderMinimizer): stop when
``|f_k - f_{k-1}| / max(|f_k|, |f_{k-1}|, 1) < tol`` or the (pseudo-)gradient
norm is below ``tol * max(1, |x|)`` or ``max_iter`` is reached.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

import torch

Objective = Callable[[torch.Tensor], "tuple[torch.Tensor, torch.Tensor]"]


@dataclass
class LbfgsResult:
    x: torch.Tensor          # [B, D]
    f: torch.Tensor          # [B]   final objective (smooth + l1)
    iterations: torch.Tensor  # [B]  iterations taken per model
    n_evals: int             # batched objective evaluations
    history: list            # per-iteration mean objective (for logging / tests)


def _pseudo_grad(x, g, l1):
    if l1 is None:
        return g
    gp = g + l1
    gm = g - l1
    pg_zero = torch.where(gp < 0, gp, torch.where(gm > 0, gm, torch.zeros_like(g)))
    return torch.where(x > 0, gp, torch.where(x < 0, gm, pg_zero))


def _l1_value(x, l1):
    if l1 is None:
        return torch.zeros(x.shape[0], dtype=x.dtype, device=x.device)
    return (l1 * x.abs()).sum(dim=1)


def minimize(fun: Objective, x0: torch.Tensor, max_iter: int = 100, m: int = 10, tol: float = 1e-6,
             l1: Optional[torch.Tensor] = None, max_ls: int = 25, c1: float = 1e-4) -> LbfgsResult:
    """Minimize B problems ``f_b(x_b) + sum_j l1[b,j] |x_b[j]|`` in lock step.

    ``fun(x [B,D]) -> (f [B], g [B,D])`` is the smooth part.
    """
    x = x0.clone()
    B, D = x.shape
    dev, dt = x.device, x.dtype
    if l1 is not None and not bool((l1 > 0).any()):
        l1 = None
    f, g = fun(x)
    n_evals = 1
    F = f + _l1_value(x, l1)
    S = torch.zeros(m, B, D, dtype=dt, device=dev)
    Y = torch.zeros(m, B, D, dtype=dt, device=dev)
    RHO = torch.zeros(m, B, dtype=dt, device=dev)  # 0 marks an empty / rejected slot
    active = torch.ones(B, dtype=torch.bool, device=dev)
    iters = torch.zeros(B, dtype=torch.int64, device=dev)
    history = [float(F.mean())]
    head = 0  # ring position of the next write
    filled = 0

    for it in range(max_iter):
        pg = _pseudo_grad(x, g, l1)
        # ---- two-loop recursion over the ring (newest first) ----
        q = pg.clone()
        alphas = []
        order = [(head - 1 - i) % m for i in range(filled)]
        for j in order:
            a = RHO[j] * (S[j] * q).sum(dim=1)
            q = q - a[:, None] * Y[j]
            alphas.append(a)
        if filled:
            j = order[0]
            yy = (Y[j] * Y[j]).sum(dim=1)
            sy = (S[j] * Y[j]).sum(dim=1)
            gamma = torch.where((RHO[j] > 0) & (yy > 0), sy / yy.clamp_min(1e-300), torch.ones_like(yy))
        else:
            gamma = 1.0 / pg.norm(dim=1).clamp_min(1e-12)  # first step: unit-length move
        r = q * gamma[:, None]
        for j, a in zip(reversed(order), reversed(alphas)):
            b = RHO[j] * (Y[j] * r).sum(dim=1)
            r = r + (a - b)[:, None] * S[j]
        d = -r
        if l1 is not None:  # keep the direction inside the pseudo-gradient's orthant
            d = torch.where(d * pg < 0, d, torch.zeros_like(d))
            xi = torch.where(x != 0, torch.sign(x), torch.sign(-pg))
        dd = (pg * d).sum(dim=1)
        bad = dd >= 0  # not a descent direction -> steepest descent
        if bool(bad.any()):
            d = torch.where(bad[:, None], -pg, d)
            dd = torch.where(bad, -(pg * pg).sum(dim=1), dd)

        # ---- batched backtracking (Armijo) ----
        step = torch.ones(B, dtype=dt, device=dev)
        accepted = ~active
        x_new, f_new, g_new, F_new = x.clone(), f.clone(), g.clone(), F.clone()
        for _ in range(max_ls):
            xt = x + step[:, None] * d
            if l1 is not None:
                xt = torch.where(torch.sign(xt) == xi, xt, torch.zeros_like(xt))
            ft, gt = fun(xt)
            n_evals += 1
            Ft = ft + _l1_value(xt, l1)
            decrease = (pg * (xt - x)).sum(dim=1) if l1 is not None else step * dd
            ok = (Ft <= F + c1 * decrease) & torch.isfinite(Ft) & ~accepted
            x_new = torch.where(ok[:, None], xt, x_new)
            f_new = torch.where(ok, ft, f_new)
            F_new = torch.where(ok, Ft, F_new)
            g_new = torch.where(ok[:, None], gt, g_new)
            accepted = accepted | ok
            if bool(accepted.all()):
                break
            step = torch.where(accepted, step, step * 0.5)
        moved = accepted & active
        # ---- history update ----
        s = x_new - x
        y = g_new - g
        sy = (s * y).sum(dim=1)
        good = moved & (sy > 1e-10 * (s.norm(dim=1) * y.norm(dim=1)).clamp_min(1e-300))
        S[head] = torch.where(good[:, None], s, torch.zeros_like(s))
        Y[head] = torch.where(good[:, None], y, torch.zeros_like(y))
        RHO[head] = torch.where(good, 1.0 / sy.clamp_min(1e-300), torch.zeros_like(sy))
        head = (head + 1) % m
        filled = min(filled + 1, m)

        rel = (F - F_new).abs() / torch.maximum(torch.maximum(F.abs(), F_new.abs()), torch.ones_like(F))
        x, f, g, F = x_new, f_new, g_new, F_new
        iters = iters + active.to(torch.int64)
        pgn = _pseudo_grad(x, g, l1).norm(dim=1)
        converged = (rel < tol) | (pgn <= tol * torch.clamp(x.norm(dim=1), min=1.0)) | ~moved
        active = active & ~converged
        history.append(float(F.mean()))
        if not bool(active.any()):
            break
    return LbfgsResult(x=x, f=F, iterations=iters, n_evals=n_evals, history=history)


# ------------------------------------------------------------------------------------------
# Parallel-trial line search: the algorithm the device kernels run (csrc/kernels/logreg_qn.hip)
# ------------------------------------------------------------------------------------------
@dataclass
class TrialResult:
    x: torch.Tensor           # [B, D]
    f: torch.Tensor           # [B] objective (data loss + regularization), float64
    iterations: torch.Tensor  # [B]
    n_evals: int              # batched evaluations (each covers B x T trial points)
    history: list             # per-iteration mean objective
    history_per_model: list = None  # [B] lists: each model's own objective per iteration


def _reg_value(x, l2v, l1v):
    r = 0.5 * (l2v.double() * x.double() * x.double()).sum(dim=1)
    if l1v is not None:
        r = r + (l1v.double() * x.double().abs()).sum(dim=1)
    return r


def minimize_trials(evaluate, x0: torch.Tensor, l2v: torch.Tensor, l1v: Optional[torch.Tensor] = None,
                    max_iter: int = 100, m: int = 10, tol: float = 1e-6, trials: int = 4, c1: float = 1e-4,
                    poll: int = 0) -> TrialResult:
    """Minimize ``B`` problems ``data(x_b) + 0.5 sum l2v x^2 + sum l1v |x|`` in lock step with
    L-BFGS (OWL-QN where ``l1v`` is non-zero), evaluating ``trials`` step lengths
    ``a 2^-t`` of every line search in ONE batched call instead of backtracking serially.

    ``evaluate(xt [B*T, D]) -> (loss [B*T] float64, grad [B*T, D])`` returns the DATA part.
    Per iteration a model takes the largest trial step satisfying the Armijo condition; if
    none does it stays put, its next steps shrink 16x, and a second consecutive failure
    freezes it.  A two-loop direction that is not a descent direction is rejected and the
    model takes steepest descent on its pseudo-gradient in the next iteration.  A model also freezes on ``|dF| / max(|F|, |F'|, 1) < tol`` or
    ``|pg| <= tol * max(1, |x|)``.  This is the reference math of the device kernels
    (``har.ops.logreg.DeviceLogregSolver``), float32 vectors with float64 reductions.
    """
    B, D = x0.shape
    dev = x0.device
    T = int(trials)
    x = x0.clone().float()
    if l1v is not None and not bool((l1v > 0).any()):
        l1v = None
    loss, G = evaluate(x)
    g = G.float() + l2v * x
    Fo = loss.double() + _reg_value(x, l2v, l1v)
    S = torch.zeros(m, B, D, device=dev)
    Y = torch.zeros(m, B, D, device=dev)
    rho = torch.zeros(m, B, dtype=torch.float64, device=dev)
    active = torch.ones(B, dtype=torch.bool, device=dev)
    fails = torch.zeros(B, dtype=torch.int64, device=dev)
    iters = torch.zeros(B, dtype=torch.int64, device=dev)
    scale = torch.ones(B, device=dev)
    steep = torch.zeros(B, dtype=torch.bool, device=dev)
    head, filled, n_evals = 0, 0, 1
    fhist = [Fo.clone()]  # per-model objectives, read back once at the end (no per-iteration sync)
    pg_fn = lambda xx, gg: _pseudo_grad(xx, gg, l1v)  # noqa: E731
    for it in range(max_iter):
        pg = pg_fn(x, g)
        q = pg.clone()
        alphas = []
        for i in range(filled):
            j = (head - 1 - i) % m
            a = rho[j] * (S[j].double() * q.double()).sum(1)
            alphas.append(a)
            q = torch.where((rho[j] != 0)[:, None], (q.double() - a[:, None] * Y[j].double()).float(), q)
        if filled:
            j = (head - 1) % m
            yy = (Y[j].double() ** 2).sum(1)
            sy = (S[j].double() * Y[j].double()).sum(1)
            gamma = torch.where((rho[j] > 0) & (yy > 0), sy / yy.clamp_min(1e-300), torch.ones_like(yy))
        else:
            gamma = 1.0 / (pg.double() ** 2).sum(1).sqrt().clamp_min(1e-12)
        q = (gamma[:, None] * q.double()).float()
        for i in reversed(range(filled)):
            j = (head - 1 - i) % m
            bcoef = rho[j] * (Y[j].double() * q.double()).sum(1)
            coef = alphas[i] - bcoef
            q = torch.where((rho[j] != 0)[:, None], (q.double() + coef[:, None] * S[j].double()).float(), q)
        d = -q
        if l1v is not None:
            d = torch.where(d * pg < 0, d, torch.zeros_like(d))
        # a model whose last direction was not a descent direction takes steepest descent now
        d = torch.where(steep[:, None], -pg, d)
        dd = (pg.double() * d.double()).sum(1)
        # T trial points per model
        steps = scale[:, None] * torch.pow(2.0, -torch.arange(T, device=dev, dtype=torch.float32))[None, :]
        xt = x[:, None, :] + steps[:, :, None] * d[:, None, :]                        # [B, T, D]
        decr = steps.double() * dd[:, None]
        if l1v is not None:
            xi = torch.where(x != 0, torch.sign(x), torch.sign(-pg))
            xt = torch.where(torch.sign(xt) == xi[:, None, :], xt, torch.zeros_like(xt))
            decr = (pg[:, None, :].double() * (xt.double() - x[:, None, :].double())).sum(2)
        xt = torch.where(active[:, None, None], xt, x[:, None, :])
        xt_flat = xt.reshape(B * T, D)
        reg = _reg_value(xt_flat, l2v.repeat_interleave(T, 0),
                         None if l1v is None else l1v.repeat_interleave(T, 0)).view(B, T)
        loss_t, G_t = evaluate(xt_flat)
        n_evals += 1
        Ft = loss_t.double().view(B, T) + reg
        ok = torch.isfinite(Ft) & (Ft <= Fo[:, None] + c1 * decr)
        first = torch.where(ok.any(1), ok.float().argmax(1), torch.full((B,), -1, device=dev, dtype=torch.int64))
        nondescent = active & (dd >= 0) & ~steep   # rejected; steepest descent next iteration
        first = torch.where(dd >= 0, torch.full_like(first, -1), first)
        take = active & (first >= 0)
        pick = first.clamp_min(0)
        ar = torch.arange(B, device=dev)
        x_new = xt[ar, pick]
        g_new = G_t.view(B, T, D)[ar, pick].float() + l2v * x_new
        F_new = Ft[ar, pick]
        s_vec = x_new - x
        y_vec = g_new - g
        sy = (s_vec.double() * y_vec.double()).sum(1)
        good = sy > 1e-10 * (s_vec.double().norm(dim=1) * y_vec.double().norm(dim=1)).clamp_min(1e-300)
        S[head] = torch.where(take[:, None], s_vec, S[head])
        Y[head] = torch.where(take[:, None], y_vec, Y[head])
        rho[head] = torch.where(take & good, 1.0 / sy.clamp_min(1e-300), torch.zeros_like(sy))
        rel = (Fo - F_new).abs() / torch.maximum(torch.maximum(Fo.abs(), F_new.abs()), torch.ones_like(Fo))
        pgn = (pg_fn(x_new, g_new).double() ** 2).sum(1).sqrt()
        xn = (x_new.double() ** 2).sum(1).sqrt()
        conv = (rel < tol) | (pgn <= tol * xn.clamp_min(1.0))
        x = torch.where(take[:, None], x_new, x)
        g = torch.where(take[:, None], g_new, g)
        Fo = torch.where(take, F_new, Fo)
        iters = iters + take.long()
        failed = active & ~take & ~nondescent
        fails = torch.where(take, torch.zeros_like(fails), fails + failed.long())
        scale = torch.where(take, torch.ones_like(scale), torch.where(failed, scale / 16, scale))
        steep = torch.where(take, torch.zeros_like(steep), steep | nondescent)
        active = active & ~(take & conv) & ~(fails >= 2)
        head = (head + 1) % m
        filled = min(filled + 1, m)
        fhist.append(Fo.clone())
        if poll and (it + 1) % poll == 0 and not bool(active.any()):
            break
    H = torch.stack(fhist).cpu()  # [iterations + 1, B]
    return TrialResult(x=x, f=Fo, iterations=iters, n_evals=n_evals, history=H.mean(1).tolist(),
                       history_per_model=[H[:, b].tolist() for b in range(B)])


# ------------------------------------------------------------------------------------------
# Breeze-semantics line searches (LogisticRegression(lineSearch="wolfe"))
# ------------------------------------------------------------------------------------------
# Spark's LogisticRegression.train runs Breeze's LBFGS (elasticNetParam = 0) or OWLQN (> 0):
#   * LBFGS.determineStepSize: StrongWolfeLineSearch(maxZoomIter = 10, maxLineSearchIter = 10),
#     c1 = 1e-4, c2 = 0.9, initial step 1 / |dir| on the first iteration and 1 afterwards; the
#     bracketing phase grows the step by 1.5, the zoom phase picks the safeguarded cubic
#     interpolant of the bracket (clamped to its inner 80 %);
#   * OWLQN.determineStepSize: BacktrackingLineSearch on the orthant-projected step, Armijo
#     (c 1e-4) plus the weak Wolfe curvature condition (c 0.9: grow the step by 2.1 while it fails),
#     shrink 0.1 on the first iteration and 0.5 afterwards, initial step 0.5 / |grad| on the first
#     iteration and 1 afterwards, at most 20 trial steps; the directional derivative is the
#     pseudo-gradient of the trial point along the search direction.
# A search that fails (a bracket / zoom / backtracking budget spent, a non-descent direction)
# resets that model's history and retries from steepest descent; a second consecutive failure stops
# the model (Breeze: FirstOrderMinimizer's failedOnce).  Convergence, per model, Breeze's
# defaultConvergenceCheck form: (max F over the last 20 iterates - F) / max(|F|, |that max|, 1e-6)
# <= tol, or |adjusted gradient|_inf / max(|x|_2, 1) <= tol, or maxIter.
# Breeze's source is not in this environment: the constants and control flow above are restated
# from its documented algorithm, so coefficient / objectiveHistory parity with Spark stays
# unpinned (no reference fixture holds them; PARITY.md).
#
# Batched: every model advances its own line-search state machine; each ROUND evaluates ONE trial
# point per model still searching, all models in ONE evaluation call (the device kernels on the
# GPU), so the rounds of an iteration are max over models, not the sum.


def _cubic_step(lt, lf, ld, rt, rf, rd):
    """Breeze CubicLineSearch.interp of brackets l < r: the cubic minimizer, clamped to
    [l + 0.1 (r - l), l + 0.9 (r - l)]; a non-real / non-finite interpolant falls back to the midpoint."""
    d1 = ld + rd - 3.0 * (lf - rf) / (lt - rt)
    disc = d1 * d1 - ld * rd
    d2 = torch.sqrt(disc.clamp_min(0.0))
    t = rt - (rt - lt) * (rd + d2 - d1) / (rd - ld + 2.0 * d2)
    lb, ub = lt + 0.1 * (rt - lt), lt + 0.9 * (rt - lt)
    t = torch.minimum(torch.maximum(t, lb), ub)
    return torch.where(torch.isfinite(t) & (disc >= 0), t, 0.5 * (lt + rt))


def _interp_bracket(lo_t, lo_f, lo_d, hi_t, hi_f, hi_d):
    """interp(low, hi) if low.t <= hi.t else interp(hi, low) (Breeze's zoom)."""
    sw = lo_t > hi_t
    a = [torch.where(sw, h, l) for l, h in ((lo_t, hi_t), (lo_f, hi_f), (lo_d, hi_d))]
    b = [torch.where(sw, l, h) for l, h in ((lo_t, hi_t), (lo_f, hi_f), (lo_d, hi_d))]
    return _cubic_step(*a, *b)


def minimize_wolfe(evaluate, x0: torch.Tensor, l2v: torch.Tensor, l1v: Optional[torch.Tensor] = None,
                   max_iter: int = 100, m: int = 10, tol: float = 1e-6, c1: float = 1e-4, c2: float = 0.9,
                   max_ls: int = 10, max_zoom: int = 10, max_backtrack: int = 20, fval_memory: int = 20,
                   trace: Optional[list] = None) -> TrialResult:
    """Minimize ``B`` problems ``data(x_b) + 0.5 sum l2v x^2 + sum l1v |x|`` with Breeze's line
    searches (module comment above): strong Wolfe for the models without an L1 term (L-BFGS),
    projected backtracking with the weak Wolfe condition for the models with one (OWL-QN).

    ``evaluate(x [B, D]) -> (loss [B] float64, grad [B, D])`` is the DATA part (as in
    ``minimize_trials`` with one trial).  float32 vectors, float64 reductions and line-search
    scalars; every operation is a batched tensor op on x's device.  ``n_evals`` counts the
    batched evaluations (the initial one plus one per line-search round).  ``trace`` (a list, optional)
    receives one dict per model and accepted step: the step ``t``, phi(0) ``f0``, phi'(0) ``d0``,
    phi(t) ``ft`` and phi'(t) ``dt`` of its line search (tests/test_wolfe.py checks the conditions)."""
    B, D = x0.shape
    dev = x0.device
    f64 = torch.float64
    x = x0.clone().float()
    owl = (l1v > 0).any(1) if l1v is not None else torch.zeros(B, dtype=torch.bool, device=dev)
    l1 = l1v if (l1v is not None and bool(owl.any())) else None
    pg_fn = lambda xx, gg: _pseudo_grad(xx, gg, l1)  # noqa: E731
    dot = lambda a, b: (a.double() * b.double()).sum(1)  # noqa: E731
    loss, G = evaluate(x)
    g = G.float() + l2v * x
    F = loss.double() + _reg_value(x, l2v, l1)
    S = torch.zeros(m, B, D, device=dev)
    Y = torch.zeros(m, B, D, device=dev)
    rho = torch.zeros(m, B, dtype=f64, device=dev)
    active = torch.ones(B, dtype=torch.bool, device=dev)
    failed_once = torch.zeros(B, dtype=torch.bool, device=dev)
    iters = torch.zeros(B, dtype=torch.int64, device=dev)
    head, filled, n_evals = 0, 0, 1
    fhist = [F.clone()]
    rounds_per_iter = []
    for it in range(max_iter):
        pg = pg_fn(x, g)
        # ---- two-loop recursion (Breeze: unscaled -grad while the history is empty) ----
        q = pg.clone()
        alphas = []
        for i in range(filled):
            j = (head - 1 - i) % m
            a = rho[j] * dot(S[j], q)
            alphas.append(a)
            q = torch.where((rho[j] != 0)[:, None], (q.double() - a[:, None] * Y[j].double()).float(), q)
        if filled:
            j = (head - 1) % m
            yy = (Y[j].double() ** 2).sum(1)
            sy = dot(S[j], Y[j])
            gamma = torch.where((rho[j] > 0) & (yy > 0), sy / yy.clamp_min(1e-300), torch.ones_like(yy))
            q = (gamma[:, None] * q.double()).float()
        for i in reversed(range(filled)):
            j = (head - 1 - i) % m
            coef = alphas[i] - rho[j] * dot(Y[j], q)
            q = torch.where((rho[j] != 0)[:, None], (q.double() + coef[:, None] * S[j].double()).float(), q)
        d = -q
        d = torch.where(owl[:, None] & ~(d * pg < 0), torch.zeros_like(d), d)
        dd0 = dot(pg, d)
        nondesc = active & ~(dd0 < 0)          # Breeze throws -> the retry from steepest descent
        d = torch.where(nondesc[:, None], -pg, d)
        dd0 = torch.where(nondesc, -dot(pg, pg), dd0)
        xi = torch.where(x != 0, torch.sign(x), torch.sign(-pg))
        first = iters == 0
        dn = dot(d, d).sqrt().clamp_min(1e-300)
        gn = dot(g, g).sqrt().clamp_min(1e-300)
        t = torch.where(owl, torch.where(first, 0.5 / gn, torch.ones_like(gn)),
                        torch.where(first, 1.0 / dn, torch.ones_like(dn)))
        shrink = torch.where(first, torch.full_like(t, 0.1), torch.full_like(t, 0.5))
        # ---- per-model line-search state ----
        searching = active.clone()
        success = torch.zeros(B, dtype=torch.bool, device=dev)
        zoom = torch.zeros(B, dtype=torch.bool, device=dev)
        n_try = torch.zeros(B, dtype=torch.int64, device=dev)   # bracket / backtracking trials
        n_zoom = torch.zeros(B, dtype=torch.int64, device=dev)
        lo_t, lo_f, lo_d = torch.zeros_like(t), F.clone(), dd0.clone()   # phi(0)
        hi_t, hi_f, hi_d = torch.zeros_like(t), F.clone(), dd0.clone()
        x_acc, g_acc, F_acc = x.clone(), g.clone(), F.clone()
        t_acc, d_acc = torch.zeros_like(t), torch.zeros_like(dd0)
        rounds = 0
        while bool(searching.any()):
            rounds += 1
            t_cur = t
            xt = x + t.float()[:, None] * d
            xt = torch.where(owl[:, None] & (torch.sign(xt) != xi), torch.zeros_like(xt), xt)
            xt = torch.where(searching[:, None], xt, x)
            lt, Gt = evaluate(xt)
            n_evals += 1
            gt = Gt.float() + l2v * xt
            Ft = lt.double() + _reg_value(xt, l2v, l1)
            dt = torch.where(owl, dot(pg_fn(xt, gt), d), dot(gt, d))
            fin = torch.isfinite(Ft)
            armijo = Ft <= F + c1 * t * dd0
            curv_strong = dt.abs() <= c2 * dd0.abs()
            done_now = torch.zeros_like(searching)
            fail_now = torch.zeros_like(searching)
            # -- OWL-QN: backtracking with the weak Wolfe condition --
            bt = searching & owl
            bt_ok = bt & fin & armijo & (dt >= c2 * dd0)
            mult = torch.where(~(fin & armijo), shrink, torch.full_like(t, 2.1))
            done_now |= bt_ok
            n_try = n_try + bt.long()
            bt_next = bt & ~bt_ok
            fail_now |= bt_next & ((n_try > max_backtrack) | (t * mult < 1e-10) | (t * mult > 1e10))
            t_bt = t * mult
            # -- L-BFGS: strong Wolfe, bracketing phase --
            br = searching & ~owl & ~zoom
            n_try = n_try + br.long()
            halve = br & ~fin
            to_zoom_a = br & fin & (~armijo | ((Ft >= lo_f) & (n_try > 1)))      # zoom(low, c)
            ok_br = br & fin & ~to_zoom_a & curv_strong
            to_zoom_b = br & fin & ~to_zoom_a & ~curv_strong & (dt >= 0)       # zoom(c, low)
            grow = br & fin & ~to_zoom_a & ~ok_br & ~to_zoom_b
            done_now |= ok_br
            # zoom(low, c): low stays, hi = c;  zoom(c, low): hi = low, low = c
            nhi_t = torch.where(to_zoom_a, t, torch.where(to_zoom_b, lo_t, hi_t))
            nhi_f = torch.where(to_zoom_a, Ft, torch.where(to_zoom_b, lo_f, hi_f))
            nhi_d = torch.where(to_zoom_a, dt, torch.where(to_zoom_b, lo_d, hi_d))
            nlo_t = torch.where(to_zoom_b | grow, t, lo_t)
            nlo_f = torch.where(to_zoom_b | grow, Ft, lo_f)
            nlo_d = torch.where(to_zoom_b | grow, dt, lo_d)
            # -- L-BFGS: zoom phase (the trial t was interpolated from the bracket) --
            zm = searching & ~owl & zoom
            n_zoom = n_zoom + zm.long()
            z_hi = zm & (~fin | ~armijo | (Ft >= lo_f))
            z_ok = zm & ~z_hi & curv_strong
            z_mv = zm & ~z_hi & ~z_ok
            z_swap = z_mv & (dt * (hi_t - lo_t) >= 0)                            # hi = low
            done_now |= z_ok
            nhi_t = torch.where(z_hi, t, torch.where(z_swap, lo_t, nhi_t))
            nhi_f = torch.where(z_hi, Ft, torch.where(z_swap, lo_f, nhi_f))
            nhi_d = torch.where(z_hi, dt, torch.where(z_swap, lo_d, nhi_d))
            nlo_t = torch.where(z_mv, t, nlo_t)
            nlo_f = torch.where(z_mv, Ft, nlo_f)
            nlo_d = torch.where(z_mv, dt, nlo_d)
            lo_t, lo_f, lo_d, hi_t, hi_f, hi_d = nlo_t, nlo_f, nlo_d, nhi_t, nhi_f, nhi_d
            zoom = zoom | to_zoom_a | to_zoom_b
            fail_now |= (br & ~done_now & ~to_zoom_a & ~to_zoom_b & (n_try >= max_ls))
            fail_now |= ((zm | to_zoom_a | to_zoom_b) & ~done_now & (n_zoom >= max_zoom))
            # next trial step
            t_zoom = _interp_bracket(lo_t, lo_f, lo_d, hi_t, hi_f, hi_d)
            t = torch.where(bt, t_bt, torch.where(halve, t / 2, torch.where(grow, t * 1.5,
                                                                          torch.where(zoom, t_zoom, t))))
            # accepted trial points
            t_acc = torch.where(done_now, t_cur, t_acc)
            d_acc = torch.where(done_now, dt, d_acc)
            x_acc = torch.where(done_now[:, None], xt, x_acc)
            g_acc = torch.where(done_now[:, None], gt, g_acc)
            F_acc = torch.where(done_now, Ft, F_acc)
            success |= done_now
            searching = searching & ~done_now & ~fail_now
        rounds_per_iter.append(rounds)
        take = active & success
        if trace is not None:
            for b in torch.nonzero(take).flatten().tolist():
                trace.append({"model": b, "iter": int(iters[b]), "owl": bool(owl[b]), "t": float(t_acc[b]),
                              "f0": float(F[b]), "d0": float(dd0[b]), "ft": float(F_acc[b]), "dt": float(d_acc[b])})
        s_vec = x_acc - x
        y_vec = g_acc - g
        sy = dot(s_vec, y_vec)
        good = take & (sy > 1e-10 * (dot(s_vec, s_vec).sqrt() * dot(y_vec, y_vec).sqrt()).clamp_min(1e-300))
        # a failed search clears the model's history (Breeze: reset, retry from steepest descent)
        failed = active & ~success
        for j in range(m):
            rho[j] = torch.where(failed, torch.zeros_like(rho[j]), rho[j])
        S[head] = torch.where(take[:, None], s_vec, S[head])
        Y[head] = torch.where(take[:, None], y_vec, Y[head])
        rho[head] = torch.where(good, 1.0 / sy.clamp_min(1e-300), torch.where(take, torch.zeros_like(sy), rho[head]))
        x = torch.where(take[:, None], x_acc, x)
        g = torch.where(take[:, None], g_acc, g)
        F = torch.where(take, F_acc, F)
        iters = iters + take.long()
        fhist.append(F.clone())
        recent = torch.stack(fhist[-(fval_memory + 1):-1]).max(0).values if len(fhist) > 1 else F
        fconv = (recent - F) / torch.maximum(torch.maximum(F.abs(), recent.abs()), torch.full_like(F, 1e-6)) <= tol
        gconv = pg_fn(x, g).abs().amax(1).double() / dot(x, x).sqrt().clamp_min(1.0) <= tol
        stop = (take & (fconv | gconv)) | (failed & failed_once)
        failed_once = torch.where(take, torch.zeros_like(failed_once), failed_once | failed)
        active = active & ~stop
        head = (head + 1) % m
        filled = min(filled + 1, m)
        if not bool(active.any()):
            break
    H = torch.stack(fhist).cpu()
    res = TrialResult(x=x, f=F, iterations=iters, n_evals=n_evals, history=H.mean(1).tolist(),
                      history_per_model=[H[:, b].tolist() for b in range(B)])
    res.rounds_per_iter = rounds_per_iter
    return res
