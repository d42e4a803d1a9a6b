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
