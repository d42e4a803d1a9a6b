"""LogisticRegression (multinomial / binomial, elastic net) — Spark ML semantics.

Reference: ``LogisticRegression(maxIter=20, regParam=0.3, elasticNetParam=0)``
(``Main/main.py:115-124``) and the 3x3 CrossValidator grid over regParam x
elasticNetParam (``Main/main.py:202-215``).  SURVEY.md C16/C18/N7.

Semantics reproduced from Spark's ``LogisticRegression.train``:

* family ``auto``: binomial for 2 classes, multinomial otherwise;
* ``standardization=True``: the problem is solved in the space of features
  scaled by 1/std (sample std over the training rows, no centering); features
  with std == 0 get coefficient 0; the L2 term ``0.5*(1-a)*reg*|beta_std|^2`` and
  L1 term ``a*reg*|beta_std|_1`` apply to standardized coefficients and never to
  the intercept;
* multinomial intercepts start at ``log1p(class_count) - mean`` and are centered
  after the fit;
* loss = weighted mean cross-entropy; optimizer L-BFGS (a = 0) / OWL-QN (a > 0),
  m = 10 corrections, ``maxIter``/``tol`` as given.

Design: ``fit_many`` trains B models (different row weights / regularization)
in one lock-stepped batched optimization on the device — the CrossValidator's
5 folds x 9 grid points are one problem of B = 45.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..data.table import Table
from ..ops import _native
from ..features.hybrid import HybridMatrix, hybrid_features
from ..features.hybrid import from_dense as hybrid_from_dense
from ..ops.logreg import DeviceLogregSolver, LogregDesign, SolverCacheEntry, logreg_margins_native, \
    native_classes_ok, pack_bucket, solver_cache_get, solver_cache_put, \
    unpack_bucket
from ..optim import lbfgs
from .base import ClassificationModel, ClassifierParams, Estimator, dp_allreduce, dp_context, dp_owner, dp_rows, \
    features_tensor, labels_tensor, new_uid, num_label_classes, resolve_device


@dataclass
class FitSpec:
    """One member of a batched fit."""
    row_weight: Optional[torch.Tensor]  # [N] weights (None = all ones)
    regParam: float
    elasticNetParam: float


class LogisticRegressionModel(ClassificationModel):
    def __init__(self, coefficientMatrix: torch.Tensor, interceptVector: torch.Tensor, binomial: bool,
                 uid: Optional[str] = None, device=None, summary: Optional[dict] = None):
        super().__init__(uid or new_uid("LogisticRegression"))
        f32 = torch.float32
        self.coefficientMatrix = coefficientMatrix if coefficientMatrix.dtype == f32 else coefficientMatrix.float()
        self.interceptVector = interceptVector if interceptVector.dtype == f32 else interceptVector.float()
        self.binomial = binomial
        self.num_classes = 2 if binomial else coefficientMatrix.shape[0]
        self.num_features = coefficientMatrix.shape[1]
        self.device = resolve_device(device) if device is not None else coefficientMatrix.device
        self.summary = summary or {}
        self.featuresCol = "features"

    @property
    def coefficients(self):
        return self.coefficientMatrix[0] if self.binomial else self.coefficientMatrix

    @property
    def intercept(self):
        return float(self.interceptVector[0]) if self.binomial else self.interceptVector

    def weight_table(self, KP: int) -> torch.Tensor:
        """[1, F+1, KP] effective weights of the evaluation kernel (row F = intercepts)."""
        W, b = self.coefficientMatrix, self.interceptVector
        out = torch.zeros(1, self.num_features + 1, KP, device=W.device)
        out[0, :self.num_features, :W.shape[0]] = W.T
        out[0, self.num_features, :W.shape[0]] = b
        return out

    def features_input(self, table):
        return hybrid_features(table, self.featuresCol, self.device)

    def predict_raw(self, X) -> torch.Tensor:
        """Margins (binomial: ``[-m, m]``).  ``X``: dense ``[N, F]`` or a HybridMatrix.  On the GPU
        the logreg_qn.hip evaluation kernel (prediction mode) runs for every input (dense columns of
        any width are staged through LDS in chunks)."""
        k = self.coefficientMatrix.shape[0]
        if isinstance(X, HybridMatrix) or X.is_cuda:
            hm = X if isinstance(X, HybridMatrix) else hybrid_from_dense(X.float(), [])
            if hm.device.type == "cuda" and native_classes_ok(k):
                KP = 8 if k <= 8 else 16
                m = logreg_margins_native(hm, self.weight_table(KP).to(hm.device), k, 1)[0, :, :k]
            else:
                Xd = hm.to_dense()
                m = Xd @ self.coefficientMatrix.to(Xd.device).T + self.interceptVector.to(Xd.device)
        else:
            m = X @ self.coefficientMatrix.to(X.device).T + self.interceptVector.to(X.device)
        if self.binomial:
            return torch.cat([-m, m], dim=1)
        return m

    def raw_to_probability(self, raw: torch.Tensor) -> torch.Tensor:
        if self.binomial:  # raw = [-m, m]
            p1 = torch.sigmoid(raw[:, 1:])
            return torch.cat([1 - p1, p1], dim=1)
        return torch.softmax(raw, dim=1)

    def __str__(self):
        return self.uid

    def state(self):
        return {"coefficientMatrix": self.coefficientMatrix.cpu(), "interceptVector": self.interceptVector.cpu(),
                "binomial": self.binomial}


_REG_CACHE = {}  # (device, per-spec (regParam, elasticNetParam)) -> [2, B] float32 device tensor


def _check_trials(t) -> None:
    if not isinstance(t, (int, np.integer)) or not 1 <= int(t) <= 4:
        raise ValueError(f"lineSearchTrials must be an integer in [1, 4] (the device solver evaluates at most 4 "
                         f"step lengths per line search), got {t!r}")


def _content_checksums(hm: HybridMatrix, y: torch.Tensor, specs, allreduce=None) -> List[float]:
    """Position-weighted fp64 checksums of the fit's data (dense features, one-hot column ids,
    labels and every spec's row weights — the CV fold masks), summed over ranks: a checkpoint
    fingerprint that changes with the data content and the fold assignment, not just its shape.
    Computed on the data's device."""
    dev = hm.device
    n = hm.n_rows
    pos = torch.arange(n, device=dev, dtype=torch.float64)  # shard-local: the fingerprint records the world size
    wr = torch.cos(pos * 0.6180339887) + 1.5  # distinct, bounded weight per row

    def cs(t: torch.Tensor) -> torch.Tensor:
        t = t.double().reshape(n, -1)
        t = torch.nan_to_num(t, nan=-7.0)
        colw = torch.sin(torch.arange(t.shape[1], device=dev, dtype=torch.float64) * 0.7548776662) + 2.0
        return (t * wr[:, None] * colw[None, :]).sum()

    parts = [cs(hm.dense) if hm.dense.numel() else torch.zeros((), dtype=torch.float64, device=dev),
             cs(hm.cat) if hm.cat.numel() else torch.zeros((), dtype=torch.float64, device=dev),
             cs(y)]
    for s in specs:
        parts.append(cs(s.row_weight) if s.row_weight is not None else torch.zeros((), dtype=torch.float64,
                                                                                   device=dev))
    v = torch.stack(parts)
    if allreduce is not None:
        allreduce(v)
    return [float(f"{x:.12g}") for x in v.cpu().tolist()]


class LogisticRegression(Estimator, ClassifierParams):
    _param_names = ("maxIter", "regParam", "elasticNetParam", "tol", "fitIntercept", "standardization", "family",
                    "featuresCol", "labelCol", "weightCol", "device", "lineSearchTrials", "lineSearch", "threshold",
                    "thresholds", "checkpointDir")

    def __init__(self, featuresCol="features", labelCol="label", maxIter: int = 100, regParam: float = 0.0,
                 elasticNetParam: float = 0.0, tol: float = 1e-6, fitIntercept: bool = True,
                 standardization: bool = True, family: str = "auto", weightCol: Optional[str] = None,
                 device=None, lineSearchTrials: int = 4, threshold: float = 0.5,
                 thresholds: Optional[Sequence[float]] = None, checkpointDir: Optional[str] = None,
                 lineSearch: str = "armijo"):
        super().__init__(new_uid("LogisticRegression"))
        # Spark: binary ``threshold`` t == thresholds [1 - t, t]; ``thresholds`` (any K) wins if set
        self.threshold, self.thresholds = threshold, thresholds
        # fit-level checkpoint: a finished batch of fits is saved (coefficients, intercepts,
        # summaries) under a fingerprint of its parameters and data; a rerun with the same
        # fingerprint (a restarted job) resumes by loading it instead of solving again
        self.checkpointDir = checkpointDir
        self.featuresCol, self.labelCol = featuresCol, labelCol
        self.maxIter, self.regParam, self.elasticNetParam = maxIter, regParam, elasticNetParam
        self.tol, self.fitIntercept, self.standardization = tol, fitIntercept, standardization
        self.family, self.weightCol, self.device = family, weightCol, device
        self.lineSearchTrials = lineSearchTrials  # step lengths 2^-t evaluated together per line search
        _check_trials(lineSearchTrials)
        # "armijo" (default, fast): lineSearchTrials step lengths per iteration in ONE batched evaluation,
        # the largest that satisfies Armijo; "wolfe": Breeze's searches — strong Wolfe (bracketing +
        # cubic zoom) for L-BFGS, projected backtracking with the Wolfe curvature condition for OWL-QN —
        # one trial per model per batched evaluation round (optim.lbfgs.minimize_wolfe)
        if lineSearch not in ("armijo", "wolfe"):
            raise ValueError(f"lineSearch must be 'armijo' or 'wolfe', got {lineSearch!r}")
        self.lineSearch = lineSearch

    # ------------------------------------------------------------------
    def fit(self, table: Table) -> LogisticRegressionModel:
        dev = resolve_device(self.device)
        hm = hybrid_features(table, self.featuresCol, dev)
        y = labels_tensor(table, self.labelCol, dev)
        w = None
        if self.weightCol:
            w = torch.as_tensor(table[self.weightCol].data.astype(np.float32), device=dev)
        num_classes = num_label_classes(table, self.labelCol, dev)
        lo, hi = dp_rows(hm.n_rows)  # data parallel: this rank's row shard + one all-reduce per evaluation
        model = self.fit_many(hm.rows(lo, hi), y[lo:hi], [FitSpec(None if w is None else w[lo:hi], self.regParam,
                                                                  self.elasticNetParam)], num_classes,
                              allreduce=dp_allreduce())[0]
        model.uid = self.uid
        return model

    def _apply_thresholds(self, model: "LogisticRegressionModel"):
        if self.thresholds is not None:
            model.setThresholds(self.thresholds)
        elif model.binomial and self.threshold != 0.5:
            model.setThresholds([1.0 - float(self.threshold), float(self.threshold)])
        return model

    def _setup(self, hm: HybridMatrix, y: torch.Tensor, specs: Sequence[FitSpec], K: int, allreduce, reuse=None):
        """Summarizer (+ its one all-reduce) -> standardization, masks, regularization vectors, x0.
        GPU: three HIP launches (logreg_setup.hip), no host round trip; CPU: the same math in torch.
        ``reuse`` (a solver-cache entry): its design, and its input buffers as the outputs."""
        dev = hm.device
        N, F = hm.n_rows, hm.n_features
        binomial = self.family == "binomial" or (self.family == "auto" and K <= 2)
        Kp = 2 if binomial else K
        B = len(specs)
        # device kernels for <= 16 classes on the GPU; wider problems run the torch objective on the
        # data's device (the CPU path's math), every spec's row weights materialized
        native = dev.type == "cuda" and native_classes_ok(Kp)
        if all(s.row_weight is None for s in specs) and native:
            rw = None                                                               # every row weight 1
        else:
            ones = None  # one fill for every unweighted spec (a CrossValidator batch has one per param map)

            def row_w(s):
                nonlocal ones
                if s.row_weight is not None:
                    return s.row_weight.to(dev).float()
                if ones is None:
                    ones = torch.ones(N, device=dev)
                return ones

            parts = [row_w(s) for s in specs]
            # the cached design: this fit's row weights stacked straight into its buffer (one launch)
            if reuse is not None and reuse.design.rw is not None and tuple(reuse.design.rw.shape) == (B, N):
                rw = torch.stack(parts, out=reuse.design.rw)
            else:
                rw = torch.stack(parts)                                               # [B, N]
        if reuse is not None:  # the cached design: this fit's row weights into its buffer
            design = reuse.design
            if rw is not None and (design.rw is None or rw.data_ptr() != design.rw.data_ptr()):
                design.rw.copy_(rw)
        else:
            design = LogregDesign(hm, y, rw, Kp, native=native)
        summ = design.summary()
        if allreduce is not None:
            allreduce(summ)
        D = Kp * (F + 1)
        if native:
            # (from pinned host memory: an asynchronous upload — from pageable memory the copy blocked the
            # host until the summary kernels ahead of it had run, ~30 us of idle GPU per fit in the trace)
            # (the per-spec regularization pairs on the device, cached by value: the pinned upload's host side
            # was ~40 us of every fit before the GPU got its first solver kernel)
            rkey = (str(dev), tuple((float(s.regParam), float(s.elasticNetParam)) for s in specs))
            reg_a = _REG_CACHE.get(rkey)
            if reg_a is None:
                reg_a = torch.tensor([[s.regParam for s in specs], [s.elasticNetParam for s in specs]],
                                     dtype=torch.float32).pin_memory().to(dev, non_blocking=True)
                if len(_REG_CACHE) >= 64:
                    _REG_CACHE.pop(next(iter(_REG_CACHE)))
                _REG_CACHE[rkey] = reg_a
            has_l1 = any(s.regParam * s.elasticNetParam > 0 for s in specs)
            if design.S != B:  # unweighted: one summary row serves every spec
                summ = summ.expand(B, -1).contiguous()
            if reuse is not None:
                inv_std, inv_wsum, pmask, l2v, l1v, x0 = reuse.bufs
            else:
                inv_std = torch.empty(B, F, device=dev)
                inv_wsum = torch.empty(B, device=dev)
                pmask = torch.empty(B, Kp, F + 1, device=dev)
                l2v = torch.empty(B, D, device=dev)
                l1v = torch.empty(B, D, device=dev) if has_l1 else None
                x0 = torch.empty(B, Kp, F + 1, device=dev)
            _native.kernels().logreg_prepare(summ.data_ptr(), reg_a[0].data_ptr(), reg_a[1].data_ptr(), B, F, Kp, Kp,
                                             int(self.standardization), int(self.fitIntercept), int(binomial),
                                             inv_std.data_ptr(), inv_wsum.data_ptr(), pmask.data_ptr(),
                                             l2v.data_ptr(), 0 if l1v is None else l1v.data_ptr(), x0.data_ptr(),
                                             _native.stream_ptr())
            return design, binomial, Kp, inv_std, inv_wsum, pmask, l2v, l1v, x0
        wsum = summ[:, 0]
        mean = summ[:, 1:1 + F] / wsum[:, None]
        ex2 = summ[:, 1 + F:1 + 2 * F] / wsum[:, None]
        counts = summ[:, 1 + 2 * F:].float()
        var = (ex2 - mean * mean) * (wsum / (wsum - 1).clamp_min(1.0))[:, None]
        std = var.clamp_min(0).sqrt().float()
        inv_wsum = (1.0 / wsum).float()
        if self.standardization:
            inv_std = torch.where(std > 0, 1.0 / std.clamp_min(1e-30), torch.zeros_like(std))
        else:
            inv_std = torch.where(std > 0, torch.ones_like(std), torch.zeros_like(std))
        reg = torch.tensor([s.regParam for s in specs], device=dev, dtype=torch.float32)
        alpha = torch.tensor([s.elasticNetParam for s in specs], device=dev, dtype=torch.float32)
        # parameters x[b] = [K, F+1] in standardized space (last column = intercept)
        x0 = torch.zeros(B, Kp, F + 1, device=dev)
        if self.fitIntercept:
            if binomial:
                p1 = (counts[:, 1] / counts.sum(1)).clamp(1e-12, 1 - 1e-12)
                x0[:, 1, F] = torch.log(p1 / (1 - p1))
            else:
                raw = torch.log1p(counts)
                x0[:, :, F] = raw - raw.mean(dim=1, keepdim=True)
        coef_mask = torch.ones(Kp, F + 1, device=dev)
        if not self.fitIntercept:
            coef_mask[:, F] = 0
        if binomial:  # pivot: class-0 row is fixed at zero
            coef_mask[0] = 0
        feat_mask = torch.cat([(inv_std > 0).float(), torch.ones(B, 1, device=dev)], dim=1)  # zero-std -> frozen
        pmask = coef_mask[None] * feat_mask[:, None, :]                                      # [B, Kp, F+1]
        notb = torch.ones(F + 1, device=dev)
        notb[F] = 0  # the intercept is never regularized
        l2v = ((reg * (1 - alpha))[:, None, None] * pmask * notb).reshape(B, D).contiguous()
        l1c = reg * alpha
        l1v = ((l1c[:, None, None] * pmask * notb).reshape(B, D).contiguous()
               if bool((l1c > 0).any()) else None)
        return design, binomial, Kp, inv_std, inv_wsum, pmask, l2v, l1v, x0 * pmask

    def fit_many(self, X, y: torch.Tensor, specs: Sequence[FitSpec], num_classes: Optional[int] = None,
                 allreduce=None, deferred: bool = False):
        """Train ``len(specs)`` models in one batched device optimization.

        ``deferred`` (device solver, no checkpoint): return ``(models, finalize)`` right after the
        solve is enqueued — the models' coefficients are device views already, their summaries
        (objective, iterations, history: host values) are filled by ``finalize()``, the one host
        sync.  A caller can enqueue work on the coefficients (the CrossValidator's fold scoring)
        before that sync, and the model objects are built while the GPU is still solving.

        ``X`` is a dense ``[N, F]`` tensor or a :class:`HybridMatrix` (one-hot indices + dense
        columns).  Data parallel: every rank passes its own row shard and ``allreduce`` (an
        in-place SUM over ranks, e.g. RCCL); the summarizer statistics and every batched
        objective evaluation's (loss, gradient) are summed across ranks — Spark's
        ``treeAggregate`` — and the replicated optimizer takes identical
        steps on every rank.
        """
        hm = X if isinstance(X, HybridMatrix) else hybrid_from_dense(X.float(), [])
        dev = hm.device
        F = hm.n_features
        K = int(num_classes or int(y.max()) + 1)
        _check_trials(self.lineSearchTrials)
        ckpt = fp = None
        if self.checkpointDir:
            import hashlib
            import json

            from ..utils.checkpoint import Checkpointer

            ctx = dp_context() if allreduce is not None else None
            fp = {"rows": int(hm.n_rows), "features": int(F), "classes": K, "maxIter": self.maxIter,
                  "tol": self.tol, "fitIntercept": self.fitIntercept, "standardization": self.standardization,
                  "family": self.family, "lineSearchTrials": self.lineSearchTrials,
                  "lineSearch": getattr(self, "lineSearch", "armijo"),
                  "specs": [[s.regParam, s.elasticNetParam, s.row_weight is None] for s in specs],
                  "content": _content_checksums(hm, y, specs, allreduce),
                  "world": ctx.world_size if ctx else 1}
            # one directory per fingerprint: the CV fits and the final refit of one job (and any
            # other fit sharing checkpointDir) never overwrite or resume each other
            key = hashlib.sha256(json.dumps(fp, sort_keys=True, default=str).encode()).hexdigest()[:16]
            ckpt = Checkpointer(os.path.join(self.checkpointDir, f"lr-{key}"), rank=ctx.rank if ctx else 0)
            last = ckpt.latest(fingerprint=fp)
            if last is not None:
                resumed = self._models_from_state(last[0], last[1], len(specs), dev)
                return (resumed, lambda: resumed) if deferred else resumed
        wolfe = getattr(self, "lineSearch", "armijo") == "wolfe"
        T = 1 if wolfe else max(1, int(self.lineSearchTrials))
        # repeated single-device fits on one resident design reuse the solver (ops/logreg.py)
        ckey = ent = None
        if (dev.type == "cuda" and allreduce is None and ckpt is None and not wolfe
                and native_classes_ok(2 if self.family == "binomial" or (self.family == "auto" and K <= 2) else K)):
            ckey = (id(hm), K, len(specs), T, self.maxIter, float(self.tol), self.family, self.fitIntercept,
                    self.standardization, any(s.regParam * s.elasticNetParam > 0 for s in specs),
                    any(s.row_weight is not None for s in specs), str(dev))
            ent = solver_cache_get(ckey, hm, y)
        design, binomial, Kp, inv_std, inv_wsum, pmask, l2v, l1v, x0 = self._setup(hm, y, specs, K, allreduce,
                                                                                    reuse=ent)
        B, D = len(specs), Kp * (F + 1)
        poll = 10 if self.maxIter > 20 else 0
        rounds = None

        def finish_coefs(xs):
            # every model's coefficients / intercepts in a few batched ops (per-model views below): a
            # 45-model CrossValidator otherwise pays ~4 small launches per model on the host
            xs = xs.view(B, Kp, F + 1) * pmask
            coef_all = xs[:, :, :F] * inv_std[:, None, :]
            icpt_all = xs[:, :, F].clone()
            if binomial:
                coef_all, icpt_all = coef_all[:, 1:2], icpt_all[:, 1:2]
            elif self.fitIntercept:
                icpt_all = icpt_all - icpt_all.mean(dim=1, keepdim=True)
            return xs, coef_all, icpt_all

        coefs_pre = pending = None
        if wolfe:
            if design.native:  # the evaluation kernels at each round's trial points (+ the DP all-reduce)
                solver = DeviceLogregSolver(design, B, 1, 10, inv_std, pmask, inv_wsum, l2v, l1v, self.maxIter,
                                            self.tol, allreduce=allreduce)
                evaluate = solver.evaluate_at
            else:
                def evaluate(xt):
                    loss, G = design.eval_torch(xt.view(-1, Kp, F + 1), 1, inv_std, pmask, inv_wsum)
                    if allreduce is not None:
                        bucket = pack_bucket(G, loss)
                        allreduce(bucket)
                        G2, loss = unpack_bucket(bucket, loss.numel(), G.shape)
                        G = G2.to(G.dtype)
                    return loss, G
            res = lbfgs.minimize_wolfe(evaluate, x0.reshape(B, D), l2v, l1v, max_iter=self.maxIter, m=10,
                                       tol=self.tol)
            xs, fobj, iters, n_evals = res.x, res.f, res.iterations, res.n_evals
            rounds = res.rounds_per_iter
            # as Spark's objectiveHistory: the start + one entry per iteration the model took (the batch
            # rows of a model that stopped earlier are cut by its own count, not by comparing values)
            history = [list(h)[: int(iters[bi]) + 1] for bi, h in enumerate(res.history_per_model)]
        elif design.native:
            if ent is not None:
                solver = ent.solver
                solver.reset()
            else:
                solver = DeviceLogregSolver(design, B, T, 10, inv_std, pmask, inv_wsum, l2v, l1v, self.maxIter,
                                            self.tol, allreduce=allreduce)
                if ckey is not None:
                    solver_cache_put(ckey, SolverCacheEntry(hm, y, design, solver,
                                                            (inv_std, inv_wsum, pmask, l2v, l1v, x0)))
            xs, fobj_d, iters_d = solver.solve(x0, poll=poll)
            n_evals = solver.n_evals
            # the coefficient post-processing enqueued BEFORE the host transfer (its sync): these
            # small kernels then run right behind the solve instead of one by one after it, with the GPU
            # idle between Python launches (LR fit kernel trace, profiles/r5/lr_grad_blocks.md)
            coefs_pre = finish_coefs(xs)
            # the cat is enqueued now; its host copy (the sync) waits until the models are built
            packed_d = torch.cat([solver.hist.reshape(-1), fobj_d.double(), iters_d.double()])

            def host_results():
                # objective history, objectives and iteration counts to the host in ONE transfer
                packed = packed_d.cpu()
                nh = solver.hist.numel()
                hist_h = packed[:nh].view(solver.hist.shape)
                fo, it = packed[nh:nh + B], packed[nh + B:].to(torch.int64)
                return fo, it, solver.histories(hist_h)

            pending = host_results
        else:
            def evaluate(xt):
                loss, G = design.eval_torch(xt.view(-1, Kp, F + 1), T if xt.shape[0] != B else 1, inv_std, pmask,
                                            inv_wsum)
                if allreduce is not None:  # ONE collective per evaluation: [gradients | exact losses]
                    bucket = pack_bucket(G, loss)
                    allreduce(bucket)
                    G2, loss = unpack_bucket(bucket, loss.numel(), G.shape)
                    G = G2.to(G.dtype)
                return loss, G

            res = lbfgs.minimize_trials(evaluate, x0.reshape(B, D), l2v, l1v, max_iter=self.maxIter, m=10,
                                        tol=self.tol, trials=T, poll=poll)
            xs, fobj, iters, n_evals = res.x, res.f, res.iterations, res.n_evals
            history = res.history_per_model  # each model's own objective per iteration
        xs, coef_all, icpt_all = coefs_pre if coefs_pre is not None else finish_coefs(xs)
        # per-model views in one unbind each: per-model tensor indexing was ~20 us of host time per
        # model (a 54-model CrossValidator batch).  Built before the host values are read, so on the
        # device solver this Python runs while the GPU is still solving
        coefs, icpts = coef_all.detach().unbind(0), icpt_all.detach().unbind(0)
        models = [self._apply_thresholds(LogisticRegressionModel(coefs[bi], icpts[bi], binomial, device=dev))
                  for bi in range(B)]

        def finalize():
            fo, it, hist = pending() if pending is not None else (fobj, iters, history)
            fobj_l, iters_l = fo.double().cpu().tolist(), it.cpu().tolist()
            for bi, mo in enumerate(models):
                mo.summary = {"objective": float(fobj_l[bi]), "iterations": int(iters_l[bi]), "n_evals": n_evals,
                              "objectiveHistory": hist[bi], "lineSearch": "wolfe" if wolfe else "armijo"}
                if rounds is not None:
                    mo.summary["lineSearchRounds"] = rounds  # batched evaluation rounds per iteration
            if ckpt is not None:
                st = {}
                for bi, mo in enumerate(models):
                    st[f"coef{bi}"], st[f"icpt{bi}"] = mo.coefficientMatrix, mo.interceptVector
                ckpt.save(1, st, {"binomial": binomial, "summaries": [dict(mo.summary) for mo in models]},
                          fingerprint=fp)
            return models

        if deferred:
            return models, finalize
        return finalize()

    def _models_from_state(self, st, meta, B: int, dev) -> List[LogisticRegressionModel]:
        out = []
        for bi in range(B):
            summary = dict(meta["summaries"][bi], resumed=True)
            summary.setdefault("objectiveHistory", [])  # checkpoints written before it was kept
            out.append(self._apply_thresholds(LogisticRegressionModel(
                st[f"coef{bi}"].to(dev), st[f"icpt{bi}"].to(dev), bool(meta["binomial"]), device=dev,
                summary=summary)))
        return out


__all__ = ["LogisticRegression", "LogisticRegressionModel", "FitSpec"]
