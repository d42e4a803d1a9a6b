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

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..data.table import Table
from ..ops import _native
from ..ops.logreg import LogregWorkspace, logreg_loss_grad_native, logreg_loss_grad_torch
from ..optim import lbfgs
from .base import ClassificationModel, ClassifierParams, Estimator, dp_allreduce, dp_context, dp_owner, dp_rows, \
    features_tensor, labels_tensor, new_uid, resolve_device


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
        self.coefficientMatrix = coefficientMatrix.float()  # [K, F] (binomial: [1, F])
        self.interceptVector = interceptVector.float()      # [K]
        self.binomial = binomial
        self.num_classes = 2 if binomial else coefficientMatrix.shape[0]
        self.num_features = coefficientMatrix.shape[1]
        self.device = resolve_device(device) if device is not None else coefficientMatrix.device
        self.summary = summary or {}

    @property
    def coefficients(self):
        return self.coefficientMatrix[0] if self.binomial else self.coefficientMatrix

    @property
    def intercept(self):
        return float(self.interceptVector[0]) if self.binomial else self.interceptVector

    def predict_raw(self, X: torch.Tensor) -> torch.Tensor:
        W = self.coefficientMatrix.to(X.device)
        b = self.interceptVector.to(X.device)
        if X.is_cuda and X.shape[1] % 4 == 0:
            from ..ops.gemm import EPI_BIAS_F32, gemm_f32
            rows = max(8, (W.shape[0] + 7) // 8 * 8)
            Wp = torch.zeros(rows, W.shape[1], device=X.device)
            Wp[: W.shape[0]] = W
            bp = torch.zeros(rows, device=X.device)
            bp[: b.shape[0]] = b
            Z = torch.empty(X.shape[0], rows, device=X.device)
            gemm_f32(X.contiguous(), Wp, Z, M=X.shape[0], N=rows, K=X.shape[1], layout=0, epi=EPI_BIAS_F32, bias=bp)
            m = Z[:, : W.shape[0]]
        else:
            m = X @ W.T + b
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


class LogisticRegression(Estimator, ClassifierParams):
    _param_names = ("maxIter", "regParam", "elasticNetParam", "tol", "fitIntercept", "standardization", "family",
                    "featuresCol", "labelCol", "weightCol", "device")

    def __init__(self, featuresCol="features", labelCol="label", maxIter: int = 100, regParam: float = 0.0,
                 elasticNetParam: float = 0.0, tol: float = 1e-6, fitIntercept: bool = True,
                 standardization: bool = True, family: str = "auto", weightCol: Optional[str] = None,
                 device=None):
        super().__init__(new_uid("LogisticRegression"))
        self.featuresCol, self.labelCol = featuresCol, labelCol
        self.maxIter, self.regParam, self.elasticNetParam = maxIter, regParam, elasticNetParam
        self.tol, self.fitIntercept, self.standardization = tol, fitIntercept, standardization
        self.family, self.weightCol, self.device = family, weightCol, device

    # ------------------------------------------------------------------
    def fit(self, table: Table) -> LogisticRegressionModel:
        dev = resolve_device(self.device)
        X = features_tensor(table, self.featuresCol, dev)
        y = labels_tensor(table, self.labelCol, dev)
        w = None
        if self.weightCol:
            w = torch.as_tensor(table[self.weightCol].data.astype(np.float32), device=dev)
        num_classes = int(max(int(y.max()) + 1, len((table[self.labelCol].meta or {}).get("vocab") or [])))
        lo, hi = dp_rows(X.shape[0])  # data parallel: this rank's row shard + one all-reduce per evaluation
        model = self.fit_many(X[lo:hi], y[lo:hi], [FitSpec(None if w is None else w[lo:hi], self.regParam,
                                                           self.elasticNetParam)], num_classes,
                              allreduce=dp_allreduce())[0]
        model.uid = self.uid
        return model

    def fit_many(self, X: torch.Tensor, y: torch.Tensor, specs: Sequence[FitSpec],
                 num_classes: Optional[int] = None, allreduce=None) -> List[LogisticRegressionModel]:
        """Train ``len(specs)`` models in one batched device optimization.

        Data parallel: every rank passes its own row shard and ``allreduce`` (an
        in-place SUM over ranks, e.g. RCCL); the summarizer statistics and every
        objective evaluation's (loss, gradient) bucket are summed across ranks —
        Spark's ``treeAggregate`` as ONE flat all-reduce — and
        the replicated optimizer then takes identical steps on every rank.
        """
        dev = X.device
        N, F = X.shape
        K = int(num_classes or int(y.max()) + 1)
        binomial = self.family == "binomial" or (self.family == "auto" and K <= 2)
        Kp = 2 if binomial else K
        B = len(specs)
        rw = torch.stack([torch.ones(N, device=dev) if s.row_weight is None else s.row_weight.to(dev).float()
                          for s in specs])                                            # [B, N]
        # weighted summarizer (Spark: MultivariateOnlineSummarizer + MultiClassSummarizer), fp64
        rwd = rw.double()
        counts = torch.zeros(B, Kp, device=dev, dtype=torch.float64)
        counts.scatter_add_(1, y.view(1, -1).expand(B, -1).clamp_max(Kp - 1), rwd)
        summ = torch.cat([rwd.sum(dim=1, keepdim=True), rwd @ X.double(), rwd @ (X.double() ** 2), counts], dim=1)
        if allreduce is not None:
            allreduce(summ)
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
        l2 = reg * (1 - alpha)
        l1_coef = reg * alpha
        D = Kp * (F + 1)
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
        coef_mask = coef_mask.expand(B, Kp, F + 1)
        feat_mask = torch.cat([(inv_std > 0).float(), torch.ones(B, 1, device=dev)], dim=1)  # zero-std -> frozen
        pmask = coef_mask * feat_mask[:, None, :]
        l1 = None
        if bool((l1_coef > 0).any()):
            l1 = torch.zeros(B, Kp, F + 1, device=dev)
            l1[:, :, :F] = l1_coef[:, None, None]
            l1 = (l1 * pmask).reshape(B, D)

        y32 = y.to(torch.int32).contiguous()
        use_native = X.is_cuda and F % 4 == 0
        ws = LogregWorkspace(X, B, Kp) if use_native else None
        Xc = X.contiguous()

        def objective(xflat):
            xv = xflat.view(B, Kp, F + 1) * pmask
            beta = xv[:, :, :F]
            W_eff = beta * inv_std[:, None, :]
            b = xv[:, :, F]
            if use_native:
                loss, gW, gb = logreg_loss_grad_native(Xc, y32, W_eff, b, rw, inv_wsum, ws)
            else:
                loss, gW, gb = logreg_loss_grad_torch(Xc, y, W_eff, b, rw, inv_wsum)
            if allreduce is not None:  # one flat bucket: [loss | dW | db] for all B models
                flat = torch.cat([loss.float().view(B, 1), gW.reshape(B, -1), gb.reshape(B, -1)], dim=1)
                allreduce(flat)
                loss = flat[:, 0]
                gW = flat[:, 1:1 + Kp * F].view(B, Kp, F)
                gb = flat[:, 1 + Kp * F:].view(B, Kp)
            gbeta = gW * inv_std[:, None, :] + l2[:, None, None] * beta
            loss = loss + 0.5 * l2 * (beta * beta).sum(dim=(1, 2))
            g = torch.cat([gbeta, gb.unsqueeze(2)], dim=2) * pmask
            return loss, g.reshape(B, D)

        res = lbfgs.minimize(objective, x0.reshape(B, D), max_iter=self.maxIter, m=10, tol=self.tol, l1=l1)
        xs = res.x.view(B, Kp, F + 1) * pmask
        models = []
        for bi in range(B):
            coef = xs[bi, :, :F] * inv_std[bi][None, :]
            icpt = xs[bi, :, F].clone()
            if binomial:
                coef, icpt = coef[1:2], icpt[1:2]
            elif self.fitIntercept:
                icpt = icpt - icpt.mean()
            summary = {"objective": float(res.f[bi]), "iterations": int(res.iterations[bi]),
                       "n_evals": res.n_evals, "objectiveHistory": res.history}
            models.append(LogisticRegressionModel(coef.detach(), icpt.detach(), binomial, device=dev,
                                                  summary=summary))
        return models


__all__ = ["LogisticRegression", "LogisticRegressionModel", "FitSpec"]
