"""NaiveBayes (multinomial / bernoulli / gaussian) — new capability (BASELINE.json
north star; not in the reference script).  API and math follow Spark ML's
``NaiveBayes(smoothing=1.0, modelType="multinomial")``.

Fitting is one pass of class-conditional moments: counts, sum x and sum x^2
per class are two products ``onehot(y)^T . [X, X^2]``; the
Gaussian model adds a second pass over the centred rows ``x - mu_y`` so its
variances are two-pass accurate — on the GPU
an exact-fp32 MFMA split-K GEMM (``har_gemm_f32``).  Scoring is a GEMM as well:
``raw = [X, X^2] . Theta^T + b``.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from ..data.table import Table
from ..ops.gemm import EPI_BIAS_F32, EPI_F32_SLAB, auto_k_split, gemm_f32
from .base import ClassificationModel, ClassifierParams, Estimator, dp_allreduce, dp_context, dp_owner, dp_rows, \
    features_tensor, labels_tensor, new_uid, num_label_classes, resolve_device


def _pad4(x: int) -> int:
    return (x + 3) // 4 * 4


def class_moments(X: torch.Tensor, y: torch.Tensor, K: int, w: Optional[torch.Tensor] = None):
    """(counts [K], sum x [K, F], sum x^2 [K, F]) with optional row weights."""
    N, F = X.shape
    Y = torch.zeros(N, K, dtype=torch.float32, device=X.device)
    Y[torch.arange(N, device=X.device), y.long()] = 1.0 if w is None else w.float()
    if X.is_cuda:
        Kp, Fp = _pad4(K), _pad4(2 * F)
        Yp = torch.zeros(N, Kp, device=X.device)
        Yp[:, :K] = Y
        XX = torch.zeros(N, Fp, device=X.device)
        XX[:, :F] = X
        XX[:, F:2 * F] = X * X
        # deterministic split-K: every batch slice writes its partial [Kp, Fp] tile into its own
        # slab (plain stores), then one fixed-order sum over the slabs — bitwise reproducible,
        # unlike float atomics
        ks = auto_k_split(Kp, Fp, N)
        splits = (N + ks - 1) // ks
        slabs = torch.empty(splits, Kp, Fp, device=X.device)
        gemm_f32(Yp, XX, slabs, M=Kp, N=Fp, K=N, layout=3, epi=EPI_F32_SLAB, k_split=ks, ldc=Fp,
                 slab_stride=Kp * Fp)
        S = slabs.sum(0)
        return Y.sum(0), S[:K, :F], S[:K, F:2 * F]
    return Y.sum(0), Y.T @ X, Y.T @ (X * X)


class NaiveBayesModel(ClassificationModel):
    def __init__(self, pi: torch.Tensor, theta: torch.Tensor, sigma: Optional[torch.Tensor], modelType: str,
                 uid=None, device=None):
        super().__init__(uid or new_uid("NaiveBayes"))
        self.pi, self.theta, self.sigma, self.modelType = pi, theta, sigma, modelType
        self.num_classes, self.num_features = theta.shape
        self.device = device or theta.device
        # scoring as one GEMM: raw = [X, X^2] . Wt^T + bias
        if modelType == "gaussian":
            inv = 1.0 / sigma
            W1 = theta * inv                       # x * mu / var
            W2 = -0.5 * inv                        # x^2 * (-1/(2 var))
            bias = pi - 0.5 * (torch.log(2 * math.pi * sigma) + theta * theta * inv).sum(1)
        elif modelType == "bernoulli":
            # log p(x=1) x + log(1-p) (1-x) = x (theta - log1m) + sum log1m
            log1m = torch.log1p(-torch.exp(theta))
            W1, W2 = theta - log1m, torch.zeros_like(theta)
            bias = pi + log1m.sum(1)
        else:  # multinomial
            W1, W2 = theta, torch.zeros_like(theta)
            bias = pi.clone()
        self._W = torch.cat([W1, W2], dim=1).float()
        self._b = bias.float()

    def predict_raw(self, X):
        X = X.to(self.device).float()
        K, F = self.theta.shape
        if self.modelType == "bernoulli" and bool(((X != 0) & (X != 1)).any()):
            raise ValueError("Bernoulli NaiveBayes requires 0/1 features")
        if X.is_cuda:
            Fp = _pad4(2 * F)
            Kp = max(8, (K + 7) // 8 * 8)
            XX = torch.zeros(X.shape[0], Fp, device=X.device)
            XX[:, :F] = X
            XX[:, F:2 * F] = X * X
            Wp = torch.zeros(Kp, Fp, device=X.device)
            Wp[:K, :2 * F] = self._W.to(X.device)
            bp = torch.zeros(Kp, device=X.device)
            bp[:K] = self._b.to(X.device)
            out = torch.empty(X.shape[0], Kp, device=X.device)
            gemm_f32(XX, Wp, out, M=X.shape[0], N=Kp, K=Fp, layout=0, epi=EPI_BIAS_F32, bias=bp)
            return out[:, :K]
        return torch.cat([X, X * X], 1) @ self._W.to(X.device).T + self._b.to(X.device)

    def raw_to_probability(self, raw):
        return torch.softmax(raw, dim=1)

    def __str__(self):
        return f"NaiveBayesModel (uid={self.uid}) with {self.num_classes} classes"

    def state(self):
        return {"pi": self.pi.cpu(), "theta": self.theta.cpu(),
                "sigma": None if self.sigma is None else self.sigma.cpu(), "modelType": self.modelType}


class NaiveBayes(Estimator, ClassifierParams):
    _param_names = ("smoothing", "modelType", "featuresCol", "labelCol", "weightCol", "device")

    def __init__(self, featuresCol="features", labelCol="label", smoothing: float = 1.0,
                 modelType: str = "multinomial", weightCol: Optional[str] = None, device=None):
        super().__init__(new_uid("NaiveBayes"))
        if modelType not in ("multinomial", "bernoulli", "gaussian"):
            raise ValueError(f"unknown modelType {modelType}")
        self.featuresCol, self.labelCol = featuresCol, labelCol
        self.smoothing, self.modelType, self.weightCol, self.device = smoothing, modelType, weightCol, device

    def fit(self, table: Table) -> NaiveBayesModel:
        dev = resolve_device(self.device)
        X = features_tensor(table, self.featuresCol, dev)
        y = labels_tensor(table, self.labelCol, dev)
        K = num_label_classes(table, self.labelCol, dev)
        w = None
        if self.weightCol:
            w = torch.as_tensor(table[self.weightCol].data, dtype=torch.float32, device=dev)
        lo, hi = dp_rows(X.shape[0])  # data parallel: per-class moments of the shard, one all-reduce
        m = self.fit_tensors(X[lo:hi], y[lo:hi], K, None if w is None else w[lo:hi], allreduce=dp_allreduce())
        m.uid = self.uid
        return m

    def _prep(self, table: Table):
        dev = resolve_device(self.device)
        return (features_tensor(table, self.featuresCol, dev), labels_tensor(table, self.labelCol, dev),
                num_label_classes(table, self.labelCol, dev))

    def fit_folds(self, X, y, K, masks: torch.Tensor):
        """One model per CrossValidator fold (``masks`` [k, N]: 1 = training row of fold f) from the
        full device matrices with the fold mask as row weights — no per-fold row gather; the
        CrossValidator then scores every fold's validation rows in one batched pass (data parallel:
        each rank's row shard, moments all-reduced)."""
        lo, hi = dp_rows(X.shape[0])
        out = []
        for f in range(masks.shape[0]):
            m = self.fit_tensors(X[lo:hi], y[lo:hi], K, masks[f, lo:hi], allreduce=dp_allreduce())
            m.uid = self.uid
            out.append(m)
        return out

    def fit_tensors(self, X, y, K, w=None, allreduce=None) -> NaiveBayesModel:
        """``allreduce`` (in-place SUM over ranks): X/y/w are this rank's shard and the
        class counts / first / second moments are summed in ONE flat bucket."""
        lam = float(self.smoothing)
        if self.modelType in ("multinomial", "bernoulli") and bool((X < 0).any()):
            raise ValueError(f"{self.modelType} NaiveBayes requires nonnegative feature values")
        n, s1, s2 = class_moments(X.float(), y, K, w)
        n, s1, s2 = n.double(), s1.double(), s2.double()
        if allreduce is not None:
            F = X.shape[1]
            buf = torch.cat([n.reshape(-1), s1.reshape(-1), s2.reshape(-1)])
            allreduce(buf)
            n, s1, s2 = buf[:K], buf[K:K + K * F].view(K, F), buf[K + K * F:].view(K, F)
        N = float(n.sum())
        pi = torch.log((n + lam) / (N + lam * K))
        sigma = None
        if self.modelType == "multinomial":
            theta = torch.log((s1 + lam) / (s1.sum(1, keepdim=True) + lam * X.shape[1]))
        elif self.modelType == "bernoulli":
            theta = torch.log((s1 + lam) / (n[:, None] + 2 * lam))
        else:
            pi = torch.log(n / N)
            mu = s1 / n.clamp_min(1)[:, None]
            # second pass over the rows: centred moments sum_i w_i (x_i - mu_{y_i})^2, so the
            # variance does not cancel the way E[x^2] - mu^2 does for large-mean features
            D = X.float() - mu.float()[y.long()]
            _, _, c2 = class_moments(D, y, K, w)
            c2 = c2.double()
            if allreduce is not None:
                allreduce(c2)
            var = (c2 / n.clamp_min(1)[:, None]).clamp_min(0)
            eps = 1e-9 * float(var.max()) if var.numel() else 1e-9
            # global variance floor (sklearn/Spark style epsilon) keeps constant features finite
            var = var + max(eps, 1e-12)
            theta, sigma = mu, var
        return NaiveBayesModel(pi.float(), theta.float(), None if sigma is None else sigma.float(),
                               self.modelType, device=X.device)
