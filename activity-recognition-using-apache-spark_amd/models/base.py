"""Estimator / Model / Transformer base classes (the Spark ML surface used by
``Main/main.py``: ``Estimator.fit(df) -> Model``, ``Model.transform(df)`` adding
``rawPrediction``, ``probability`` and ``prediction`` — ``result.txt:147-151``)."""
from __future__ import annotations

import copy
import random
import secrets
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from ..data.table import Column, DeviceColumn, Table


# uid generator: seeded once from the OS entropy pool, then 80 random bits per uid (a urandom
# syscall per uid cost ~5 us, paid 54 times by a CrossValidator's batched LR fit)
_UID_RNG = random.Random(secrets.randbits(128))


def new_uid(prefix: str) -> str:
    """Spark-style uid: ``<Class>_<20 hex chars>`` (e.g. ``LogisticRegression_446cab28d15c5195e1ba``)."""
    return f"{prefix}_{_UID_RNG.getrandbits(80):020x}"


def resolve_device(device=None) -> torch.device:
    if isinstance(device, torch.device):
        return device
    if device is None or device == "auto":
        return torch.device("cuda" if torch.cuda.is_available() else "cpu")
    return torch.device(device)


class Params:
    """Minimal Spark ``Params``: named parameters, ``copy(extra)``, ``set``."""

    _param_names: Tuple[str, ...] = ()

    def params(self) -> Dict:
        return {k: getattr(self, k) for k in self._param_names if hasattr(self, k)}

    def set(self, **kw):
        for k, v in kw.items():
            if self._param_names and k not in self._param_names:
                raise KeyError(f"{type(self).__name__} has no param {k}")
            setattr(self, k, v)
        return self

    def copy(self, extra: Optional[Dict] = None):
        c = copy.copy(self)
        if extra:
            c.set(**extra)
        return c


class Transformer(Params):
    def __init__(self, uid: Optional[str] = None):
        self.uid = uid or new_uid(type(self).__name__)

    def transform(self, table: Table) -> Table:  # pragma: no cover - abstract
        raise NotImplementedError

    def __str__(self):
        return self.uid


class Estimator(Params):
    def __init__(self, uid: Optional[str] = None):
        self.uid = uid or new_uid(type(self).__name__)

    def fit(self, table: Table):  # pragma: no cover - abstract
        raise NotImplementedError

    def __str__(self):
        return self.uid


class Model(Transformer):
    def state(self) -> Dict:
        return {}


# ---------------------------------------------------------------------------
# Data-parallel scope.  Inside ``with data_parallel(ctx):`` every ``Estimator.fit(table)``
# (and CrossValidator's batched fits) trains on this rank's contiguous row shard and
# combines its partial statistics with collectives over ``ctx`` (RCCL on GPUs, gloo on
# CPU) — the analogue of Spark running the same ``fit`` over partitioned RDDs with
# ``treeAggregate`` / ``reduceByKey``.  Every rank holds the whole
# (small) input table; global row ids stay meaningful, so split / fold / bootstrap draws
# are the same as in one process.
_DP_CTX = None


class data_parallel:
    def __init__(self, ctx):
        self.ctx = ctx if (ctx is not None and ctx.is_distributed) else None

    def __enter__(self):
        global _DP_CTX
        self._prev, _DP_CTX = _DP_CTX, self.ctx
        return self.ctx

    def __exit__(self, *exc):
        global _DP_CTX
        _DP_CTX = self._prev
        return False


def dp_context():
    """The active distributed context (None outside ``data_parallel`` or for world size 1)."""
    return _DP_CTX


def dp_rows(n: int) -> Tuple[int, int]:
    """This rank's contiguous [lo, hi) share of ``n`` rows (all rows outside DP)."""
    ctx = _DP_CTX
    if ctx is None:
        return 0, n
    return (n * ctx.rank) // ctx.world_size, (n * (ctx.rank + 1)) // ctx.world_size


def dp_allreduce():
    """In-place SUM over ranks (None outside DP)."""
    if _DP_CTX is None:
        return None
    from ..parallel.data_parallel import allreduce_sum

    return allreduce_sum(_DP_CTX)


def dp_owner():
    """Owner-computes node communicator for tree levels (None outside DP)."""
    if _DP_CTX is None:
        return None
    from ..parallel.data_parallel import NodeOwner

    return NodeOwner(_DP_CTX)


def features_tensor(table: Table, col: str, device, dtype=torch.float32) -> torch.Tensor:
    """Device matrix of a feature column, transferred once per (column, device, dtype) and cached
    on the column (HBM-resident for every later fit / predict — SURVEY.md N12)."""
    c = table[col]
    key = ("dense", str(device), str(dtype))
    hit = c.cache.get(key) if c.cache is not None else None
    if hit is not None:
        return hit
    if isinstance(c, DeviceColumn):  # already in HBM: densify the hybrid layout on the device
        t = (c.hybrid.to_dense() if c.kind == "vector" else c.tensor[:, None]).to(device=device, dtype=dtype)
        t = t.contiguous()
    else:
        arr = c.data if c.kind == "vector" else c.data[:, None]
        t = torch.as_tensor(np.ascontiguousarray(arr, dtype=np.float32)).to(device=device, dtype=dtype)
    if c.cache is not None:
        c.cache[key] = t
    return t


def labels_tensor(table: Table, col: str, device) -> torch.Tensor:
    """int64 label tensor of ``col`` on ``device``, cached on the (immutable) column."""
    c = table[col]
    key = ("labels", str(device))
    cache = getattr(c, "cache", None)
    if cache is not None and key in cache:
        return cache[key]
    if isinstance(c, DeviceColumn):
        t = c.tensor.to(device=device, dtype=torch.int64)
    else:
        t = torch.as_tensor(c.data.astype(np.int64)).to(device)
    if cache is not None:
        cache[key] = t
    return t


def num_label_classes(table: Table, col: str, device) -> int:
    """max(label) + 1, at least the indexer vocabulary size — cached on the column, so a fit on a
    resident table does not wait on a device -> host read before its first launch."""
    c = table[col]
    cache = getattr(c, "cache", None)
    key = ("num_classes", str(device))
    if cache is not None and key in cache:
        return cache[key]
    y = labels_tensor(table, col, device)
    k = int(max(int(y.max()) + 1 if y.numel() else 0, len((c.meta or {}).get("vocab") or [])))
    if cache is not None:
        cache[key] = k
    return k


class ClassifierParams(Params):
    featuresCol = "features"
    labelCol = "label"
    predictionCol = "prediction"
    probabilityCol = "probability"
    rawPredictionCol = "rawPrediction"


class ClassificationModel(Model, ClassifierParams):
    """``transform`` = one device pass producing raw scores, probabilities, argmax."""

    num_classes: int = 0
    num_features: int = 0
    device: torch.device = torch.device("cpu")

    def predict_raw(self, X: torch.Tensor) -> torch.Tensor:  # pragma: no cover - abstract
        raise NotImplementedError

    def raw_to_probability(self, raw: torch.Tensor) -> torch.Tensor:
        s = raw.sum(dim=1, keepdim=True)
        return torch.where(s > 0, raw / s.clamp_min(1e-300), torch.full_like(raw, 1.0 / raw.shape[1]))

    # Spark ProbabilisticClassificationModel.thresholds: the class with the largest p / t wins; a
    # zero threshold makes its class win wherever its probability is positive.  None = argmax(p).
    thresholds = None

    def setThresholds(self, value):
        if value is not None:
            t = [float(v) for v in value]
            if any(v < 0 for v in t) or sum(1 for v in t if v == 0) > 1:
                raise ValueError("thresholds must be >= 0 with at most one zero")
            value = t
        self.thresholds = value
        return self

    def _predict_from_probability(self, prob: torch.Tensor) -> torch.Tensor:
        if self.thresholds is None:
            return torch.argmax(prob, dim=1)
        t = torch.as_tensor(self.thresholds, dtype=prob.dtype, device=prob.device)
        if t.numel() != prob.shape[1]:
            raise ValueError(f"{t.numel()} thresholds for {prob.shape[1]} classes")
        scaled = torch.where(t > 0, prob / t.clamp_min(1e-300),
                             torch.where(prob > 0, torch.full_like(prob, float("inf")), torch.zeros_like(prob)))
        return torch.argmax(scaled, dim=1)

    def predict_all(self, X: torch.Tensor):
        raw = self.predict_raw(X)
        prob = self.raw_to_probability(raw)
        pred = self._predict_from_probability(prob)
        return raw, prob, pred

    def predict(self, X: torch.Tensor) -> torch.Tensor:
        return self.predict_all(X)[2]

    def features_input(self, table: Table):
        """What ``predict_all`` consumes for ``table`` (the cached dense device matrix by default)."""
        return features_tensor(table, self.featuresCol, self.device)

    def transform(self, table: Table) -> Table:
        raw, prob, pred = self.predict_all(self.features_input(table))
        t = table.with_column(Column(self.rawPredictionCol, "vector", raw.double().cpu().numpy()))
        t = t.with_column(Column(self.probabilityCol, "vector", prob.double().cpu().numpy()))
        return t.with_column(Column(self.predictionCol, "double", pred.double().cpu().numpy(),
                                    meta={"nullable": False}))
