"""Spark-compatible evaluators plus the single ``evaluate_all`` path.

The reference repeats ~60 lines of evaluator boilerplate per model, six times
(``Main/main.py:132-195`` and copies).  Here one call computes
every number those blocks print — 3 binary, 4 multiclass, 4 regression metrics
and the "Additional Factors" counts — from one confusion matrix, one moment
reduction and one sort.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass
from typing import Dict, Optional

import numpy as np

from ..data.table import Table
from . import metrics as M


class Evaluator:
    metricName: str = ""

    def evaluate(self, table: Table, params: Optional[Dict] = None) -> float:
        raise NotImplementedError

    def isLargerBetter(self) -> bool:
        return True

    def evaluate_batched(self, label, pred, mask, num_classes: int, raw=None, host: bool = True):
        """This evaluator's metric for B models at once (``pred``/``mask`` [B, N]); the
        CrossValidator scores all (param map, fold) models with one call.  ``host=False`` may return
        a device tensor (regression metrics: no host read inside)."""
        return M.batched_metrics(self._metric(None), label, pred, mask, num_classes, raw, host=host)

    def _metric(self, params):
        if params:
            for k, v in params.items():
                if k in ("metricName", getattr(self, "_metric_key", "metricName")):
                    return v
        return self.metricName


class BinaryClassificationEvaluator(Evaluator):
    def __init__(self, labelCol="label", rawPredictionCol="rawPrediction", metricName="areaUnderROC"):
        self.labelCol, self.rawPredictionCol, self.metricName = labelCol, rawPredictionCol, metricName

    def evaluate(self, table: Table, params=None) -> float:
        raw = table[self.rawPredictionCol].data
        score = raw[:, 1] if raw.ndim == 2 else raw
        return M.binary_metrics(score, table[self.labelCol].data)[self._metric(params)]


class MulticlassClassificationEvaluator(Evaluator):
    def __init__(self, labelCol="label", predictionCol="prediction", metricName="f1"):
        self.labelCol, self.predictionCol, self.metricName = labelCol, predictionCol, metricName

    def evaluate(self, table: Table, params=None) -> float:
        y = table[self.labelCol].data.astype(np.int64)
        p = table[self.predictionCol].data.astype(np.int64)
        K = int(max(y.max(initial=0), p.max(initial=0)) + 1)
        return M.multiclass_metrics(y, p, K)[self._metric(params)]


class RegressionEvaluator(Evaluator):
    def __init__(self, labelCol="label", predictionCol="prediction", metricName="rmse"):
        self.labelCol, self.predictionCol, self.metricName = labelCol, predictionCol, metricName

    def evaluate(self, table: Table, params=None) -> float:
        return M.regression_metrics(table[self.labelCol].data, table[self.predictionCol].data)[self._metric(params)]

    def isLargerBetter(self) -> bool:
        return self.metricName in ("r2", "var")


@dataclass
class MetricsRecord:
    """Every number one reference evaluation block prints."""
    raw_prediction: float       # BinaryClassificationEvaluator() default metric (= areaUnderROC)
    area_under_pr: float
    area_under_roc: float
    f1: float
    weighted_precision: float
    weighted_recall: float
    accuracy: float
    rmse: float
    mse: float
    r2: float
    mae: float
    count_total: int
    correct: int
    wrong: int
    ratio_wrong: float
    ratio_correct: float

    def as_dict(self):
        return asdict(self)


def evaluate_all(label, prediction, raw_prediction, num_classes: int) -> MetricsRecord:
    """``label``/``prediction`` [N] and ``raw_prediction`` [N, K] (tensors or arrays, any device)."""
    import torch

    lab = torch.as_tensor(label)
    pred = torch.as_tensor(prediction).to(lab.device)
    raw = torch.as_tensor(raw_prediction)
    cm = M.confusion_matrix(lab, pred, num_classes)
    mc = M.multiclass_from_confusion(cm)
    score = raw[:, 1] if raw.ndim == 2 and raw.shape[1] > 1 else raw.reshape(-1)
    bn = M.binary_metrics(score, lab)
    rg = M.regression_metrics(lab, pred)
    n = int(lab.numel())
    correct = int(torch.diag(cm).sum())
    wrong = n - correct
    return MetricsRecord(raw_prediction=bn["areaUnderROC"], area_under_pr=bn["areaUnderPR"],
                         area_under_roc=bn["areaUnderROC"], f1=mc["f1"], weighted_precision=mc["weightedPrecision"],
                         weighted_recall=mc["weightedRecall"], accuracy=mc["accuracy"], rmse=rg["rmse"],
                         mse=rg["mse"], r2=rg["r2"], mae=rg["mae"], count_total=n, correct=correct, wrong=wrong,
                         ratio_wrong=wrong / n if n else 0.0, ratio_correct=correct / n if n else 0.0)
