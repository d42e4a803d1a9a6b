"""Metric definitions (Spark MLlib semantics) over device or host tensors.

* multiclass — ``MulticlassMetrics``: confusion matrix from (prediction, label);
  weighted precision/recall/F1 weight each *true* label by its frequency;
  precision of a class never predicted is 0; weightedRecall == accuracy.
  Used by ``MulticlassClassificationEvaluator`` (``Main/main.py:146-156``).
* binary — ``BinaryClassificationMetrics`` as the reference calls it on a
  6-class model (``Main/main.py:135-143``): score = ``rawPrediction[1]``,
  positive iff label > 0.5; scores sorted descending with ties grouped; ROC
  gets (0,0)/(1,1) end points, PR starts at (0, precision of the first
  threshold); areas by the trapezoid rule; precision with no predicted
  positives is 1.0.
* regression — ``RegressionMetrics`` on class indices: rmse, mse, r2
  (``1 - SS_err / SS_tot``), mae (``Main/main.py:158-177``).

On the GPU the confusion matrix and the regression moments are single HIP
reductions (``csrc/kernels/metrics.hip``); the ROC/PR curve is a device sort +
one HIP pass over the sorted scores (``csrc/kernels/roc.hip``).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch

from ..ops import metrics as mops


def _t(x, dtype=None):
    t = torch.as_tensor(np.asarray(x)) if not isinstance(x, torch.Tensor) else x
    return t if dtype is None else t.to(dtype)


def confusion_matrix(label, pred, num_classes: int) -> torch.Tensor:
    label = _t(label).to(torch.int64)
    pred = _t(pred).to(torch.int64)
    return mops.confusion_matrix(label, pred, num_classes)


def multiclass_from_confusion(cm: torch.Tensor) -> Dict[str, float]:
    cm = cm.double().cpu()
    n = cm.sum()
    tp = torch.diag(cm)
    label_count = cm.sum(dim=1)   # rows = true label
    pred_count = cm.sum(dim=0)    # cols = prediction
    present = label_count > 0
    prec = torch.where(pred_count > 0, tp / pred_count.clamp_min(1), torch.zeros_like(tp))
    rec = torch.where(label_count > 0, tp / label_count.clamp_min(1), torch.zeros_like(tp))
    f1 = torch.where(prec + rec > 0, 2 * prec * rec / (prec + rec).clamp_min(1e-300), torch.zeros_like(tp))
    w = torch.where(present, label_count / n, torch.zeros_like(label_count))
    return {
        "accuracy": float(tp.sum() / n) if n > 0 else 0.0,
        "weightedPrecision": float((prec * w).sum()),
        "weightedRecall": float((rec * w).sum()),
        "f1": float((f1 * w).sum()),
        "weightedFMeasure": float((f1 * w).sum()),
        "weightedTruePositiveRate": float((rec * w).sum()),
    }


def multiclass_metrics(label, pred, num_classes: int) -> Dict[str, float]:
    return multiclass_from_confusion(confusion_matrix(label, pred, num_classes))


def binary_metrics(score, label) -> Dict[str, float]:
    """areaUnderROC / areaUnderPR for scores vs. (label > 0.5)."""
    if isinstance(score, torch.Tensor) and score.is_cuda:
        auroc, aupr = mops.roc_pr_auc(score, _t(label))
        return {"areaUnderROC": auroc, "areaUnderPR": aupr}
    s = _t(score, torch.float64).reshape(-1)
    y = (_t(label, torch.float64).reshape(-1) > 0.5).to(torch.float64)
    order = torch.argsort(s, descending=True, stable=True)
    s, y = s[order], y[order]
    P = float(y.sum())
    Nn = float(y.numel() - y.sum())
    # group ties: keep the last index of each distinct score
    last = torch.ones_like(s, dtype=torch.bool)
    if s.numel() > 1:
        last[:-1] = s[1:] != s[:-1]
    tp = torch.cumsum(y, 0)[last]
    fp = torch.cumsum(1 - y, 0)[last]
    tpr = tp / P if P > 0 else torch.zeros_like(tp)
    fpr = fp / Nn if Nn > 0 else torch.zeros_like(fp)
    z = torch.zeros(1, dtype=torch.float64, device=tp.device)
    o = torch.ones(1, dtype=torch.float64, device=tp.device)
    roc_x = torch.cat([z, fpr, o])
    roc_y = torch.cat([z, tpr, o])
    auroc = float(torch.trapz(roc_y, roc_x))
    precision = torch.where(tp + fp > 0, tp / (tp + fp).clamp_min(1), torch.ones_like(tp))
    recall = tpr
    pr_x = torch.cat([z, recall])
    pr_y = torch.cat([precision[:1] if precision.numel() else o, precision])
    aupr = float(torch.trapz(pr_y, pr_x))
    return {"areaUnderROC": auroc, "areaUnderPR": aupr}


def regression_metrics(label, pred) -> Dict[str, float]:
    y = _t(label, torch.float64).reshape(-1)
    yh = _t(pred, torch.float64).reshape(-1)
    n, se, ae, sy, syy = mops.regression_moments(y, yh)
    mse = se / n
    var_y = syy / n - (sy / n) ** 2
    ss_tot = var_y * n
    r2 = 1.0 - se / ss_tot if ss_tot > 0 else float("nan")
    return {"rmse": float(np.sqrt(mse)), "mse": float(mse), "r2": float(r2), "mae": float(ae / n),
            "var": float(var_y)}
