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


def batched_metrics(metric: str, label: torch.Tensor, pred: torch.Tensor, mask: torch.Tensor, num_classes: int,
                    raw: torch.Tensor = None, host: bool = True):
    """One metric for B models at once: ``pred`` / ``mask`` are ``[B, N]`` (mask = the rows each
    model is scored on, e.g. its CrossValidator validation fold); returns ``[B]`` with the same
    definitions as the single-model functions above.  On the GPU multiclass metrics come from ONE
    batched confusion-matrix launch (metrics.hip) and binary metrics from ONE segmented sort + ONE
    batched roc.hip launch; regression metrics from masked moments; one host read.  On the CPU the
    same definitions in torch (one-hot einsum, one sort per model for the binary areas).
    ``host=False``: the regression metrics stay a device tensor (no host read here; the caller reads
    it after its own sync) — the other metrics are returned as on the host."""
    B, N = pred.shape
    y = label.to(pred.device).long().view(1, N)
    w = mask.to(torch.float64)
    if metric not in ("areaUnderROC", "areaUnderPR", "rmse", "mse", "r2", "mae", "var") and N:
        lo, hi = torch.stack([y.min(), y.max()]).tolist()
        if lo < 0 or hi >= num_classes:  # as the single-model confusion matrix (one_hot raises there)
            raise ValueError(f"labels out of range [0, {num_classes}): min {lo}, max {hi}")
    if metric in ("areaUnderROC", "areaUnderPR") and pred.is_cuda:
        sc = raw[:, :, 1] if raw.shape[-1] > 1 else raw.reshape(B, N)
        auroc, aupr = mops.roc_pr_auc_batched(sc, label, mask.bool())
        return np.asarray(auroc if metric == "areaUnderROC" else aupr, dtype=np.float64)
    if metric in ("areaUnderROC", "areaUnderPR"):
        out = []
        for b in range(B):
            rows = torch.nonzero(mask[b]).squeeze(1)
            sc = raw[b][rows][:, 1] if raw.shape[-1] > 1 else raw[b][rows].reshape(-1)
            out.append(binary_metrics(sc, label.to(rows.device)[rows])[metric])
        return np.asarray(out, dtype=np.float64)
    if metric in ("rmse", "mse", "r2", "mae", "var"):
        # only the requested metric's terms (each is a few [B, N] launches; the CrossValidator asks one)
        yd = y.double().expand(B, N)
        n = w.sum(1).clamp_min(1e-300)
        def out_(t):
            return t.cpu().numpy() if host else t

        if metric == "mae":
            return out_((w * (pred.double() - yd).abs()).sum(1) / n)

        def var_y():
            my = (w * yd).sum(1) / n
            return (w * yd * yd).sum(1) / n - my * my

        if metric == "var":
            return out_(var_y())
        e = pred.double() - yd
        se = (w * e * e).sum(1)
        if metric == "mse":
            out = se / n
        elif metric == "rmse":
            out = (se / n).sqrt()
        else:  # r2
            ss_tot = var_y() * n
            out = torch.where(ss_tot > 0, 1.0 - se / ss_tot.clamp_min(1e-300), torch.full_like(se, float("nan")))
        return out_(out)
    K = num_classes
    # the batched kernel counts rows (0/1 masks: CrossValidator folds); fractional row weights take
    # the weighted einsum below, as on the CPU
    if pred.is_cuda and K * K <= 4096 and bool(((mask == 0) | (mask == 1)).all()):
        cm = mops.confusion_matrix_batched(y.view(N), pred.long().clamp(0, K - 1), mask.bool(), K).double()
    else:
        Y1 = torch.nn.functional.one_hot(y.view(N), K).double()                  # [N, K]
        P1 = torch.nn.functional.one_hot(pred.long().clamp(0, K - 1), K).double()  # [B, N, K]
        cm = torch.einsum("bn,nk,bnj->bkj", w, Y1, P1)                            # [B, true, pred]
    n = cm.sum((1, 2))
    tp = torch.diagonal(cm, dim1=1, dim2=2)
    lc, pc = cm.sum(2), cm.sum(1)
    prec = torch.where(pc > 0, tp / pc.clamp_min(1), torch.zeros_like(tp))
    rec = torch.where(lc > 0, tp / lc.clamp_min(1), torch.zeros_like(tp))
    f1 = torch.where(prec + rec > 0, 2 * prec * rec / (prec + rec).clamp_min(1e-300), torch.zeros_like(tp))
    wt = torch.where(lc > 0, lc / n.clamp_min(1e-300)[:, None], torch.zeros_like(lc))
    res = {"accuracy": tp.sum(1) / n.clamp_min(1e-300), "weightedPrecision": (prec * wt).sum(1),
           "weightedRecall": (rec * wt).sum(1), "f1": (f1 * wt).sum(1)}
    res["weightedFMeasure"] = res["f1"]
    res["weightedTruePositiveRate"] = res["weightedRecall"]
    return res[metric].cpu().numpy()
