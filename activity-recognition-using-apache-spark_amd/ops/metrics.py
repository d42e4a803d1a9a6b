"""Device reductions for evaluation: confusion matrix and
regression moments in one pass each (``csrc/kernels/metrics.hip``)."""
from __future__ import annotations

import torch

from . import _native


def confusion_matrix(label: torch.Tensor, pred: torch.Tensor, K: int) -> torch.Tensor:
    """``cm[true, pred]`` counts (int64)."""
    if label.is_cuda:
        lab = label.to(torch.int32).contiguous()
        prd = pred.to(device=label.device, dtype=torch.int32).contiguous()
        if int(lab.numel()) and (int(lab.max()) >= K or int(prd.max()) >= K or int(lab.min()) < 0 or int(prd.min()) < 0):
            raise ValueError("confusion_matrix: label/prediction out of range")
        cm = torch.zeros(K * K, dtype=torch.int64, device=label.device)
        _native.kernels().confusion_matrix(lab.data_ptr(), prd.data_ptr(), lab.numel(), K, cm.data_ptr(),
                                           _native.stream_ptr())
        return cm.view(K, K)
    idx = label.to(torch.int64) * K + pred.to(torch.int64)
    return torch.bincount(idx, minlength=K * K).view(K, K)


def roc_pr_auc(score: torch.Tensor, label: torch.Tensor):
    """(areaUnderROC, areaUnderPR) of ``score`` vs ``label > 0.5`` on the device (K19): a
    descending sort (rocPRIM radix sort behind ``torch.sort``), then ONE HIP pass over the sorted
    scores that forms the tie-grouped curve points and sums the trapezoids
    (``csrc/kernels/roc.hip``).  Scores are compared in fp32 (the models' raw predictions)."""
    s = score.reshape(-1).to(torch.float32)
    y = label.reshape(-1).to(device=s.device, dtype=torch.float32)
    vals, order = torch.sort(s, descending=True)
    ys = y[order].contiguous()
    vals = vals.contiguous()
    out = torch.zeros(4, dtype=torch.float64, device=s.device)
    _native.kernels().roc_pr_sums(vals.data_ptr(), ys.data_ptr(), vals.numel(), out.data_ptr(),
                                  _native.stream_ptr())
    roc, pr, P, N = out.cpu().tolist()
    # the curve closes at (1, 1); without negatives its last point is (0, 1) and the closing
    # segment is the whole area (without positives tpr is 0 everywhere)
    return _auc_from_sums(roc, pr, P, N)


def _auc_from_sums(roc, pr, P, N):
    auroc = (roc / (2.0 * P * N) if P > 0 and N > 0 else 0.0) + (0.0 if N > 0 else (1.0 + (P > 0)) / 2.0)
    aupr = pr / (2.0 * P) if P > 0 else 0.0
    return auroc, aupr


def confusion_matrix_batched(label: torch.Tensor, pred: torch.Tensor, mask: torch.Tensor, K: int) -> torch.Tensor:
    """[B, K, K] int64 confusion matrices of B models' predictions ``pred [B, N]`` over the rows
    ``mask [B, N]`` selects (CrossValidator validation folds): one HIP launch (grid row chunks x B)."""
    B, N = pred.shape
    lo_hi = torch.stack([label.min(), label.max()]).tolist() if label.numel() else [0, 0]
    if lo_hi[0] < 0 or lo_hi[1] >= K:  # (the kernel would drop such rows silently)
        raise ValueError(f"labels out of range [0, {K}): min {lo_hi[0]}, max {lo_hi[1]}")
    lab = label.to(device=pred.device, dtype=torch.int32).contiguous()
    prd = pred.to(torch.int32).contiguous()
    msk = mask.to(device=pred.device, dtype=torch.uint8).contiguous()
    cm = torch.empty(B, K, K, dtype=torch.int64, device=pred.device)
    _native.kernels().confusion_matrix_batched(lab.data_ptr(), prd.data_ptr(), msk.data_ptr(), N, B, K, cm.data_ptr(),
                                               _native.stream_ptr())
    return cm


def roc_pr_auc_batched(score: torch.Tensor, label: torch.Tensor, mask: torch.Tensor):
    """(areaUnderROC [B], areaUnderPR [B]) of B models' scores ``score [B, N]`` vs ``label > 0.5`` over
    the rows ``mask [B, N]`` selects: ONE segmented descending sort of all B rows (the unselected rows
    keyed -inf sort to the back), ONE roc.hip launch with a workgroup per model, ONE host read."""
    B, N = score.shape
    # two stable sorts: by score (descending), then selected rows first — an unselected row can never
    # be counted in place of a selected one, not even when a selected score is -inf itself
    m = mask.to(device=score.device, dtype=torch.bool)
    vals, order = torch.sort(score.to(torch.float32), dim=1, descending=True, stable=True)
    _, sel_first = torch.sort((~torch.gather(m, 1, order)).to(torch.uint8), dim=1, stable=True)
    order = torch.gather(order, 1, sel_first)
    vals = torch.gather(vals, 1, sel_first)
    y = label.to(device=score.device, dtype=torch.float32).reshape(1, N).expand(B, N)
    ys = torch.gather(y, 1, order).contiguous()
    ns = mask.to(score.device).sum(1).to(torch.int32).contiguous()
    out = torch.zeros(B, 4, dtype=torch.float64, device=score.device)
    _native.kernels().roc_pr_sums_batched(vals.contiguous().data_ptr(), ys.data_ptr(), ns.data_ptr(), B, N,
                                          out.data_ptr(), _native.stream_ptr())
    o = out.cpu().tolist()
    res = [_auc_from_sums(*r) for r in o]
    return [r[0] for r in res], [r[1] for r in res]


def regression_moments(y: torch.Tensor, yhat: torch.Tensor):
    """(n, sum (y-yh)^2, sum |y-yh|, sum y, sum y^2) — fp64 accumulation."""
    if y.is_cuda:
        out = torch.zeros(6, dtype=torch.float64, device=y.device)
        yf = y.to(torch.float32).contiguous()
        yh = yhat.to(device=y.device, dtype=torch.float32).contiguous()
        _native.kernels().regression_moments(yf.data_ptr(), yh.data_ptr(), yf.numel(), out.data_ptr(),
                                             _native.stream_ptr())
        o = out.cpu().tolist()
        return o[0], o[1], o[2], o[3], o[4]
    d = (y - yhat).double()
    yd = y.double()
    return float(y.numel()), float((d * d).sum()), float(d.abs().sum()), float(yd.sum()), float((yd * yd).sum())
