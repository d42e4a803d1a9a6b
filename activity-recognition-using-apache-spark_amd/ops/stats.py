"""Column statistics (K4) and feature binning (K12) — ``csrc/kernels/stats.hip``."""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from . import _native


def column_stats(X: torch.Tensor, w: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[5, F] fp64: weighted count, sum, sum of squares, min, max per column (NaN skipped)."""
    X = X.float()
    if X.is_cuda:
        Xc = X.contiguous()
        n, F = Xc.shape
        mod = _native.kernels()
        ws = torch.empty(max(1, mod.column_stats_workspace(n, F)), dtype=torch.float64, device=X.device)
        out = torch.empty(5, F, dtype=torch.float64, device=X.device)
        wc = None if w is None else w.float().contiguous()
        mod.column_stats(Xc.data_ptr(), n, F, Xc.stride(0), _native.ptr(wc), out.data_ptr(), ws.data_ptr(),
                         _native.stream_ptr())
        return out
    Xd = X.double()
    ok = ~torch.isnan(Xd)
    wd = torch.ones(X.shape[0], dtype=torch.float64) if w is None else w.double()
    wm = (wd[:, None] * ok) * (wd[:, None] != 0)
    x0 = torch.where(ok, Xd, torch.zeros_like(Xd))
    sel = wm > 0
    mn = torch.where(sel, Xd, torch.full_like(Xd, float("inf"))).min(0).values
    mx = torch.where(sel, Xd, torch.full_like(Xd, -float("inf"))).max(0).values
    return torch.stack([wm.sum(0), (wm * x0).sum(0), (wm * x0 * x0).sum(0), mn, mx])


def mean_std(X: torch.Tensor, w: Optional[torch.Tensor] = None, unbiased: bool = False):
    st = column_stats(X, w)
    n, s, q = st[0], st[1], st[2]
    mean = s / n.clamp_min(1e-300)
    var = (q / n.clamp_min(1e-300) - mean * mean).clamp_min(0)
    if unbiased:
        var = var * n / (n - 1).clamp_min(1)
    return mean, var.sqrt()


def bin_features(X: torch.Tensor, thresholds) -> torch.Tensor:
    """uint8 bins [F, N] (feature-major), ``x <= thr[b]`` goes left at split b."""
    from . import tree as T

    if not X.is_cuda:
        return torch.from_numpy(T.bin_features(X.detach().float().cpu().numpy(), thresholds))
    F = X.shape[1]
    tt = T.ThresholdTable.from_any(thresholds)
    maxb = max(1, int(tt.counts.max(initial=0)))
    nthr = torch.from_numpy(tt.counts.astype(np.int32)).to(X.device)
    thr_t = torch.from_numpy(tt.padded(maxb)).to(X.device)
    Xc = X.float().contiguous()
    out = torch.empty(F, Xc.shape[0], dtype=torch.uint8, device=X.device)
    _native.kernels().bin_features(Xc.data_ptr(), Xc.shape[0], F, Xc.stride(0), thr_t.data_ptr(), maxb,
                                   nthr.data_ptr(), out.data_ptr(), _native.stream_ptr())
    return out
