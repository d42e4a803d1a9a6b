"""Device reductions behind the DataFrame surface (SURVEY.md K4 column_stats, K3/K5 value counts).

* ``value_counts(codes, V)`` — counts of dictionary codes: Spark's ``countByValue`` inside
  ``StringIndexer.fit`` (``Main/main.py:55-61``) and ``groupBy(col).count()`` (``:35-38``).
  GPU: ``har_value_counts`` (LDS-privatized counters, integer atomics — exact).
* ``describe_device(cols)`` — ``describe()`` (``Main/main.py:43``): count / mean / sample
  stddev / min / max of fp64 columns, two passes (sum, then the sum of squared deviations
  from the mean) with the ``har_column_stats_f64`` plane kernel, fp64 throughout.

Each returns host NumPy (the values are printed); one device -> host copy per call.  With
CPU tensors the same math runs in PyTorch (the test oracle path).
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch

from ..ops import _native


def value_counts(codes: torch.Tensor, V: int) -> np.ndarray:
    codes = codes.to(torch.int64).contiguous()
    if codes.is_cuda:
        out = torch.empty(V, dtype=torch.int64, device=codes.device)
        _native.kernels().value_counts(codes.data_ptr(), codes.numel(), V, out.data_ptr(), _native.stream_ptr())
        return out.cpu().numpy()
    ok = (codes >= 0) & (codes < V)
    return torch.bincount(codes[ok], minlength=V)[:V].numpy().astype(np.int64)


def _stats_planes(X: torch.Tensor, center=None) -> torch.Tensor:
    """[5, C] fp64 (count, sum, sum of (x - center)^2, min, max) of the planes X [C, N] (NaN skipped)."""
    C, N = X.shape
    if X.is_cuda:
        mod = _native.kernels()
        nb = (N + 255) // 256
        ws = torch.empty(max(1, nb * 5 * C), dtype=torch.float64, device=X.device)
        out = torch.empty(5, C, dtype=torch.float64, device=X.device)
        mod.column_stats_f64(X.data_ptr(), N, C, 0 if center is None else center.data_ptr(), out.data_ptr(),
                             ws.data_ptr(), _native.stream_ptr())
        return out
    ok = ~torch.isnan(X)
    x0 = torch.where(ok, X, torch.zeros_like(X))
    d = torch.where(ok, X - (0.0 if center is None else center[:, None]), torch.zeros_like(X))
    return torch.stack([ok.sum(1).double(), x0.sum(1), (d * d).sum(1),
                        torch.where(ok, X, torch.full_like(X, float("inf"))).min(1).values,
                        torch.where(ok, X, torch.full_like(X, -float("inf"))).max(1).values])


def describe_device(cols: List) -> tuple:
    """(count, mean, stddev (sample), min, max) NumPy arrays for DeviceColumns of numeric kind."""
    planes = []
    for c in cols:
        x = c.tensor.double()
        if c.missing_t is not None:
            x = torch.where(c.missing_t, torch.full_like(x, float("nan")), x)
        planes.append(x)
    X = torch.stack(planes).contiguous()                        # [C, N] fp64
    st = _stats_planes(X)
    n = st[0]
    mean = st[1] / n.clamp_min(1)
    m2 = _stats_planes(X, mean.contiguous())[2]                # second pass: centred squares
    std = (m2 / (n - 1).clamp_min(1)).sqrt()
    out = torch.stack([n, mean, std, st[3], st[4]]).cpu().numpy()
    return out[0], out[1], out[2], out[3], out[4]
