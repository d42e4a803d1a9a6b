"""Sliding-window featurization of raw accelerometer / IMU streams.

The reference ingests WISDM's *pre-computed* window table; the transform that
produced it (10-s windows; per-axis binned distribution, average, time between
peaks, average absolute deviation, standard deviation; average resultant —
Kwapisz et al. 2010, cited by the reference paper) is re-implemented here so
raw streams can be featurized on the GPU, plus the north-star extras (min, max,
energy, axis correlation).  GPU: one HIP kernel (``har_window_features``, one
wave per window, LDS-staged samples, two-pass wave reductions).  CPU: the same
definitions in PyTorch (oracle).

Feature row for A axes (``feature_names``), WISDM-43 first when A = 3:
``[A x 10 bins][avg A][peak A][absdev A][std A][resultant A/3][min A][max A][energy A][corr 3 per triad]``.
"""
from __future__ import annotations

from typing import List, Sequence

import torch

from ..ops import _native

NBINS = 10


def n_features(axes: int) -> int:
    return 17 * axes + 4 * (axes // 3)


def feature_names(axis_names: Sequence[str] = ("X", "Y", "Z")) -> List[str]:
    A = len(axis_names)
    names = [f"{a}{i}" for a in axis_names for i in range(NBINS)]
    for suf in ("AVG", "PEAK", "ABSDEV", "STDDEV"):
        names += [a + suf for a in axis_names]
    names += ["RESULTANT" if A == 3 else f"RESULTANT{g}" for g in range(A // 3)]
    for suf in ("MIN", "MAX", "ENERGY"):
        names += [a + suf for a in axis_names]
    for g in range(A // 3):
        x, y, z = axis_names[3 * g: 3 * g + 3]
        names += [f"CORR_{x}{y}", f"CORR_{x}{z}", f"CORR_{y}{z}"]
    return names


def window_count(n_samples: int, window: int, stride: int) -> int:
    return 0 if n_samples < window else (n_samples - window) // stride + 1


def window_features_torch(stream: torch.Tensor, window: int, stride: int, hz: float) -> torch.Tensor:
    """CPU/oracle implementation (float64 internally)."""
    S, A = stream.shape
    nw = window_count(S, window, stride)
    x = stream.double().unfold(0, window, stride)            # [nw, A, W]
    x = x[:nw]
    mean = x.mean(-1)
    mn, mx = x.min(-1).values, x.max(-1).values
    en = (x * x).mean(-1)
    d = x - mean[..., None]
    absdev = d.abs().mean(-1)
    var = (d * d).mean(-1)
    rng = mx - mn
    b = torch.where(rng[..., None] > 0, ((x - mn[..., None]) / rng.clamp_min(1e-300)[..., None] * NBINS).floor(),
                    torch.zeros_like(x)).clamp(0, NBINS - 1).long()
    bins = torch.nn.functional.one_hot(b, NBINS).double().mean(-2)   # [nw, A, 10]
    thr = mean + 0.5 * (mx - mean)
    mid = x[..., 1:-1]
    pk = (mid > x[..., :-2]) & (mid >= x[..., 2:]) & (mid > thr[..., None])
    t = torch.arange(1, window - 1, dtype=torch.float64, device=x.device)
    npk = pk.sum(-1)
    first = torch.where(pk, t, torch.full_like(mid, float("inf"))).min(-1).values
    last = torch.where(pk, t, torch.full_like(mid, -1.0)).max(-1).values
    peak = torch.where(npk >= 2, (last - first) / (npk - 1).clamp_min(1) * (1000.0 / hz),
                       torch.full_like(first, float("nan")))
    T3 = A // 3
    res, corr = [], []
    for g in range(T3):
        xx, yy, zz = x[:, 3 * g], x[:, 3 * g + 1], x[:, 3 * g + 2]
        res.append(torch.sqrt(xx * xx + yy * yy + zz * zz).mean(-1, keepdim=True))
        sd = var[:, 3 * g: 3 * g + 3].sqrt()
        dd = d[:, 3 * g: 3 * g + 3]
        for i, j in ((0, 1), (0, 2), (1, 2)):
            c = (dd[:, i] * dd[:, j]).mean(-1)
            den = sd[:, i] * sd[:, j]
            corr.append(torch.where(den > 0, c / den.clamp_min(1e-300), torch.zeros_like(c))[:, None])
    out = torch.cat([bins.reshape(nw, -1), mean, peak, absdev, var.sqrt()] + res + [mn, mx, en] + corr, dim=1)
    return out.float()


_WIDE_WARNED = set()
_WIDE_CHUNK_BYTES = 1 << 30  # float64 temporaries per chunk of the wide-window fallback


def _wide_windows(stream: torch.Tensor, window: int, stride: int, hz: float) -> torch.Tensor:
    """Windows the HIP kernel cannot stage (contract code -5: one block's window images — 4 windows of
    ``window x axes`` floats per axis triad — exceed the 160 KB LDS, e.g. 9 axes x 2,600 samples): the
    float64 torch definition on the stream's device, in chunks of ~1 GB of temporaries."""
    S, A = stream.shape
    nw = window_count(S, window, stride)
    key = (A, window)
    if key not in _WIDE_WARNED:
        _WIDE_WARNED.add(key)
        import warnings

        warnings.warn(f"window_features: {A}-axis windows of {window} samples exceed the kernel's LDS images; "
                      f"computed with the torch definition on {stream.device}")
    per = max(1, _WIDE_CHUNK_BYTES // (A * window * 8 * 6))
    outs = [window_features_torch(stream[w0 * stride: (w0 + min(per, nw - w0) - 1) * stride + window],
                                  window, stride, hz) for w0 in range(0, nw, per)]
    return torch.cat(outs) if outs else torch.empty(0, n_features(A), device=stream.device)


def _is_wide(err: RuntimeError) -> bool:
    return "contract violation code -5" in str(err)


def window_features(stream: torch.Tensor, window: int, stride: int, hz: float) -> torch.Tensor:
    """[S, A] raw samples -> [n_windows, n_features(A)] features (GPU kernel on device tensors; windows too
    wide for its LDS images: the torch definition on the device, with a warning)."""
    S, A = stream.shape
    if A % 3 or A > 9:
        raise ValueError("axes must be 3, 6 or 9")
    if not stream.is_cuda:
        return window_features_torch(stream, window, stride, hz)
    nw = window_count(S, window, stride)
    F = n_features(A)
    out = torch.empty(nw, F, dtype=torch.float32, device=stream.device)
    if nw:
        s = stream.contiguous().float()
        try:
            _native.kernels().window_features(s.data_ptr(), S, A, window, stride, nw, float(hz), NBINS,
                                              out.data_ptr(), F, _native.stream_ptr())
        except RuntimeError as e:
            if not _is_wide(e):
                raise
            return _wide_windows(s, window, stride, hz)
    return out


def window_features_mlp(stream: torch.Tensor, window: int, stride: int, hz: float, mean: torch.Tensor,
                        inv_std: torch.Tensor, in_pad: int, nan_value: float = -1.0,
                        out: torch.Tensor = None) -> torch.Tensor:
    """Training input in ONE pass: [S, A] raw samples -> bf16 [n_windows, in_pad] rows of
    ``((isnan(f) ? nan_value : f) - mean) * inv_std`` with zero padding — the window kernel's
    MLP output mode (no fp32 feature matrix, no separate NaN-fill / scale / cast / pad kernels)."""
    S, A = stream.shape
    nw = window_count(S, window, stride)
    F = n_features(A)
    if not stream.is_cuda:
        X = torch.nan_to_num(window_features_torch(stream, window, stride, hz).float(), nan=nan_value)
        Xs = (X - mean.float().cpu()) * inv_std.float().cpu()
        res = torch.zeros(nw, in_pad, dtype=torch.bfloat16)
        res[:, :F] = Xs.to(torch.bfloat16)
        return res
    if out is None:
        out = torch.empty(nw, in_pad, dtype=torch.bfloat16, device=stream.device)
    if nw:
        s = stream.contiguous().float()
        m = mean.float().contiguous()
        r = inv_std.float().contiguous()
        try:
            _native.kernels().window_features_mlp(s.data_ptr(), S, A, window, stride, nw, float(hz), m.data_ptr(),
                                                  r.data_ptr(), float(nan_value), out.data_ptr(), in_pad,
                                                  _native.stream_ptr())
        except RuntimeError as e:
            if not _is_wide(e):
                raise
            X = torch.nan_to_num(_wide_windows(s, window, stride, hz), nan=nan_value)
            out.zero_()
            out[:, :F] = ((X - m) * r).to(torch.bfloat16)
    return out


class WindowFeaturizer:
    """``transform(stream [S, A]) -> features [W, F]`` with the WISDM window defaults
    (10 s at ``hz``; non-overlapping unless ``overlap`` > 0)."""

    def __init__(self, hz: float = 20.0, seconds: float = 10.0, overlap: float = 0.0,
                 axis_names: Sequence[str] = ("X", "Y", "Z")):
        self.hz = hz
        self.window = int(round(hz * seconds))
        self.stride = max(1, int(round(self.window * (1.0 - overlap))))
        self.axis_names = list(axis_names)

    @property
    def names(self) -> List[str]:
        return feature_names(self.axis_names)

    def transform(self, stream: torch.Tensor) -> torch.Tensor:
        return window_features(stream, self.window, self.stride, self.hz)

    def halo(self) -> int:
        """Samples a shard must read past its end so no window straddling the cut is lost (§5.7)."""
        return max(0, self.window - self.stride)
