"""Batched multinomial logistic-regression loss/gradient (kernel K9).

For B models with effective weights ``W [B, K, F]`` and intercepts ``b [B, K]``
over one resident feature matrix ``X [N, F]``:

    Z   = X . W^T + b                  (one GEMM for all B*K columns)
    P   = softmax over each model's K columns
    R   = rw[b, i] / sum_i rw[b, i] * (P - onehot(y))
    loss[b] = sum_i rw[b,i] * CE_i / sum_i rw[b,i]
    dW  = R^T . X ,   db = sum_i R

``rw`` carries the per-model row weights (fold membership in CrossValidator,
Spark's instance weights otherwise), so 45 CV fits share the two GEMMs.

GPU path (gfx950): ``har_gemm_f32`` (exact-fp32 ``v_mfma_f32_16x16x4_f32``,
bias fused in the epilogue) -> ``har_logreg_softmax_grad`` (fused softmax + CE +
residual + per-model loss reduction) -> ``har_gemm_f32`` split-K with fp32
atomics for ``R^T . X``.  CPU path: the same math in PyTorch (test oracle).
"""
from __future__ import annotations

import torch

from . import _native
from .gemm import EPI_BIAS_F32, EPI_F32_ATOMIC, gemm_f32


def _pad8(x: int) -> int:
    return (x + 7) // 8 * 8


def logreg_loss_grad_torch(X, y, W, b, rw, inv_wsum):
    B, K, F = W.shape
    Z = X @ W.reshape(B * K, F).T + b.reshape(1, B * K)           # [N, B*K]
    Z = Z.view(-1, B, K)
    lse = torch.logsumexp(Z, dim=2)                                  # [N, B]
    zy = Z.gather(2, y.view(-1, 1, 1).expand(-1, B, 1)).squeeze(2)   # [N, B]
    wn = rw.T * inv_wsum.view(1, B)                                  # [N, B]
    loss = ((lse - zy) * wn).sum(dim=0)
    P = torch.softmax(Z, dim=2)
    P.scatter_add_(2, y.view(-1, 1, 1).expand(-1, B, 1), -torch.ones_like(P[:, :, :1]))
    R = P * wn.unsqueeze(2)                                          # [N, B, K]
    gW = (R.reshape(-1, B * K).T @ X).view(B, K, F)
    gb = R.sum(dim=0)
    return loss, gW, gb


class LogregWorkspace:
    """Device buffers reused across the ~30-60 objective evaluations of a fit."""

    def __init__(self, X: torch.Tensor, B: int, K: int):
        N, F = X.shape
        self.N, self.F, self.B, self.K = N, F, B, K
        self.cols = _pad8(B * K)
        dev = X.device
        self.Wflat = torch.zeros(self.cols, F, device=dev, dtype=torch.float32)
        self.bflat = torch.zeros(self.cols, device=dev, dtype=torch.float32)
        self.Z = torch.empty(N, self.cols, device=dev, dtype=torch.float32)
        self.R = torch.empty(N, self.cols, device=dev, dtype=torch.float32)
        self.G = torch.empty(self.cols, F, device=dev, dtype=torch.float32)
        self.loss = torch.empty(B, device=dev, dtype=torch.float64)


def logreg_loss_grad_native(X, y32, W, b, rw, inv_wsum, ws: LogregWorkspace):
    B, K, F = W.shape
    N = X.shape[0]
    if F % 4:
        raise ValueError("native logreg path needs F % 4 == 0 (pad the feature matrix)")
    mod = _native.kernels()
    s = _native.stream_ptr()
    ws.Wflat[: B * K].copy_(W.reshape(B * K, F))
    ws.bflat[: B * K].copy_(b.reshape(-1))
    # Z = X . W^T + b        (A = X K-major, B = W K-major)
    gemm_f32(X, ws.Wflat, ws.Z, M=N, N=ws.cols, K=F, layout=0, epi=EPI_BIAS_F32, bias=ws.bflat)
    ws.loss.zero_()
    mod.logreg_softmax_grad(ws.Z.data_ptr(), N, B, K, ws.cols, y32.data_ptr(), rw.data_ptr(),
                            inv_wsum.data_ptr(), ws.R.data_ptr(), ws.loss.data_ptr(), s)
    # G = R^T . X            (A = R M-major [N][cols], B = X N-major [N][F]); split-K over rows
    ws.G.zero_()
    gemm_f32(ws.R, X, ws.G, M=ws.cols, N=F, K=N, layout=3, epi=EPI_F32_ATOMIC,
             k_split=max(32, ((N + 63) // 64 + 31) // 32 * 32))
    gW = ws.G[: B * K].view(B, K, F)
    gb = ws.R[:, : B * K].sum(dim=0).view(B, K)
    return ws.loss.to(torch.float32), gW, gb
