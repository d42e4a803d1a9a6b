"""Front-end of the MFMA GEMM kernel family (``csrc/kernels/gemm.hip``).

``layout`` bit 0: A stored M-major ([K][lda]); bit 1: B stored N-major ([K][ldb]).
So ``layout=0`` is ``A[M,K] . B[N,K]^T`` (forward of a Linear layer),
``layout=2`` is ``A[M,K] . B[K,N]`` (data gradient), ``layout=3`` is
``A[K,M]^T . B[K,N]`` (weight gradient).
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _native

EPI_F32, EPI_F32_ATOMIC, EPI_BIAS_RELU, EPI_BIAS, EPI_RELU_GRAD, EPI_BIAS_F32 = range(6)
_TARGET_BLOCKS = 1024  # >> 256 CUs, bounded atomic traffic


def _tile_counts(M: int, N: int):
    if N <= 32:
        bm, bn = 128, 32
    elif N <= 64:
        bm, bn = 128, 64
    elif M <= 64:
        bm, bn = 64, 128
    else:
        bm, bn = 128, 128
    return (M + bm - 1) // bm, (N + bn - 1) // bn


def auto_k_split(M: int, N: int, K: int) -> int:
    tm, tn = _tile_counts(M, N)
    splits = max(1, min((K + 31) // 32, _TARGET_BLOCKS // max(1, tm * tn)))
    ks = (K + splits - 1) // splits
    return max(32, (ks + 31) // 32 * 32)


def _check(t: torch.Tensor, name: str):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    if t.stride(-1) != 1:
        raise ValueError(f"{name} must have a contiguous last dimension")
    if t.data_ptr() % 16:
        raise ValueError(f"{name} must be 16-byte aligned")


def _gemm(bf16: bool, A, B, C, M, N, K, layout, epi, bias=None, mask=None, colsum=None,
          k_split: Optional[int] = None, alpha: float = 1.0, lda=None, ldb=None, ldc=None):
    for t, n in ((A, "A"), (B, "B"), (C, "C")):
        _check(t, n)
    if epi == EPI_F32_ATOMIC and k_split is None:
        k_split = auto_k_split(M, N, K)
    lda = A.stride(0) if lda is None else lda
    ldb = B.stride(0) if ldb is None else ldb
    ldc = C.stride(0) if ldc is None else ldc
    ldm = mask.stride(0) if mask is not None else 0
    # host-side shape contract (mirrors the kernel's): rows addressed must exist
    a_rows = K if layout & 1 else M
    b_rows = K if layout & 2 else N
    if A.shape[0] < a_rows or B.shape[0] < b_rows or C.shape[0] < M:
        raise ValueError(f"gemm operand too small: A{tuple(A.shape)} B{tuple(B.shape)} C{tuple(C.shape)} "
                         f"for M={M} N={N} K={K} layout={layout}")
    _native.kernels().gemm(bf16, layout, epi, A.data_ptr(), B.data_ptr(), C.data_ptr(), _native.ptr(bias),
                           _native.ptr(mask), _native.ptr(colsum), M, N, K, lda, ldb, ldc, ldm,
                           int(k_split or 0), float(alpha), _native.stream_ptr())
    return C


def gemm_bf16(A, B, C, M, N, K, layout=0, epi=EPI_F32, **kw):
    return _gemm(True, A, B, C, M, N, K, layout, epi, **kw)


def gemm_f32(A, B, C, M, N, K, layout=0, epi=EPI_F32, **kw):
    return _gemm(False, A, B, C, M, N, K, layout, epi, **kw)
