"""Front-end of the MFMA GEMM kernel family (``csrc/kernels/gemm.hip``).

``layout`` bit 0: A stored M-major ([K][lda]); bit 1: B stored N-major ([K][ldb]).
So ``layout=0`` is ``A[M,K] . B[N,K]^T`` (forward of a Linear layer),
``layout=2`` is ``A[M,K] . B[K,N]`` (data gradient), ``layout=3`` is
``A[K,M]^T . B[K,N]`` (weight gradient).

Split-K products (``EPI_F32_ATOMIC`` / ``EPI_F32_SLAB``) run ``ceil(K/k_split)``
workgroup slices; ``EPI_F32_SLAB`` writes each slice's partial tile into its
own slab (``C + z*slab_stride``) for a deterministic reduction pass.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _native

EPI_F32, EPI_F32_ATOMIC, EPI_BIAS_RELU, EPI_BIAS, EPI_RELU_GRAD, EPI_BIAS_F32, EPI_F32_SLAB = range(7)
TILES = {0: (128, 128, 32), 1: (128, 64, 32), 2: (128, 32, 32), 3: (64, 128, 32), 4: (64, 64, 32), 5: (32, 64, 32),
         6: (128, 256, 32), 7: (64, 256, 32), 8: (64, 64, 128), 9: (128, 128, 64), 10: (128, 256, 64),
         11: (32, 64, 128), 12: (64, 128, 64), 13: (128, 64, 128), 18: (128, 128, 64), 20: (64, 64, 128)}
# (BM, BN, BK); 18 and 20 run 8 waves (4 x 2), the rest <= 2 x 4
_TARGET_BLOCKS = 1024  # >> 256 CUs, bounded split-K traffic


def auto_tile(M: int, N: int) -> int:
    if N <= 32:
        return 2
    if N <= 64:
        return 1
    if M <= 64:
        return 3
    return 0


def tile_counts(M: int, N: int, tile: int = -1):
    bm, bn, _ = TILES[auto_tile(M, N) if tile < 0 else tile]
    return (M + bm - 1) // bm, (N + bn - 1) // bn


def auto_k_split(M: int, N: int, K: int, tile: int = -1) -> int:
    tm, tn = tile_counts(M, N, tile)
    splits = max(1, min((K + 31) // 32, _TARGET_BLOCKS // max(1, tm * tn)))
    bk = TILES[auto_tile(M, N) if tile < 0 else tile][2]
    ks = (K + splits - 1) // splits
    return max(bk, (ks + bk - 1) // bk * bk)


def _check(t: torch.Tensor, name: str):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    if t.stride(-1) != 1:
        raise ValueError(f"{name} must have a contiguous last dimension")
    if t.data_ptr() % 16:
        raise ValueError(f"{name} must be 16-byte aligned")


def _gemm(bf16: bool, A, B, C, M, N, K, layout, epi, bias=None, mask=None, rowsum=None,
          k_split: Optional[int] = None, alpha: float = 1.0, lda=None, ldb=None, ldc=None, tile: int = -1,
          slab_stride: int = 0, slab_stride_rowsum: int = 0):
    for t, n in ((A, "A"), (B, "B"), (C, "C")):
        _check(t, n)
    if epi in (EPI_F32_ATOMIC, EPI_F32_SLAB) and k_split is None:
        k_split = auto_k_split(M, N, K, tile)
    lda = A.stride(0) if lda is None else lda
    ldb = B.stride(0) if ldb is None else ldb
    ldc = C.stride(0) if ldc is None else ldc
    ldm = mask.stride(0) if mask is not None else 0
    # host-side shape contract (mirrors the kernel's): rows addressed must exist
    a_rows = K if layout & 1 else M
    b_rows = K if layout & 2 else N
    if A.shape[0] < a_rows or B.shape[0] < b_rows or (epi != EPI_F32_SLAB and C.shape[0] < M):
        raise ValueError(f"gemm operand too small: A{tuple(A.shape)} B{tuple(B.shape)} C{tuple(C.shape)} "
                         f"for M={M} N={N} K={K} layout={layout}")
    if epi == EPI_F32_SLAB:
        splits = (K + k_split - 1) // k_split
        need = (splits - 1) * slab_stride + (M - 1) * ldc + N
        if C.numel() < need:
            raise ValueError(f"slab buffer too small ({C.numel()} < {need})")
    _native.kernels().gemm(bf16, layout, epi, A.data_ptr(), B.data_ptr(), C.data_ptr(), _native.ptr(bias),
                           _native.ptr(mask), _native.ptr(rowsum), M, N, K, lda, ldb, ldc, ldm,
                           int(k_split or 0), int(tile), int(slab_stride), int(slab_stride_rowsum), float(alpha),
                           _native.stream_ptr())
    return C


def gemm_bf16(A, B, C, M, N, K, layout=0, epi=EPI_F32, **kw):
    return _gemm(True, A, B, C, M, N, K, layout, epi, **kw)


def gemm_f32(A, B, C, M, N, K, layout=0, epi=EPI_F32, **kw):
    return _gemm(False, A, B, C, M, N, K, layout, epi, **kw)
