#!/usr/bin/env python3
"""Tile sweep of the MFMA GEMM for the shapes of one MLP training step (GPU).

Times every candidate tile for each (layout, epilogue, M, N, K) of the flagship
step, interleaved in rounds in ONE process (guide §5.4 rule 24), and prints the
median microseconds.  Used to pick the tile table in har/models/mlp.py.
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from har.ops.gemm import EPI_BIAS_RELU, EPI_F32_SLAB, EPI_RELU_GRAD, gemm_bf16  # noqa: E402


def main():
    B = int(os.environ.get("BATCH", 65536))
    H = int(os.environ.get("HIDDEN", 256))
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    bf = lambda *s: (torch.randn(*s, device=dev, generator=g) * 0.1).to(torch.bfloat16)  # noqa: E731
    X, h1, h2 = bf(B, 64), bf(B, H), bf(B, H)
    W0, W1, Wo = bf(H, 64), bf(H, H), bf(32, H)
    dl = bf(B, 32)
    out = torch.empty(B, H, dtype=torch.bfloat16, device=dev)
    bias = torch.zeros(H, device=dev)
    S = 64
    ks = B // S
    slab = torch.empty(S * (H * H + H), device=dev)
    rowsum = torch.empty(S * (H * H + H), device=dev)
    cases = {
        "fwd_L1": (lambda t: gemm_bf16(X, W0, out, M=B, N=H, K=64, layout=0, epi=EPI_BIAS_RELU, bias=bias, tile=t),
                   [12, 3]),
        "fwd_L2": (lambda t: gemm_bf16(h1, W1, out, M=B, N=H, K=H, layout=0, epi=EPI_BIAS_RELU, bias=bias, tile=t),
                   [0, 3, 6, 7, 9, 10, 12]),
        "dgrad_L1": (lambda t: gemm_bf16(h2, W1, out, M=B, N=H, K=H, layout=2, epi=EPI_RELU_GRAD, mask=h1, tile=t),
                     [6, 18]),
        "wgrad_W1": (lambda t: gemm_bf16(h2, h1, slab, M=H, N=H, K=B, layout=3, epi=EPI_F32_SLAB, k_split=ks, ldc=H,
                                         slab_stride=H * H + H, rowsum=rowsum, slab_stride_rowsum=H * H + H, tile=t),
                     [9, 18]),
        "wgrad_W1_norowsum": (lambda t: gemm_bf16(h2, h1, slab, M=H, N=H, K=B, layout=3, epi=EPI_F32_SLAB,
                                                  k_split=ks, ldc=H, slab_stride=H * H + H, tile=t), [0, 9]),
        "wgrad_W0": (lambda t: gemm_bf16(h2, X, slab, M=H, N=64, K=B, layout=3, epi=EPI_F32_SLAB, k_split=ks, ldc=64,
                                         slab_stride=H * H + H, rowsum=rowsum, slab_stride_rowsum=H * H + H, tile=t),
                     [8, 20]),
        "wgrad_Wout": (lambda t: gemm_bf16(dl, h2, slab, M=32, N=H, K=B, layout=3, epi=EPI_F32_SLAB, k_split=ks,
                                           ldc=H, slab_stride=H * H + H, rowsum=rowsum, slab_stride_rowsum=H * H + H,
                                           tile=t),
                       [2, 3, 5, 11, 12]),
    }
    res = {k: {t: [] for t in ts} for k, (_, ts) in cases.items()}
    graphs = {}
    for k, (fn, ts) in cases.items():
        for t in ts:
            fn(t)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()  # 20 back-to-back launches: kernel time, not Python launch time
            with torch.cuda.graph(g):
                for _ in range(20):
                    fn(t)
            graphs[(k, t)] = g
    torch.cuda.synchronize()
    for rnd in range(7):
        for k, (fn, ts) in cases.items():
            for t in ts:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                graphs[(k, t)].replay()
                e1.record()
                torch.cuda.synchronize()
                res[k][t].append(e0.elapsed_time(e1) * 50.0)  # us per call
    summary = {k: {t: sorted(v)[len(v) // 2] for t, v in d.items()} for k, d in res.items()}
    for k, d in summary.items():
        best = min(d, key=d.get)
        print(f"{k:12s} " + "  ".join(f"tile{t}={us:7.1f}us" for t, us in d.items()) + f"   best=tile{best}")
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
