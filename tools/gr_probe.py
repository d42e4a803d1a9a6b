#!/usr/bin/env python3
"""Time mlp.hip grad_reduce_adam alone (GPU) at the bench shape (43-256-256-6, B = 65536):
full step reduction, Adam only, reduce only, and each gradient region on its own, next to
a torch.sum over the same slabs — where do the reduction's microseconds go?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from har.models.mlp import MLPEngine, pad_input_bf16  # noqa: E402
from har.ops import _native  # noqa: E402


def timed(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    dev = torch.device("cuda")
    B = 65536
    eng = MLPEngine([43, 256, 256, 6], B, dev, seed=1)
    g = torch.Generator(device=dev).manual_seed(0)
    X = pad_input_bf16(torch.randn(B, 43, device=dev, generator=g), eng.layout.in_pad)
    y = torch.randint(0, 6, (B,), device=dev, generator=g).to(torch.int32)
    for _ in range(3):
        eng.train_step(X, y, B)
    torch.cuda.synchronize()
    mod = _native.kernels()
    regs = eng._grad_regions()
    b1, b2 = eng.betas

    def call(rs, mode):
        cols = list(zip(*rs)) if rs else [[]] * 5
        mod.grad_reduce_adam(list(cols[2]), list(cols[0]), [e - a for a, e in zip(cols[0], cols[1])], list(cols[4]),
                             list(cols[3]), eng.layout.total, eng.G.data_ptr(), eng.P.data_ptr(), eng.m.data_ptr(),
                             eng.v.data_ptr(), eng.Pb.data_ptr(), 0.0, b1, b2, float(eng.eps), 0.0,
                             eng.step_count.data_ptr(), 0, mode, _native.stream_ptr())

    R, S, A = eng.GR_REDUCE, eng.GR_STORE, eng.GR_ADAM
    print("regions (start, end, S, stride):", [(a, e, s, ld) for a, e, _, s, ld in regs])
    slab_mb = sum((e - a) * s * 4 for a, e, _, s, _ in regs) / 1e6
    print(f"slab bytes read per reduction: {slab_mb:.1f} MB")
    for name, rs, mode in [("reduce+adam (step)", regs, R | A), ("reduce+store", regs, R | S),
                           ("adam only", [], A), ("store only (G -> G)", [], S)] + \
                          [(f"region {i} reduce+store", [rg], R | S) for i, rg in enumerate(regs)]:
        med, mn = timed(lambda: call(rs, mode))
        print(f"{name:28s} median {med:7.1f} us  min {mn:7.1f} us")
    n_bwd = eng.step_S
    w0, b1o = eng.layout.by_name["W0"].offset, eng.layout.by_name["b1"].offset
    sl = eng.slabs[:n_bwd, w0:b1o]
    out = torch.empty(sl.shape[1], device=dev)
    med, mn = timed(lambda: torch.sum(sl, dim=0, out=out))
    print(f"{'torch.sum bwd slabs':28s} median {med:7.1f} us  min {mn:7.1f} us  ({sl.numel() * 4 / 1e6:.1f} MB)")
    big = torch.empty(64 * 1024 * 1024 // 4 * 4, device=dev)
    med, mn = timed(lambda: big.sum())
    print(f"{'torch.sum 256 MB':28s} median {med:7.1f} us  -> {big.numel() * 4 / med / 1e6:.2f} TB/s")


if __name__ == "__main__":
    main()
