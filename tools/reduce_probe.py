#!/usr/bin/env python3
"""Time the gradient reduction + Adam kernel of the flagship step over subsets of its gradient
regions (all / the backward's 64 row-slice slabs only / the forward's 256 dWout slabs only), to
see which region bounds it.  python tools/reduce_probe.py [B]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from har.models.mlp import MLPEngine, pad_input_bf16  # noqa: E402
from har.ops import _native  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mlp_phase_probe import timed  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    dev = torch.device("cuda")
    eng = MLPEngine([43, 256, 256, 6], B, dev, seed=1)
    g = torch.Generator(device=dev).manual_seed(0)
    X = pad_input_bf16(torch.randn(B, 43, device=dev, generator=g), eng.layout.in_pad)
    y = torch.randint(0, 6, (B,), device=dev, generator=g).to(torch.int32)
    eng.forward_backward_native(X, y, 1.0 / B)
    regs = eng._grad_regions()
    mod = _native.kernels()
    b1, b2 = eng.betas

    def run(rs, mode):
        cols = list(zip(*rs))
        mod.grad_reduce_adam(list(cols[2]), list(cols[0]), [e - a for a, e in zip(cols[0], cols[1])], list(cols[4]),
                             list(cols[3]), eng.layout.total, eng.G.data_ptr(), eng.P.data_ptr(), eng.m.data_ptr(),
                             eng.v.data_ptr(), eng.Pb.data_ptr(), 0.0, b1, b2, 1e-8, 0.0, eng.step_count.data_ptr(),
                             0, mode, _native.stream_ptr())
    for nm, rs in (("all", regs), ("bwd slabs", regs[:1]), ("fwd dWout slabs", regs[1:])):
        for mode, mn in ((1 | 4, "reduce+adam"), (1 | 2, "reduce+store")):
            print(f"{nm:18s} {mn:14s} {timed(lambda: run(rs, mode)):7.2f} us   regions={[(a, e, n) for a, e, _, n, _ in rs]}")
    for S in (1, 4, 16, 64):  # slab-count sweep of the backward region
        r0 = [(regs[0][0], regs[0][1], regs[0][2], S, regs[0][4])]
        print(f"bwd region S={S:<4d}  reduce+adam    {timed(lambda: run(r0, 5)):7.2f} us")
    for S in (1, 16, 64, 256):
        r1 = [(a, e, p, S, ld) for a, e, p, _, ld in regs[1:]]
        print(f"Wout region S={S:<4d} reduce+adam    {timed(lambda: run(r1, 5)):7.2f} us")
    print(f"{'adam only':18s} {'':14s} {timed(lambda: run([(0, 4, regs[0][2], 1, 4)], 4)):7.2f} us")


if __name__ == "__main__":
    main()
