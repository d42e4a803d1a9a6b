#!/usr/bin/env python3
"""Time the fused MLP forward+head kernel alone for several batch sizes (GPU): the
intercept of time vs tiles-per-wave is the prologue (weights -> LDS), the slope the
per-16-row-tile cost."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from har.models.mlp import MLPEngine, pad_input_bf16  # noqa: E402
from har.ops import _native  # noqa: E402


def main():
    dev = torch.device("cuda")
    H = int(os.environ.get("HIDDEN", 256))
    Bmax = 262144
    eng = MLPEngine([43, H, H, 6], Bmax, dev, seed=1)
    g = torch.Generator(device=dev).manual_seed(0)
    X = pad_input_bf16(torch.randn(Bmax, 43, device=dev, generator=g), eng.layout.in_pad)
    y = torch.randint(0, 6, (Bmax,), device=dev, generator=g).to(torch.int32)
    mod, L = _native.kernels(), eng.layout
    sizes = [int(b) for b in os.environ.get("PROBE_B", "1024,4096,16384,32768,65536,131072,262144").split(",")]
    for B in sizes:
        def run():
            mod.mlp_fwd_head(X.data_ptr(), L.in_pad, eng._w(eng.Pb, "W0").data_ptr(), eng._w(eng.P, "b0").data_ptr(),
                             eng._w(eng.Pb, "W1").data_ptr(), eng._w(eng.P, "b1").data_ptr(), H,
                             eng._w(eng.Pb, "Wout").data_ptr(), eng._w(eng.P, "bout").data_ptr(), y.data_ptr(), B,
                             6, 1.0 / B, eng.acts[1].data_ptr(), eng.dbuf[1].data_ptr(), eng.fslab.data_ptr(),
                             eng.fblock_loss.data_ptr(), eng.fblock_correct.data_ptr(), _native.stream_ptr())
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        nwg = mod.mlp_fwd_head_grid(B)
        print(f"B={B:7d} grid={nwg:4d} tiles/wave={B / 16 / (nwg * 4):6.2f}  median {ts[10]:8.1f} us  "
              f"min {ts[0]:8.1f} us  {B / ts[10]:.0f} rows/us")


if __name__ == "__main__":
    main()
