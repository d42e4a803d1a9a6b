"""Flagship MLP step time with a MALL-resident batch set (8 batches = 67 MB of bf16 rows, bench.py's
shape) vs a cold one (160 batches = 1.3 GB, the 1B-sample pass's situation: every batch read from HBM
once per epoch), each without and with the next batch's rows (1) / rows and labels (2) prefetched by
the reduction launch (``train_step(prefetch=...)``).  Eager steps cycling through the batches, HIP-event timed.

    python tools/probes/mlp_cold_x_probe.py [n_batches ...]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from bench import N_CLASSES, N_FEATURES, synthetic_windows  # noqa: E402
from har.models.mlp import MLPEngine, pad_input_bf16  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B = 65536
    eng = MLPEngine([N_FEATURES, 256, 256, N_CLASSES], B, dev, lr=1e-3, seed=1234)
    for nb in [int(a) for a in sys.argv[1:]] or [8, 160, 8, 160]:
        X, y = synthetic_windows(B * nb, seed=100, device=dev)
        Xin = pad_input_bf16(X, eng.layout.in_pad)
        y32 = y.to(torch.int32).contiguous()
        del X, y

        # none, the next rows, the next rows + labels, their first quarter / eighth (the forward's first
        # two / one tiles per workgroup: later tiles are staged two tiles ahead by the kernel itself)
        for pf in [int(a) for a in os.environ.get("PF_MODES", "0,1,2").split(",")]:
            def step(i):
                j, k = i % nb, (i + 1) % nb
                part = {3: B // 4, 4: B // 8}.get(pf, B)
                nxt = (None, Xin[k * B:(k + 1) * B], (Xin[k * B:(k + 1) * B], y32[k * B:(k + 1) * B]),
                       (Xin[k * B:k * B + part], y32[k * B:k * B + part]),
                       (Xin[k * B:k * B + part], y32[k * B:k * B + part]))[pf]
                eng.train_step(Xin[j * B:(j + 1) * B], y32[j * B:(j + 1) * B], B, prefetch=nxt)

            for i in range(max(40, nb)):
                step(i)
            torch.cuda.synchronize()
            n = 2 * nb if nb > 100 else 200
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(n):
                step(i)
            e1.record()
            torch.cuda.synchronize()
            print(f"batches {nb:4d} ({Xin.numel() * 2 / 1e6:7.1f} MB of rows) prefetch {int(pf)}: "
                  f"{e0.elapsed_time(e1) * 1e3 / n:6.2f} us/step", flush=True)
        del Xin, y32


if __name__ == "__main__":
    main()
