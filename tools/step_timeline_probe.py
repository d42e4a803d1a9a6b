#!/usr/bin/env python3
"""Where the fixed cost of a short timed window goes (bench.py's driver command times 20 steps):
the flagship MLP step run as bench.py runs it (eager native plan, 8 resident batch slots), with a HIP
event before every step, timed exactly like bench.py's timed() (sync, host clock, K steps, sync).
Prints the host-clock total, the GPU span first-event -> last-event, and the per-step GPU times."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from bench import synthetic_windows
    from har.models.mlp import MLPEngine, pad_input_bf16

    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda")
    B = 65536
    eng = MLPEngine([43, 256, 256, 6], B, dev, lr=1e-3, seed=1234)
    X, y = synthetic_windows(B * 8, seed=100, device=dev)
    Xin = pad_input_bf16(X, eng.layout.in_pad)
    y32 = y.to(torch.int32).contiguous()

    def step(i):
        j = i % 8
        eng.train_step(Xin[j * B:(j + 1) * B], y32[j * B:(j + 1) * B], B)

    # ~0.3 s of steps first (clock out of idle, as the bench's WISDM run does)
    for i in range(300):
        step(i)
    for rep in range(3):
        for i in range(W):
            step(i)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            ev[i].record()
            step(W + i)
        ev[K].record()
        torch.cuda.synchronize()
        host = time.perf_counter() - t0
        per = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(K)]
        span = ev[0].elapsed_time(ev[K]) * 1e3
        print(f"rep {rep}: host {host * 1e6 / K:.1f} us/step over {K}; GPU span {span / K:.1f} us/step; "
              f"first 5 steps {[round(p, 1) for p in per[:5]]}, median {sorted(per)[K // 2]:.1f}, last {per[-1]:.1f}; "
              f"host - GPU span = {host * 1e6 - span:.0f} us")


if __name__ == "__main__":
    main()
