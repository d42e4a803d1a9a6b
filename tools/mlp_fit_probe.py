#!/usr/bin/env python3
"""Where the small-batch MLP fit's time goes: the bench's WISDM fit (43-256-256-6,
batch 256, ~15 steps per epoch) timed cold at 1, 2, 3, 4 and 60 epochs, so the differences give the
engine set-up + first (eager) epoch, the epoch-graph capture, one replayed epoch and the steady state;
plus the step kernels alone (graph replay of one step, as tools/mlp_phase_probe.py).

    python tools/mlp_fit_probe.py [--hidden 256] [--data tests/data/wisdm_data.csv]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--data", default=os.path.join(ROOT, "tests", "data", "wisdm_data.csv"))
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from har.models.mlp import MLPEngine, MultilayerPerceptronClassifier
    from har.suite import load_wisdm

    dev = torch.device("cuda")
    train, _, _ = load_wisdm(args.data, "numeric43", 2018, device=dev)
    K = len(train["label"].meta["vocab"])
    F = train["features"].data.shape[1]
    layers = [F, args.hidden, args.hidden, K]

    def fit(epochs):
        est = MultilayerPerceptronClassifier(layers=layers, maxIter=epochs, blockSize=256, stepSize=2e-3,
                                             seed=2018, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        est.fit(train)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    fit(3)  # module loads, allocator warm-up
    res = {}
    for e in (1, 2, 3, 4, 60):
        res[e] = min(fit(e) for _ in range(args.reps))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        MLPEngine(layers, 256, dev, lr=2e-3, seed=2018)
    torch.cuda.synchronize()
    ctor = (time.perf_counter() - t0) / args.reps
    n = train.count()
    spe = max(1, n // 256)
    print(f"WISDM fit {'-'.join(map(str, layers))}, {n} rows, {spe} steps/epoch (min of {args.reps} cold fits, ms)")
    for e, t in res.items():
        print(f"  {e:3d} epochs: {t * 1e3:8.2f}")
    print(f"  engine ctor            {ctor * 1e3:8.2f}")
    print(f"  epoch 0 (eager) + setup  {res[1] * 1e3:8.2f}")
    print(f"  epoch 1 (capture+replay) {(res[2] - res[1]) * 1e3:8.2f}")
    print(f"  epoch 2 (replay)         {(res[3] - res[2]) * 1e3:8.2f}")
    print(f"  steady epoch (3..59)     {(res[60] - res[4]) / 56 * 1e3:8.2f}  = "
          f"{(res[60] - res[4]) / 56 / spe * 1e6:.1f} us/step")


if __name__ == "__main__":
    main()
