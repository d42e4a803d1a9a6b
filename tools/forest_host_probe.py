#!/usr/bin/env python3
"""Host enqueue time vs device time of the forest level loop (rf config data, 1 GPU).

usage: python tools/forest_host_probe.py [--trees 100] [--rows 60000] [--depth 10] [--fits 6]
Prints per fit: level loop host enqueue ms, wait for the device ms, whole fit ms.  When the
enqueue time is close to the loop's total the loop is host (launch) bound."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trees", type=int, default=100)
    ap.add_argument("--rows", type=int, default=60000)
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--fits", type=int, default=6)
    ap.add_argument("--dt", action="store_true")
    a = ap.parse_args()
    import torch

    from har.models import tree as tree_mod
    from har.models.tree import DecisionTreeClassifier, RandomForestClassifier
    from har.ops import tree as T

    g = torch.Generator().manual_seed(0)
    mu = torch.randn(6, 43, generator=g) * 1.5
    y = torch.randint(0, 6, (a.rows,), generator=g)
    X = (mu[y] + torch.randn(a.rows, 43, generator=g)).cuda()
    y = y.cuda()
    thr = T.find_thresholds(X[:10000].cpu().numpy(), 32)
    for i in range(a.fits):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        est = (DecisionTreeClassifier(maxDepth=a.depth) if a.dt else
               RandomForestClassifier(numTrees=a.trees, maxDepth=a.depth, seed=7))
        est.fit_tensors(X, y, 6, thresholds=thr)
        t1 = time.perf_counter()
        s, e, d = tree_mod.LAST_LEVEL_TIMES
        print(f"fit {i}: before loop {1e3 * (s - t0):.3f} ms, loop enqueue {1e3 * (e - s):.3f} ms, "
              f"wait {1e3 * (d - e):.3f} ms, fit {1e3 * (t1 - t0):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
