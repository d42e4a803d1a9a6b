#!/usr/bin/env python3
"""Host profile of the reference LogisticRegression fit (WISDM, 3100-dim encoding) on the GPU:
wall time per fit, then cProfile of 5 more fits (where the host spends the fit).
With --cold: main.py's order instead (device warm-up, then the FIRST fit of each model profiled).
usage: python tools/lr_probe.py [--model lr|lrcv] [--fits 5] [--cold]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="lr")
    ap.add_argument("--fits", type=int, default=5)
    ap.add_argument("--cold", action="store_true")
    ap.add_argument("--encoding", default="reference", help="reference (3100-dim one-hot) or numeric43 (dense)")
    a = ap.parse_args()
    import torch

    from har.config import DEFAULT_WISDM, RunConfig
    from har.suite import build_estimator, load_wisdm, n_feature_columns, warm_up_device

    dev = torch.device("cuda")
    cfg = RunConfig(cv_metric="mae")
    train, test, _ = load_wisdm(DEFAULT_WISDM, a.encoding, cfg.seed, device=dev)
    nf, nc = n_feature_columns(train), len(train["label"].meta["vocab"])

    def fit(model=a.model):
        est = build_estimator(model, cfg, dev, nf, nc)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        est.fit(train)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    if a.cold:
        warm_up_device(dev, train, cfg)
        for model in ("lr", "lrcv"):
            pr = cProfile.Profile()
            pr.enable()
            t = fit(model)
            pr.disable()
            print(f"first {model} fit: {1e3 * t:.3f} ms", flush=True)
            pstats.Stats(pr).sort_stats("cumtime").print_stats(35)
        return
    for i in range(3):
        print(f"fit {i}: {1e3 * fit():.3f} ms", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    tot = sum(fit() for _ in range(a.fits))
    pr.disable()
    print(f"mean of {a.fits} profiled fits: {1e3 * tot / a.fits:.3f} ms")
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
