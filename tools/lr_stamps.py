#!/usr/bin/env python3
"""Phase stamps of the LR kernels (logreg_qn.hip STAMP instantiations): one warm fit, then one fit with
the stamp buffers set; prints, for the LAST launch of each kernel, the median / max cycles between its
stamps over the workgroups (s_memtime: shader clock).
usage: python tools/lr_stamps.py [--model lr|lrcv]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = {
    "eval": ["stage dense chunk + margins", "one-hot gathers", "softmax / residual / R", "tile loss sums",
             "pass B (dense gradient)", "intercept sums + slab"],
    "direction": ["P1 / Gram / rho loads", "recursion (thread 0) + barrier", "element sweep (trial points)",
                  "block sums", "P2 stores"],
    "grad": ["col_slice + tile-loss loads", "one-hot slices (row lists)", "dense / intercept slab sums",
             "scale + store"],
    "update": ["P2 reduce", "pick (thread 0)", "element sweep (history)", "block sums + P3 / P1 stores",
               "release fence + counter", "(last chunk) P3 reduce", "(last chunk) finalize"],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="lr")
    a = ap.parse_args()
    import torch

    from har.config import DEFAULT_WISDM, RunConfig
    from har.ops import _native
    from har.suite import build_estimator, load_wisdm, n_feature_columns

    dev = torch.device("cuda")
    cfg = RunConfig(cv_metric="mae")
    train, _, _ = load_wisdm(DEFAULT_WISDM, "reference", cfg.seed, device=dev)
    nf, nc = n_feature_columns(train), len(train["label"].meta["vocab"])
    mod = _native.kernels()
    for _ in range(2):
        build_estimator(a.model, cfg, dev, nf, nc).fit(train)
    torch.cuda.synchronize()
    rows = 1 << 16
    bufs = {k: torch.zeros(rows * 16, dtype=torch.int64, device=dev) for k in PHASES}
    mod.lr_set_stamps(bufs["eval"].data_ptr(), bufs["direction"].data_ptr(), bufs["update"].data_ptr(), bufs["grad"].data_ptr())
    try:
        build_estimator(a.model, cfg, dev, nf, nc).fit(train)
        torch.cuda.synchronize()
    finally:
        mod.lr_set_stamps(0, 0, 0, 0)
    for k, names in PHASES.items():
        st = bufs[k].view(rows, 16).cpu().numpy().astype(np.int64)
        live = st[:, 0] != 0
        st = st[live]
        print(f"--- {k}: {len(st)} workgroups stamped (the last launch of each workgroup slot)")
        tot = []
        for i, nm in enumerate(names):
            ok = (st[:, i + 1] != 0) & (st[:, i] != 0)
            if not ok.any():
                continue
            d = st[ok, i + 1] - st[ok, i]
            print(f"  {nm:40s} median {np.median(d):8.0f}  max {d.max():8.0f} cycles")
        last = max(j for j in range(16) if (st[:, j] != 0).any())
        d = st[:, last] - st[:, 0]
        d = d[st[:, last] != 0]
        print(f"  {'entry -> last stamp':40s} median {np.median(d):8.0f}  max {d.max():8.0f} cycles")


if __name__ == "__main__":
    main()
