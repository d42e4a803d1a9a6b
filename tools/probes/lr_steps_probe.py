"""Host timeline of one LogisticRegression fit (the reference suite's LR: maxIter 20, reg 0.3) on the GPU:
perf_counter marks at the entry / exit of the fit's Python stages (wrappers around them, no syncs), the
fit wall time with the final sync — how long the GPU waits for the host before the solve starts.

    python tools/probes/lr_steps_probe.py > out.txt"""
import functools
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from har.config import RunConfig  # noqa: E402
from har.suite import build_estimator, load_wisdm, n_feature_columns, warm_up_device  # noqa: E402
from har.models import logreg as LR  # noqa: E402
from har.ops import logreg as OLR  # noqa: E402

dev = torch.device("cuda:0")
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
cfg = RunConfig()
train, test, _ = load_wisdm(os.path.join(root, "tests", "data", "wisdm_data.csv"), "reference", cfg.seed, device=dev)
nf, nc = n_feature_columns(train), len(train["label"].meta["vocab"])
warm_up_device(dev, train, cfg, ["lr"])
marks = []


def wrap(obj, name, label):
    f = getattr(obj, name)

    @functools.wraps(f)
    def g(*a, **k):
        marks.append((label + " >", time.perf_counter()))
        r = f(*a, **k)
        marks.append((label + " <", time.perf_counter()))
        return r
    setattr(obj, name, g)


wrap(LR.LogisticRegression, "fit_many", "fit_many")
wrap(LR.LogisticRegression, "_setup", "_setup")
wrap(OLR.LogregDesign, "summary", "summary")
wrap(OLR.DeviceLogregSolver, "reset", "reset")
wrap(OLR.DeviceLogregSolver, "solve", "solve")

res = []
for r in range(30):
    est = build_estimator("lr", cfg, dev, nf, nc)
    torch.cuda.synchronize()
    marks.clear()
    t0 = time.perf_counter()
    est.fit(train)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    if r >= 5:
        res.append(([(n, (t - t0) * 1e6) for n, t in marks], (t1 - t0) * 1e6, (t2 - t0) * 1e6))
print(f"fit wall (with sync) median {np.median([x[2] for x in res]):.1f} us; host returns at {np.median([x[1] for x in res]):.1f} us")
for i, (n, _) in enumerate(res[0][0]):
    print(f"   {n:16s} {np.median([x[0][i][1] for x in res]):8.1f} us")
