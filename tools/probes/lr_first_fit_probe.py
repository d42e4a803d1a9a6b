"""Where the FIRST LogisticRegression fit of a process spends its host time (main.py fits each model once,
after the device warm-up): cProfile over that first fit, then the steady-state fit time for comparison.

    python tools/probes/lr_first_fit_probe.py [lr|lrcv] > out.txt"""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from har.config import RunConfig  # noqa: E402
from har.suite import build_estimator, load_wisdm, n_feature_columns, warm_up_device  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "lr"
dev = torch.device("cuda:0")
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
cfg = RunConfig(cv_metric="mae")
train, test, _ = load_wisdm(os.path.join(root, "tests", "data", "wisdm_data.csv"), "reference", cfg.seed, device=dev)
nf, nc = n_feature_columns(train), len(train["label"].meta["vocab"])
warm_up_device(dev, train, cfg, [name])
est = build_estimator(name, cfg, dev, nf, nc)
torch.cuda.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
est.fit(train)
torch.cuda.synchronize()
pr.disable()
first = time.perf_counter() - t0
ts = []
for _ in range(10):
    e = build_estimator(name, cfg, dev, nf, nc)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.fit(train)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
print(f"{name}: first fit {first * 1e3:.3f} ms (under cProfile), steady {sorted(ts)[5] * 1e3:.3f} ms")
for key in ("cumulative", "tottime"):
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(key).print_stats(30)
    print(f"==== by {key}")
    print(s.getvalue())
