"""Host-side profile of the reference suite's LR CrossValidator fit (3x3 grid x 5 folds) on the GPU:
wall time per fit, then cProfile over a few fits (where the Python between kernel launches goes).

    python tools/probes/lrcv_host_probe.py [n_profiled] > out.txt"""
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

dev = torch.device("cuda:0")
path = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests", "data",
                    "wisdm_data.csv")
cfg = RunConfig(cv_metric="mae")
train, test, _ = load_wisdm(path, "reference", cfg.seed, device=dev)
nf, nc = n_feature_columns(train), len(train["label"].meta["vocab"])
warm_up_device(dev, train, cfg, ["lrcv"])


def one():
    est = build_estimator("lrcv", cfg, dev, nf, nc)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    est.fit(train)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


ts = [one() for _ in range(8)]
print("fit ms:", " ".join(f"{t * 1e3:.3f}" for t in ts))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
pr = cProfile.Profile()
pr.enable()
for _ in range(n):
    one()
pr.disable()
for key in ("cumulative", "tottime"):
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(key).print_stats(35)
    print(f"==== by {key} ({n} fits)")
    print(s.getvalue())
