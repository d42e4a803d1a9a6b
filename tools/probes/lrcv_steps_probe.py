"""Wall-clock split of the LR CrossValidator fit's host steps (the CrossValidator.fit LR branch,
tuning/crossval.py, replayed step by step with a device sync + timer after each step, and once without
the syncs for the total): where the GPU waits on Python.

    python tools/probes/lrcv_steps_probe.py > out.txt"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from har.config import RunConfig  # noqa: E402
from har.suite import build_estimator, load_wisdm, n_feature_columns, warm_up_device  # noqa: E402
from har.features.hybrid import hybrid_features  # noqa: E402
from har.models.base import labels_tensor, num_label_classes  # noqa: E402
from har.models.logreg import FitSpec  # noqa: E402
from har.ops import rng  # noqa: E402
from har.tuning.crossval import _batched_predictions, _lr_margins  # noqa: E402

dev = torch.device("cuda:0")
root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
cfg = RunConfig(cv_metric="mae")
train, test, _ = load_wisdm(os.path.join(root, "tests", "data", "wisdm_data.csv"), "reference", cfg.seed, device=dev)
nf, nc = n_feature_columns(train), len(train["label"].meta["vocab"])
warm_up_device(dev, train, cfg, ["lrcv"])


def steps(sync):
    marks = []
    cv = build_estimator("lrcv", cfg, dev, nf, nc)
    torch.cuda.synchronize()
    t0 = time.perf_counter()

    def mark(name):
        if sync:
            torch.cuda.synchronize()
        marks.append((name, time.perf_counter()))

    est, maps, ev, k = cv.estimator, cv.estimatorParamMaps, cv.evaluator, cv.numFolds
    n_rows = train.count()
    hm = hybrid_features(train, est.featuresCol, dev)
    y = labels_tensor(train, est.labelCol, dev)
    K = num_label_classes(train, est.labelCol, dev)
    mark("inputs")
    fold_t = rng.device_buckets(cv.seed, rng.STREAM_KFOLD, 0, n_rows, [1.0] * k, dev)
    in_fold = fold_t[None, :] == torch.arange(k, device=dev)[:, None]
    train_w = (~in_fold).float()
    mark("folds")
    specs, index = [], []
    for mi, pm in enumerate(maps):
        sub = est.copy(pm)
        for f in range(k):
            specs.append(FitSpec(train_w[f], sub.regParam, sub.elasticNetParam))
            index.append((mi, f))
    n_cv = len(specs)
    for pm in maps:
        sub = est.copy(pm)
        specs.append(FitSpec(None, sub.regParam, sub.elasticNetParam))
    base = est.copy(maps[0])
    mark("specs")
    models_all, finalize = base.fit_many(hm, y, specs, K, deferred=True)
    mark("fit_many (solve enqueued, models built)")
    models = models_all[:n_cv]
    raw = _lr_margins(models, hm)
    pred = _batched_predictions(models, raw)
    mask = in_fold[torch.arange(len(index), device=dev) % k]
    vals = ev.evaluate_batched(y, pred, mask, K, raw, host=False)
    mark("scoring enqueued")
    finalize()
    mark("finalize (sync + summaries)")
    vals = vals.cpu().numpy()
    metrics = np.zeros((len(maps), k))
    for (mi, f), v in zip(index, vals):
        metrics[mi, f] = v
    avg = metrics.mean(axis=1)
    int(np.argmin(avg))
    mark("selection")
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    return total, [(n, (t - t0) * 1e3) for n, t in marks]


for _ in range(5):
    steps(False)
for sync in (False, True):
    tot, ms = zip(*[steps(sync) for _ in range(6)])
    print(f"sync={sync}: total ms median {np.median(tot) * 1e3:.3f}")
    for i, (name, _) in enumerate(ms[0]):
        print(f"   {name:45s} {np.median([m[i][1] for m in ms]):8.3f} ms (cumulative)")
