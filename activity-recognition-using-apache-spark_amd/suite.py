"""Estimator factory and the reference benchmark suite.

``build_estimator`` turns a classifier name of the CLI (``lr``, ``lrcv``, ``dt``,
``dtcv``, ``rf``, ``rfcv``, ``nb``, ``mlp``) into the estimator the reference
constructs at ``Main/main.py:115`` (LR), ``:202-212`` (LR CrossValidator over the
3x3 regParam x elasticNetParam grid), ``:297`` (DT depth 3), ``:379-395`` (DT CV),
``:478`` (RF 100 trees depth 4) and ``:560-576`` (RF CV).

``run_reference_suite`` times those fits on the WISDM table the way the
reference's ``time()`` brackets do (``Main/main.py:116-119, 214-217, 299-302,
480-483``) — fit wall time over the 70/30 training split — but with the device
synchronized on both sides, and reports, per model, training windows/s next to
the reference's own number for the SAME model (run A:
``result.txt:142,187,232,277``) and the test accuracy next to the reference's
(``result.txt:167,212,257,302``).
"""
from __future__ import annotations

import statistics
import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .config import RunConfig
from .models.base import data_parallel, features_tensor, labels_tensor
from .utils.timing import device_sync

# Reference run A (Main/wisdm_main_ver_0.0/main_result/result.txt): train seconds and accuracy
REFERENCE_RUN_A = {
    "lr": {"train_s": 9.061, "accuracy": 0.614769, "line": "result.txt:142,167"},
    "lrcv": {"train_s": 129.948, "accuracy": 0.714462, "line": "result.txt:187,212"},
    "dt": {"train_s": 12.189, "accuracy": 0.730462, "line": "result.txt:232,257"},
    "rf": {"train_s": 20.472, "accuracy": 0.632, "line": "result.txt:277,302"},
}
REFERENCE_N_TRAIN = 3793  # result.txt:105


def reference_windows_per_s(name: str) -> float:
    """BASELINE.md §3 derived training throughput of the reference for model ``name``."""
    return REFERENCE_N_TRAIN / REFERENCE_RUN_A[name]["train_s"]


def cv_evaluator(metric: str):
    from .evaluation.evaluators import MulticlassClassificationEvaluator, RegressionEvaluator

    if metric in ("mae", "rmse", "mse", "r2"):
        return RegressionEvaluator(labelCol="label", predictionCol="prediction", metricName=metric)
    return MulticlassClassificationEvaluator(labelCol="label", predictionCol="prediction", metricName=metric)


def build_estimator(name: str, cfg: RunConfig, dev, n_features: int, n_classes: int):
    from .models.logreg import LogisticRegression
    from .models.mlp import MultilayerPerceptronClassifier
    from .models.naive_bayes import NaiveBayes
    from .models.tree import DecisionTreeClassifier, RandomForestClassifier
    from .tuning.crossval import CrossValidator, ParamGridBuilder

    if name == "lr":
        return LogisticRegression(maxIter=cfg.lr_max_iter, regParam=cfg.lr_reg, elasticNetParam=cfg.lr_elastic_net,
                                  device=dev)
    if name == "dt":
        return DecisionTreeClassifier(featuresCol="features", labelCol="label", maxDepth=cfg.dt_max_depth,
                                      maxBins=cfg.max_bins, device=dev)
    if name == "rf":
        return RandomForestClassifier(featuresCol="features", labelCol="label", numTrees=cfg.rf_num_trees,
                                      maxDepth=cfg.rf_max_depth, maxBins=cfg.max_bins, seed=cfg.seed, device=dev,
                                      parallelism=cfg.rf_parallel)
    if name == "nb":
        return NaiveBayes(modelType=cfg.nb_model_type, device=dev)
    if name == "mlp":
        return MultilayerPerceptronClassifier(layers=[n_features] + list(cfg.mlp_hidden) + [n_classes],
                                              maxIter=cfg.mlp_epochs, blockSize=cfg.mlp_batch, stepSize=cfg.mlp_lr,
                                              seed=cfg.seed, device=dev)
    if name.endswith("cv"):
        base = build_estimator(name[:-2], cfg, dev, n_features, n_classes)
        grid = ParamGridBuilder()
        if name == "lrcv":
            grid = grid.addGrid("regParam", cfg.cv_reg_grid).addGrid("elasticNetParam", cfg.cv_en_grid)
        return CrossValidator(estimator=base, estimatorParamMaps=grid.build(), evaluator=cv_evaluator(cfg.cv_metric),
                              numFolds=cfg.cv_folds, seed=cfg.seed)
    raise ValueError(f"unknown classifier {name}")


def n_feature_columns(table, col: str = "features") -> int:
    """Width of an assembled feature vector from its metadata (no host copy of a device column)."""
    c = table[col]
    size = (c.meta or {}).get("size")
    return int(size) if size is not None else int(c.data.shape[1])


def warm_up_device(dev, train, cfg: RunConfig, classifiers: Optional[Sequence[str]] = None, test=None):
    """Load the HIP code objects and warm the allocator outside the timed regions — the
    analogue of the reference's SparkContext start-up, which its timers also exclude
    (``Main/main.py:8-9`` vs the ``time()`` brackets at ``:116-124``)."""
    small = train.head(min(256, train.count()))
    n_classes = len(train["label"].meta["vocab"])
    for name in classifiers or cfg.classifiers:
        # the CrossValidators too (on the same 256 rows): their batched solve, fold scoring and
        # evaluator run code (torch reductions, batched metrics) a plain fit never touches
        est = build_estimator(name, cfg, dev, n_feature_columns(small), n_classes)
        inner = getattr(est, "estimator", None) or est
        for attr, v in (("maxIter", 2), ("numTrees", 2)):
            if hasattr(inner, attr):
                setattr(inner, attr, v)
        m = est.fit(small)
        m = getattr(m, "bestModel", m)
        m.predict_all(m.features_input(small))  # the model's own feature layout, as transform() uses
        if test is not None:  # the full-size prediction launch configuration too (main.py times it)
            m.predict_all(m.features_input(test))
    if dev.type == "cuda" and any(c.startswith("lr") for c in (classifiers or cfg.classifiers)):
        # a LogisticRegression fit over the whole table sorts its one-hot CSC keys with a larger
        # radix-sort configuration than the 256-row fits above select (its first launch cost ~15 ms
        # inside the first timed fit): warm that configuration on synthetic keys of the same count
        from .features.hybrid import hybrid_features

        n_keys = train.count() * max(1, int(hybrid_features(small, "features", dev).cat.shape[1]))
        torch.sort(torch.arange(n_keys, 0, -1, device=dev, dtype=torch.int64))
    device_sync(dev)


def load_wisdm(path: str, encoding: str = "reference", seed: int = 2018, split=(0.7, 0.3), device=None):
    """CSV -> feature pipeline -> 70/30 split; returns (train, test, seconds).  On a GPU device the
    table is parsed, encoded and split in HBM (DeviceColumn) by the HIP ETL kernels."""
    from .data.csv_io import read_csv
    from .data.split import random_split
    from .features import wisdm

    t0 = time.perf_counter()
    cuda = device is not None and torch.device(device).type == "cuda"
    raw = read_csv(path, device=device if cuda else None)
    _, _, df = wisdm.prepare(raw, encoding)
    train, test = random_split(df, list(split), seed=seed)
    return train, test, time.perf_counter() - t0


def run_reference_suite(dev, path: str, models: Sequence[str] = ("lr", "lrcv", "dt", "rf"), repeats: int = 3,
                        warmup: int = 1, cv_metric: str = "mae", ctx=None) -> Dict:
    """Time the reference's four fits on WISDM (reference encoding, 70/30, seed 2018).

    Returns per model: median fit seconds over ``repeats`` timed fits (after ``warmup``
    untimed fits of the same model), training windows/s, accuracy on the test split and
    the same numbers of the reference run A with the ratio.  Every fit is also reported in
    order (``fit_s_every`` with ``fit_kind_every``): ``first_fit_s`` is the first, eager fit —
    what ``main.py``, which fits each model once, gets — and ``first_fit_vs_baseline`` its ratio;
    a tree signature fitted again is captured into a HIP graph on its second fit and replayed
    from the third (``models/tree.py`` ``_fit_device``), so the steady-state median of the trees
    is a replay.  The CrossValidator uses
    ``cv_metric`` (``mae``: the evaluator the reference's CV actually minimized,
    ``Main/main.py:175``).  Under ``ctx`` (torch.distributed) every fit is data parallel.
    """
    cfg = RunConfig(cv_metric=cv_metric)
    t_load = time.perf_counter()
    train, test, _ = load_wisdm(path, "reference", cfg.seed, device=dev)
    device_sync(dev)
    load_s = time.perf_counter() - t_load
    n_train = train.count()
    n_features = n_feature_columns(train)
    n_classes = len(train["label"].meta["vocab"])
    X_test = features_tensor(test, "features", dev)
    y_test = labels_tensor(test, "label", dev)
    t_w = time.perf_counter()
    if dev.type == "cuda":
        warm_up_device(dev, train, cfg, list(models))
    warm_s = time.perf_counter() - t_w
    from .models import tree as tree_mod

    out: Dict[str, Dict] = {}
    for name in models:
        times: List[float] = []
        every: List[float] = []
        kinds: List[str] = []
        model = None
        for r in range(warmup + repeats):
            tree_mod.LAST_FIT_KIND = "eager"
            est = build_estimator(name, cfg, dev, n_features, n_classes)
            device_sync(dev)
            t0 = time.perf_counter()
            with data_parallel(ctx):
                model = est.fit(train)
            device_sync(dev)
            dt = time.perf_counter() - t0
            if ctx is not None and ctx.is_distributed:
                from .parallel import dist as hdist
                dt = hdist.max_over_ranks(ctx, dt)
            every.append(dt)
            kinds.append(tree_mod.LAST_FIT_KIND if name in ("dt", "rf", "dtcv", "rfcv") else "eager")
            if r >= warmup:
                times.append(dt)
        best = model.bestModel if hasattr(model, "bestModel") else model
        device_sync(dev)
        t0 = time.perf_counter()
        pred = best.predict(best.features_input(test) if hasattr(best, "features_input") else X_test)
        device_sync(dev)
        pred_s = time.perf_counter() - t0
        acc = float((pred.to(y_test.device) == y_test).float().mean())
        fit_s = statistics.median(times)
        ref = REFERENCE_RUN_A.get(name)
        rec = {"fit_s": fit_s, "fit_s_all": times, "fit_s_every": every, "fit_kind_every": kinds,
               "first_fit_s": every[0], "first_fit_kind": kinds[0], "train_windows_per_s": n_train / fit_s,
               "predict_s": pred_s, "predict_windows_per_s": test.count() / max(pred_s, 1e-12),
               "accuracy": acc}
        if ref is not None:
            rec.update({"ref_fit_s": ref["train_s"], "ref_train_windows_per_s": reference_windows_per_s(name),
                        "vs_baseline": (n_train / fit_s) / reference_windows_per_s(name),
                        "first_fit_vs_baseline": ref["train_s"] / every[0],
                        "ref_accuracy": ref["accuracy"], "accuracy_delta": acc - ref["accuracy"],
                        "ref_source": ref["line"]})
        out[name] = rec
    tot = sum(out[m]["fit_s"] for m in models)
    ref_tot = sum(REFERENCE_RUN_A[m]["train_s"] for m in models if m in REFERENCE_RUN_A)
    summary = {"n_train": n_train, "n_test": test.count(), "n_features": n_features, "load_pipeline_split_s": load_s,
               "device_warmup_s": warm_s, "models": out, "suite_fit_s": tot,
               "suite_first_fit_s": sum(out[m]["first_fit_s"] for m in models),
               "suite_train_windows_per_s": len(models) * n_train / tot}
    if all(m in REFERENCE_RUN_A for m in models):
        summary["ref_suite_fit_s"] = ref_tot
        summary["ref_suite_train_windows_per_s"] = len(models) * REFERENCE_N_TRAIN / ref_tot
        summary["suite_vs_baseline"] = summary["suite_train_windows_per_s"] / summary["ref_suite_train_windows_per_s"]
    from .ops.logreg import solver_cache_clear

    solver_cache_clear()  # the suite's resident tables go out of scope with it
    return summary


def wisdm_mlp_accuracy(dev, path: str, layers_hidden=(256, 256), epochs: int = 60, batch: int = 256,
                       lr: float = 2e-3, seed: int = 2018) -> Dict:
    """Train the bench's MLP architecture (43-h-h-6, bf16 MFMA engine) on the REAL WISDM table
    (numeric-43 encoding, 70/30 split, seed 2018) and report its test accuracy."""
    from .models.mlp import MultilayerPerceptronClassifier

    train, test, _ = load_wisdm(path, "numeric43", seed, device=dev)
    K = len(train["label"].meta["vocab"])
    F = train["features"].data.shape[1]
    est = MultilayerPerceptronClassifier(layers=[F] + list(layers_hidden) + [K], maxIter=epochs, blockSize=batch,
                                         stepSize=lr, seed=seed, device=dev)
    # two fits of the same estimator: the first in the process pays the one-time costs (code-object
    # loads of the step kernels, allocator growth) and is reported as first_fit_s; fit_s is the
    # second, the cost of every later fit (the reference suite's fit_s / first_fit_s convention)
    times = []
    for _ in range(2):
        device_sync(dev)
        t0 = time.perf_counter()
        model = est.fit(train)
        device_sync(dev)
        times.append(time.perf_counter() - t0)
    X_test = features_tensor(test, "features", dev)
    y_test = labels_tensor(test, "label", dev)
    acc = float((model.predict(X_test) == y_test).float().mean())
    return {"accuracy": acc, "fit_s": times[1], "first_fit_s": times[0], "n_train": train.count(), "n_test": test.count(),
            "layers": [F] + list(layers_hidden) + [K], "epochs": epochs, "batch": batch,
            "encoding": "numeric43 (all 43 WISDM features, '?' -> -1)", "split": "70/30 Philox seed 2018"}
