#!/usr/bin/env python3
"""``main.py`` — the reference entry point (``Main/main.py``), MI355X-native.

Same flow and artefacts as the PySpark script: load the WISDM CSV, print the
schema / sample / class counts / describe, run the feature pipeline, split
70/30 (seed 2018), train and evaluate LogisticRegression, LR+CrossValidator,
DecisionTree(+CV), RandomForest(+CV) — plus NaiveBayes and an MLP — and write
``result.txt``, ``additional_param.csv``, ``crossFold_additional_param.csv``
(identical headers), a ``metrics.jsonl`` record and optional plots / saved models.

    python main.py                                  # the reference run (all six models)
    python main.py --classifiers lr --device cpu     # BASELINE config 1 (plumbing)
    python main.py --preset rf-deep                  # RF 100 trees x depth 10 on the GPU
    python main.py --preset all-numeric --save-models models/
    python main.py --csv-device                      # CSV parsed + dictionary-encoded by the HIP kernels
    python main.py --report                          # + Results table, charts and index.html (report/)
    python main.py --raw raw.csv --hz 20 --window-sec 10 --overlap 0.5   # raw user,activity,timestamp,x,y,z rows
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 main.py   # data parallel over 8 GPUs (RCCL)

Under ``torch.distributed.run`` every rank loads the (small) table and every model is
fit data-parallel on the rank's row shard (``har.models.base.data_parallel``): one
all-reduce per L-BFGS evaluation for LR / LR-CV, owner-computed tree levels
(reduce-scatter + all-gather) for DT / RF (+CV), gradient all-reduce for the MLP,
one moment all-reduce for NaiveBayes.  Rank 0 writes the artefacts.

Paths default to the reference layout relative to the working directory
(``wisdm_main_ver_0.0/main_result``); ``--data`` points at the CSV.
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from har.config import RunConfig, config_from_args  # noqa: E402
from har.data.csv_io import read_csv  # noqa: E402
from har.data.split import random_split  # noqa: E402
from har.data.table import describe_text  # noqa: E402
from har.evaluation.evaluators import evaluate_all  # noqa: E402
from har.features import wisdm  # noqa: E402
from har.models.base import data_parallel, features_tensor, resolve_device  # noqa: E402
from har.parallel import dist as hdist  # noqa: E402
from har.report import csvout  # noqa: E402
from har.report.text import (BANNER_CLASSIFY, BANNER_PIPELINE, BANNER_TRAIN, RunLog, evaluation_block,  # noqa: E402
                             model_header, section)
from har.suite import build_estimator, n_feature_columns, warm_up_device  # noqa: E402
from har.utils import persist  # noqa: E402
from har.utils.timing import PhaseTimer, device_sync  # noqa: E402


def run(cfg: RunConfig, ctx=None) -> dict:
    dev = ctx.device if ctx is not None else resolve_device(None if cfg.device == "auto" else cfg.device)
    main_rank = ctx is None or ctx.is_main
    os.makedirs(cfg.out_dir, exist_ok=True)
    log = RunLog(os.path.join(cfg.out_dir, "result.txt") if main_rank else os.devnull, echo=cfg.echo and main_rank)
    t_run = time.perf_counter()
    timer = PhaseTimer(dev)

    log.print("Loading Data Set...")
    with timer.phase("load_csv"):
        if cfg.raw:  # raw sensor rows -> device windowing + featurization -> the WISDM table
            from har.features.raw import raw_to_table

            raw = raw_to_table(cfg.raw, hz=cfg.hz, window_sec=cfg.window_sec, overlap=cfg.overlap, device=dev,
                               ctx=ctx)
            log.print(f"Raw stream {cfg.raw}: {raw.count()} windows of {int(round(cfg.hz * cfg.window_sec))} "
                      f"samples ({cfg.window_sec:g} s at {cfg.hz:g} Hz, overlap {cfg.overlap:g})")
        else:
            raw = read_csv(cfg.data, device=dev if (cfg.csv_device and dev.type == "cuda") else None)
    with timer.phase("feature_pipeline"):
        data, pipe_model, df = wisdm.prepare(raw, cfg.encoding)
    section(log, "Data Schema")
    log.print(data.print_schema(), end="")
    section(log, "Sample Data")
    log.print(data.show(5), end="")
    section(log, "Activity Count")
    log.print(data.group_count("activity").show(), end="")
    numeric_features = [n for n, t in data.dtypes if t in ("double", "int")]
    section(log, "Summary")
    log.print(describe_text(data.describe(numeric_features)))

    log.print(BANNER_PIPELINE)
    cols = data.columns
    df = df.select(["label", "features"] + cols)
    section(log, "Model Pipeline Schema")
    log.print(df.print_schema(), end="")
    section(log, "Sample Feature Data")
    import pandas as pd

    head = df.head(5)
    log.print(pd.DataFrame({c: [tuple(np.round(v[:9], 2)) if head[c].kind == "vector" else v
                                for v in head[c].data] for c in head.columns}))

    with timer.phase("random_split"):
        train, test = random_split(df, cfg.split, seed=cfg.seed)
    log.print(BANNER_TRAIN)
    log.print("Training Dataset Count : " + str(train.count()))
    log.print("Test Dataset Count     : " + str(test.count()))
    keep = [c for c in test.columns if c not in wisdm.MINIMIZED_VIEW]
    log.print(train.select(keep).show(5), end="")
    log.print(test.select(keep).show(5), end="")
    test_data = test.select([c for c in test.columns if c not in wisdm.SKIPPED_FOR_TEST])
    log.print(test_data.show(5), end="")

    if dev.type == "cuda":
        with timer.phase("device_warmup"):
            warm_up_device(dev, train, cfg, test=test_data)
        # not part of any "trained in" time below (the reference's timers exclude SparkContext start-up too)
        log.print("Device warm-up (HIP code objects, allocator) %.6f seconds" % timer.get("device_warmup"))
    log.print(BANNER_CLASSIFY)
    n_features = n_feature_columns(df)
    vocab = df["label"].meta["vocab"]
    n_classes = len(vocab)
    plain_rows, cv_rows, records = [], [], {}
    X_test = features_tensor(test_data, "features", dev)
    y_test = torch.as_tensor(test_data["label"].data.astype(np.int64), device=dev)
    for name in cfg.classifiers:
        est = build_estimator(name, cfg, dev, n_features, n_classes)
        with timer.phase(f"fit:{name}"), data_parallel(ctx):
            model = est.fit(train)
        train_s = round(timer.get(f"fit:{name}"), 6)  # us resolution: sub-ms fits do not print as 0
        best = model.bestModel if hasattr(model, "bestModel") else model
        # the model's own input layout of the test rows (LR: the cached one-hot index + dense matrix,
        # trees / NB / MLP: the dense device matrix), prepared outside the timer like the table itself
        X_in = best.features_input(test_data) if hasattr(best, "features_input") else X_test
        with timer.phase(f"predict:{name}"):
            raw_pred, prob, pred = best.predict_all(X_in)
        test_s = round(timer.get(f"predict:{name}"), 6)
        label = str(model) + (" for Logistic Regression" if name == "lrcv" else "")
        model_header(log, label, train_s, test_s)
        preds = model.transform(test_data)
        show_class = 5 if name == "lr" else 0
        pv = preds.filter(preds["prediction"].data == show_class).select(
            ["UID", "probability", "label", "prediction"]).order_by("probability", ascending=False)
        log.print(pv.show(n=5, truncate=30), end="")
        with timer.phase(f"evaluate:{name}"):
            r = evaluate_all(y_test, pred, raw_pred, n_classes)
        evaluation_block(log, r)
        row = (csvout.cv_row if name.endswith("cv") else csvout.plain_row)(str(model), r, train_s, test_s)
        (cv_rows if name.endswith("cv") else plain_rows).append(row)
        records[name] = {"model": str(model), "train_s": train_s, "predict_s": test_s,
                         "train_windows_per_s": train.count() / max(train_s, 1e-9),
                         "predict_windows_per_s": test.count() / max(test_s, 1e-9), **r.as_dict()}
        if cfg.save_models and main_rank:
            persist.save(model, os.path.join(cfg.save_models, name), labels=vocab)
    if cfg.save_models and main_rank:
        persist.save(pipe_model, os.path.join(cfg.save_models, "pipeline"), labels=vocab)
    world = ctx.world_size if ctx is not None else 1
    if not main_rank:
        log.close()
        return {"device": str(dev), "world_size": world, "models": records}

    if plain_rows:
        csvout.write_rows(os.path.join(cfg.out_dir, "additional_param.csv"), csvout.PLAIN_FIELDS, plain_rows,
                          append=cfg.append_csv)
    if cv_rows:
        csvout.write_rows(os.path.join(cfg.out_dir, "crossFold_additional_param.csv"), csvout.CV_FIELDS, cv_rows,
                          append=cfg.append_csv)
    summary = {"device": str(dev), "world_size": world, "encoding": cfg.encoding, "n_train": train.count(), "n_test": test.count(),
               "seed": cfg.seed, "wall_s": time.perf_counter() - t_run, "models": records,
               "phases_s": {k: round(v, 6) for k, v in timer.as_dict().items()}}
    csvout.append_jsonl(os.path.join(cfg.out_dir, "metrics.jsonl"), summary)
    log.close()
    if cfg.report:
        from har.report.summary import write_report

        with open(os.path.join(cfg.out_dir, "result.txt")) as fh:
            write_report(summary, os.path.join(cfg.out_dir, "report"), fh.read())
    if cfg.plots:
        from har.report.plots import write_plots

        write_plots(data, numeric_features, cfg.plot_dir, seed=cfg.seed)
    return summary


def main(argv=None):
    cfg = config_from_args(argv)
    ctx = None
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:  # launched by torch.distributed.run: one rank per GPU
        ctx = hdist.init(device=None if cfg.device == "auto" else cfg.device)
    summary = run(cfg, ctx)
    from har.ops.logreg import solver_cache_clear

    solver_cache_clear()  # the run's tables are dropped: release the cached LR solvers' device memory
    if ctx is not None:
        hdist.shutdown(ctx)
        if not ctx.is_main:
            return
    print(json.dumps({k: {kk: (round(vv, 6) if isinstance(vv, float) else vv) for kk, vv in v.items()
                          if kk in ("accuracy", "f1", "train_s", "predict_s")} for k, v in summary["models"].items()}))


if __name__ == "__main__":
    main()
