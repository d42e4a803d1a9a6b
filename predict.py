#!/usr/bin/env python3
"""``predict.py`` — batch inference / serving from saved models.

The reference never persists a model and its "Prediction made in" timer measures
only Spark's lazy query-plan construction (``Main/main.py:121-123``),
so it has no inference path to compare against.  This entry point closes that gap:
it loads the ``PipelineModel`` (encoder vocabularies) and any classifier written by
``main.py --save-models DIR`` (saved-model format: SURVEY.md §7.6), encodes raw CSV
rows exactly as at training time, predicts on the device and reports inference
throughput with device-synchronized timers.

    python main.py --preset all-numeric --save-models models/
    python predict.py --models models/ --model rf --data new_windows.csv --out preds.csv
    python predict.py --models models/ --model mlp --data wisdm_data.csv --csv-device --repeat 20

Output CSV columns: ``row, UID (if present), prediction, label_name, probability``.
When the input still has the ``ACTIVITY`` column the script also prints the
reference's evaluation block (accuracy, weighted F1, ...).  Rows whose string
categories were never seen at training time are rejected by the indexers unless
``--handle-invalid keep`` (Spark's ``handleInvalid`` semantics).
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from har.config import DEFAULT_WISDM  # noqa: E402
from har.data.csv_io import read_csv  # noqa: E402
from har.features.encode import StringIndexerModel  # noqa: E402
from har.models.base import features_tensor, resolve_device  # noqa: E402
from har.utils import persist  # noqa: E402
from har.utils.timing import device_sync  # noqa: E402


def encode(pipeline, table, handle_invalid: str = "error"):
    """Apply the fitted pipeline; a label indexer whose input column is absent (unlabeled
    serving data) is skipped."""
    for st in pipeline.stages:
        if isinstance(st, StringIndexerModel):
            if st.inputCol not in table.columns:
                continue
            if handle_invalid != "error":
                st.handleInvalid = handle_invalid
        table = st.transform(table)
    return table


def run(args) -> dict:
    dev = resolve_device(None if args.device == "auto" else args.device)
    pipe = persist.load(os.path.join(args.models, "pipeline"), device=dev)
    model = persist.load(os.path.join(args.models, args.model), device=dev)
    with open(os.path.join(args.models, args.model, "metadata.json")) as f:
        labels = json.load(f).get("labels")
    model = getattr(model, "bestModel", model)
    t0 = time.perf_counter()
    raw = read_csv(args.data, device=dev if (args.csv_device and dev.type == "cuda") else None)
    table = encode(pipe, raw, args.handle_invalid)
    X = features_tensor(table, "features", dev)
    device_sync(dev)
    t_ingest = time.perf_counter() - t0
    out = model.predict_all(X)  # warm-up (code objects, allocator)
    device_sync(dev)
    t1 = time.perf_counter()
    for _ in range(args.repeat):
        out = model.predict_all(X)
    device_sync(dev)
    t_pred = (time.perf_counter() - t1) / max(1, args.repeat)
    raw_pred, prob, pred = out
    n = X.shape[0]
    rec = {"model": str(model), "rows": n, "device": str(dev), "ingest_encode_s": round(t_ingest, 6),
           "predict_s": round(t_pred, 6), "predict_windows_per_s": n / max(t_pred, 1e-12)}
    if "label" in table.columns:
        from har.evaluation.evaluators import evaluate_all

        y = torch.as_tensor(table["label"].data.astype(np.int64), device=dev)
        r = evaluate_all(y, pred, raw_pred, int(raw_pred.shape[1]))
        rec.update({"accuracy": r.accuracy, "f1": r.f1})
    if args.out:
        p = pred.long().cpu().numpy()
        pr = prob.float().cpu().numpy()
        uid = table["UID"].data if "UID" in table.columns else None
        with open(args.out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["row"] + (["UID"] if uid is not None else []) + ["prediction", "label_name", "probability"])
            for i in range(n):
                name = labels[p[i]] if labels and p[i] < len(labels) else ""
                w.writerow([i] + ([int(uid[i])] if uid is not None else []) + [int(p[i]), name, float(pr[i, p[i]])])
    return rec


def main(argv=None):
    ap = argparse.ArgumentParser(description="Batch inference from models saved by main.py --save-models")
    ap.add_argument("--models", required=True, help="directory written by main.py --save-models")
    ap.add_argument("--model", default="rf", help="sub-directory name: lr, lrcv, dt, dtcv, rf, rfcv, nb, mlp")
    ap.add_argument("--data", default=DEFAULT_WISDM)
    ap.add_argument("--out", default="")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--csv-device", action="store_true", help="parse the CSV with the HIP kernels")
    ap.add_argument("--repeat", type=int, default=1, help="timed prediction passes (throughput)")
    ap.add_argument("--handle-invalid", default="error", choices=["error", "skip", "keep"])
    rec = run(ap.parse_args(argv))
    print(json.dumps(rec))
    return rec


if __name__ == "__main__":
    main()
