"""Saved-model format (SURVEY.md §7.6 — the reference never saves a model).

Layout, modelled on Spark's ``MLWritable`` directory (``metadata/`` JSON +
``data/``) without Parquet::

    <dir>/metadata.json   {"class", "uid", "version", "timestamp", "params",
                           "numFeatures", "numClasses", "labels", "state": {non-tensor state}}
    <dir>/data.pt         dict of tensors (torch.save; loaded with weights_only=True)
    <dir>/stages/NN_<uid>/ (PipelineModel / CrossValidatorModel children)

Everything needed to rebuild the model is in these two files; loading executes
no code from them (JSON + ``torch.load(weights_only=True)``).
"""
from __future__ import annotations

import json
import os
import time
from typing import Any, Dict

import numpy as np
import torch

FORMAT_VERSION = "har-1"


def _split_state(state: Dict[str, Any]):
    tensors, meta = {}, {}
    for k, v in state.items():
        if isinstance(v, torch.Tensor):
            tensors[k] = v.detach().cpu()
        elif isinstance(v, np.ndarray):
            tensors[k] = torch.from_numpy(np.ascontiguousarray(v))
        else:
            meta[k] = v
    return tensors, meta


def _jsonable(x):
    if isinstance(x, (str, int, float, bool)) or x is None:
        return x
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    if isinstance(x, dict):
        return {str(k): _jsonable(v) for k, v in x.items()}
    if isinstance(x, (np.integer,)):
        return int(x)
    if isinstance(x, (np.floating,)):
        return float(x)
    return str(x)


def save(obj, path: str, labels=None):
    from ..features.encode import PipelineModel
    from ..tuning.crossval import CrossValidatorModel

    os.makedirs(path, exist_ok=True)
    state = obj.state() if hasattr(obj, "state") else {}
    tensors, meta = _split_state(state)
    md = {"class": type(obj).__name__, "uid": getattr(obj, "uid", None), "version": FORMAT_VERSION,
          "timestamp": int(time.time() * 1000),
          "params": _jsonable(obj.params() if hasattr(obj, "params") else {}),
          "numFeatures": getattr(obj, "num_features", None), "numClasses": getattr(obj, "num_classes", None),
          "labels": labels, "state": _jsonable(meta)}
    children = []
    if isinstance(obj, PipelineModel):
        children = obj.stages
    elif isinstance(obj, CrossValidatorModel):
        children = [obj.bestModel]
        md["state"]["avgMetrics"] = list(obj.avgMetrics)
        md["state"]["bestIndex"] = obj.bestIndex
    for i, ch in enumerate(children):
        save(ch, os.path.join(path, "stages", f"{i:02d}_{getattr(ch, 'uid', type(ch).__name__)}"))
    md["children"] = len(children)
    with open(os.path.join(path, "metadata.json"), "w") as f:
        json.dump(md, f, indent=1)
    if tensors:
        torch.save(tensors, os.path.join(path, "data.pt"))


def load(path: str, device=None):
    with open(os.path.join(path, "metadata.json")) as f:
        md = json.load(f)
    dp = os.path.join(path, "data.pt")
    tensors = torch.load(dp, weights_only=True, map_location="cpu") if os.path.exists(dp) else {}
    children = []
    sdir = os.path.join(path, "stages")
    if md.get("children"):
        for name in sorted(os.listdir(sdir)):
            children.append(load(os.path.join(sdir, name), device))
    return _build(md, tensors, children, device)


def _dev(device):
    from ..models.base import resolve_device

    return resolve_device(device)


def _build(md, t, children, device):
    cls, st, uid = md["class"], md["state"], md["uid"]
    p = md.get("params") or {}
    if cls == "LogisticRegressionModel":
        from ..models.logreg import LogisticRegressionModel

        d = _dev(device)
        return LogisticRegressionModel(t["coefficientMatrix"].to(d), t["interceptVector"].to(d), st["binomial"],
                                       uid=uid, device=d)
    if cls in ("DecisionTreeClassificationModel", "RandomForestClassificationModel"):
        from ..models import tree as tr

        d = _dev(device)
        arrs = tr.ForestArrays(t["feature"].to(d), t["threshold"].to(d), t["left"].to(d), t["right"].to(d),
                               t["stats"].to(d), t["n_nodes"].numpy(), int(st["max_depth"]))
        C = tr.DecisionTreeClassificationModel if cls.startswith("Decision") else tr.RandomForestClassificationModel
        return C(arrs, md["numFeatures"], md["numClasses"], uid=uid, device=d)
    if cls == "NaiveBayesModel":
        from ..models.naive_bayes import NaiveBayesModel

        d = _dev(device)
        return NaiveBayesModel(t["pi"].to(d), t["theta"].to(d), t["sigma"].to(d) if "sigma" in t else None,
                               st["modelType"], uid=uid, device=d)
    if cls == "MultilayerPerceptronClassificationModel":
        from ..models.mlp import MLPEngine, MultilayerPerceptronClassificationModel

        d = _dev(device)
        eng = MLPEngine(st["layers"], 4096, d)
        eng.P.copy_(t["params"].to(d))
        if eng.native:
            eng.refresh_bf16()
        m = MultilayerPerceptronClassificationModel(eng, uid=uid)
        m.mean = t.get("mean")
        m.inv_std = t.get("inv_std")
        return m
    if cls == "StringIndexerModel":
        from ..features.encode import StringIndexerModel

        return StringIndexerModel(p["inputCol"], p["outputCol"], st["labels"], p.get("handleInvalid", "error"),
                                  uid=uid)
    if cls == "OneHotEncoderModel":
        from ..features.encode import OneHotEncoderModel

        return OneHotEncoderModel(p["inputCols"], p["outputCols"], st["sizes"], p.get("dropLast", True), uid=uid)
    if cls == "VectorAssembler":
        from ..features.encode import VectorAssembler

        v = VectorAssembler(p["inputCols"], p["outputCol"])
        v.uid = uid
        return v
    if cls == "CastToDouble":
        from ..features.wisdm import CastToDouble

        c = CastToDouble(st.get("inputCols") or p.get("inputCols"), st.get("missing_value", -1.0))
        c.uid = uid
        return c
    if cls == "PipelineModel":
        from ..features.encode import PipelineModel

        return PipelineModel(children, uid=uid)
    if cls in ("CrossValidatorModel", "TrainValidationSplitModel"):
        from ..tuning.crossval import CrossValidatorModel

        return CrossValidatorModel(children[0], st.get("avgMetrics", []), st.get("bestIndex", 0), uid=uid)
    raise ValueError(f"don't know how to load {cls}")
