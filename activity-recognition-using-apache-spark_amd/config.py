"""Run configuration: dataclass + CLI + presets.

The reference has no config system — every hyper-parameter is a literal in
``Main/main.py`` (split ``:80``, LR ``:115``, CV grid ``:202-204``, DT ``:297``, RF ``:478``)
and the Spark master is an undefined variable (``:8``).  ``RunConfig`` defaults
reproduce those literals exactly (preset ``reference``); other presets cover the
BASELINE.json configurations.  Presets can also be loaded from YAML
(``--preset-file``, parsed with ``yaml.safe_load``).
"""
from __future__ import annotations

import argparse
import dataclasses
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import os as _os

_REF_WISDM = "/root/reference/Main/wisdm_main_ver_0.0/data/wisdm_data.csv"
_VENDORED_WISDM = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "tests", "data",
                                "wisdm_data.csv")
DEFAULT_WISDM = _REF_WISDM if _os.path.exists(_REF_WISDM) else _VENDORED_WISDM


@dataclass
class RunConfig:
    data: str = DEFAULT_WISDM
    out_dir: str = "wisdm_main_ver_0.0/main_result"
    plot_dir: str = "wisdm_main_ver_0.0/plot"
    encoding: str = "reference"            # reference | numeric43
    classifiers: List[str] = field(default_factory=lambda: ["lr", "lrcv", "dt", "dtcv", "rf", "rfcv"])
    split: List[float] = field(default_factory=lambda: [0.7, 0.3])
    seed: int = 2018
    device: str = "auto"
    # on a GPU: parse + dictionary-encode the CSV with the HIP kernels and keep the table in HBM
    # (the feature pipeline then runs on the device); --no-csv-device keeps the host parser
    csv_device: bool = True
    # raw accelerometer rows (user,activity,timestamp,x,y,z) instead of the pre-windowed table:
    # windowed + featurized on the device into the WISDM columns (features/raw.py)
    raw: Optional[str] = None
    hz: float = 20.0                       # WISDM v1.1 sampling rate (BASELINE.json configs use 50)
    window_sec: float = 10.0               # WISDM window length
    overlap: float = 0.0                   # fraction of a window shared with the next one
    # LogisticRegression (main.py:115)
    lr_max_iter: int = 20
    lr_reg: float = 0.3
    lr_elastic_net: float = 0.0
    # CrossValidator (main.py:202-212)
    cv_folds: int = 5
    cv_reg_grid: List[float] = field(default_factory=lambda: [0.1, 0.3, 0.5])
    cv_en_grid: List[float] = field(default_factory=lambda: [0.0, 0.1, 0.2])
    cv_metric: str = "accuracy"            # reference behaviour: "mae" (RegressionEvaluator leak, main.py:175)
    # DecisionTree (main.py:297) / RandomForest (main.py:478)
    dt_max_depth: int = 3
    rf_num_trees: int = 100
    rf_max_depth: int = 4
    max_bins: int = 32
    # RF over N ranks (torchrun): "tree" = every rank all rows, numTrees / N trees, one all-gather;
    # "data" = row shards + per-level owner reduction; "auto" = tree while the table is small
    rf_parallel: str = "auto"
    # NaiveBayes / MLP (new)
    nb_model_type: str = "gaussian"
    mlp_hidden: List[int] = field(default_factory=lambda: [128, 128])
    mlp_epochs: int = 60
    mlp_batch: int = 256
    mlp_lr: float = 2e-3
    # artefacts
    plots: bool = False
    report: bool = False                   # Results table + charts + index.html (report/summary.py)
    save_models: Optional[str] = None
    append_csv: bool = False
    echo: bool = False


PRESETS: Dict[str, Dict] = {
    "reference": {},
    # BASELINE.json config 1: LR on CPU (plumbing)
    "lr-cpu": {"classifiers": ["lr"], "device": "cpu"},
    # BASELINE.json config 2: RF 100 trees depth 10 on one GPU
    "rf-deep": {"classifiers": ["rf"], "rf_max_depth": 10, "encoding": "numeric43"},
    # BASELINE.json config 3: 3-layer MLP (bf16 on GPU)
    "mlp": {"classifiers": ["mlp"], "encoding": "numeric43"},
    # everything the framework offers on the better encoding
    "all-numeric": {"classifiers": ["lr", "dt", "rf", "nb", "mlp"], "encoding": "numeric43", "rf_max_depth": 10},
}


def _list(t):
    return lambda s: [t(x) for x in s.split(",") if x != ""]


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="MI355X-native WISDM activity recognition (reference: Main/main.py)")
    ap.add_argument("--preset", default="reference", choices=sorted(PRESETS))
    ap.add_argument("--preset-file", default=None, help="YAML file with RunConfig fields")
    d = RunConfig()
    for f in dataclasses.fields(RunConfig):
        name = "--" + f.name.replace("_", "-")
        default = getattr(d, f.name)
        if isinstance(default, bool):
            ap.add_argument(name, dest=f.name, action=argparse.BooleanOptionalAction, default=None)
        elif isinstance(default, list):
            t = float if (default and isinstance(default[0], float)) else (int if default and isinstance(default[0], int) else str)
            ap.add_argument(name, dest=f.name, type=_list(t), default=None)
        else:
            ap.add_argument(name, dest=f.name, type=type(default) if default is not None else str, default=None)
    return ap


def config_from_args(argv=None) -> RunConfig:
    ap = build_parser()
    a = ap.parse_args(argv)
    cfg = RunConfig()
    for k, v in PRESETS[a.preset].items():
        setattr(cfg, k, v)
    if a.preset_file:
        import yaml

        with open(a.preset_file) as fh:
            for k, v in (yaml.safe_load(fh) or {}).items():
                if not hasattr(cfg, k):
                    raise KeyError(f"unknown config key {k}")
                setattr(cfg, k, v)
    for f in dataclasses.fields(RunConfig):
        v = getattr(a, f.name)
        if v is not None:
            setattr(cfg, f.name, v)
    return cfg
