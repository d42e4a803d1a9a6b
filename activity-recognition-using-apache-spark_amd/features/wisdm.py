"""WISDM v1.1 *transformed* table: column sets and the two feature encodings.

* ``reference`` — exactly the reference pipeline (``Main/main.py:22-77``): drop USER
  and the 30 binned-distribution columns, StringIndexer + OneHotEncoder on the
  ``?``-bearing XPEAK/YPEAK/ZPEAK strings, ACTIVITY -> label, and a VectorAssembler
  of the three one-hot blocks + 10 numeric columns => 3100-dim features with block
  offsets 0 / 934 / 2335 / 3090 (``result.txt:110``).
* ``numeric43`` — all 43 WISDM features as numbers (``?`` -> -1, which keeps the
  "no peak found" signal): X0..Z9, XAVG..ZAVG, XPEAK..ZPEAK, the deviations and
  RESULTANT.  This is the encoding the MLP and the deep forests use.
"""
from __future__ import annotations

from typing import List

import numpy as np

from ..data.table import Column, DeviceColumn, Table
from ..models.base import Transformer, new_uid
from .encode import OneHotEncoder, Pipeline, StringIndexer, VectorAssembler

BIN_COLS = [f"{a}{i}" for a in "XYZ" for i in range(10)]
DROP_LIST = ["USER"] + BIN_COLS
PEAK_COLS = ["XPEAK", "YPEAK", "ZPEAK"]
NUMERIC_COLS = ["XAVG", "YAVG", "ZAVG", "XABSDEV", "YABSDEV", "ZABSDEV", "XSTDDEV", "YSTDDEV", "ZSTDDEV",
                "RESULTANT"]
ALL43 = BIN_COLS + ["XAVG", "YAVG", "ZAVG"] + PEAK_COLS + ["XABSDEV", "YABSDEV", "ZABSDEV", "XSTDDEV", "YSTDDEV",
                                                         "ZSTDDEV", "RESULTANT"]
LABEL_COL = "ACTIVITY"
MINIMIZED_VIEW = ["XPEAK", "YPEAK", "ZPEAK", "XABSDEV", "YABSDEV", "ZABSDEV"]
SKIPPED_FOR_TEST = ["XPEAK", "YPEAK", "ZPEAK", "XAVG", "YAVG", "ZAVG", "XABSDEV", "YABSDEV", "ZABSDEV", "XSTDDEV",
                    "YSTDDEV", "ZSTDDEV", "RESULTANT", "ACTIVITY"]


class CastToDouble(Transformer):
    """String/numeric columns -> double; unparsable values (``?``) -> ``missing_value``."""

    _param_names = ("inputCols", "missing_value")

    def __init__(self, inputCols: List[str], missing_value: float = -1.0):
        super().__init__(new_uid("CastToDouble"))
        self.inputCols, self.missing_value = list(inputCols), missing_value

    def transform(self, table: Table) -> Table:
        t = table
        for c in self.inputCols:
            col = t[c]
            if isinstance(col, DeviceColumn):  # the device CSV's fp64 parse of every field
                import torch

                v = col.numeric_t if col.kind == "string" else col.tensor.double()
                bad = torch.isnan(v) if col.kind == "string" else (
                    col.missing_t if col.missing_t is not None else torch.zeros_like(v, dtype=torch.bool))
                t = t.with_column(DeviceColumn(c, "double", torch.where(bad, torch.full_like(v, self.missing_value), v)))
                continue
            if col.kind == "string":
                vals = np.empty(len(col), dtype=np.float64)
                for i, s in enumerate(col.data):
                    try:
                        vals[i] = float(s)
                    except (TypeError, ValueError):
                        vals[i] = self.missing_value
            else:
                vals = col.data.astype(np.float64)
                if col.missing is not None:
                    vals = np.where(col.missing, self.missing_value, vals)
            t = t.with_column(Column(c, "double", vals))
        return t


def reference_pipeline() -> Pipeline:
    stages = []
    for c in PEAK_COLS:
        stages += [StringIndexer(inputCol=c, outputCol=c + "Index"),
                   OneHotEncoder(inputCols=[c + "Index"], outputCols=[c + "classVec"])]
    stages.append(StringIndexer(inputCol=LABEL_COL, outputCol="label"))
    stages.append(VectorAssembler(inputCols=[c + "classVec" for c in PEAK_COLS] + NUMERIC_COLS,
                                  outputCol="features"))
    return Pipeline(stages)


def numeric43_pipeline() -> Pipeline:
    return Pipeline([CastToDouble(PEAK_COLS, -1.0), StringIndexer(inputCol=LABEL_COL, outputCol="label"),
                     VectorAssembler(inputCols=ALL43, outputCol="features")])


def prepare(table: Table, encoding: str = "reference"):
    """(projected table, fitted pipeline model, transformed table)."""
    if encoding == "reference":
        data = table.drop(DROP_LIST)
        model = reference_pipeline().fit(data)
    elif encoding == "numeric43":
        data = table.drop(["USER"])
        model = numeric43_pipeline().fit(data)
    else:
        raise ValueError(f"unknown encoding {encoding}")
    return data, model, model.transform(data)
