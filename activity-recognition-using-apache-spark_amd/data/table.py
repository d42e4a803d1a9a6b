"""Columnar table — the DataFrame surface the reference script uses.

Replaces the Spark SQL DataFrame calls of ``Main/main.py:16-100``:
``select`` (``:26,76,88-100``), ``printSchema`` (``:28,75``), ``show`` (``:30,38,89-100``),
``groupBy().count().orderBy()`` (``:35-38``), ``describe()`` (``:43``), ``take`` (``:40,77``),
``count`` (``:84-85``), ``filter`` (``:127``).

Columns are NumPy arrays on the host (``int``/``long``/``double``/``string``) or
2-D ``vector`` columns (dense ``float32`` matrices, one row per table row); the
models move the numeric block to HBM once (``to_tensor``) and keep it resident.
A missing value (``?`` or empty in a numeric column) is NaN in ``double``
columns; the column-level ``missing`` mask is kept alongside.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np

KINDS = ("int", "long", "double", "string", "vector")


def java_double_str(x: float) -> str:
    """Java ``Double.toString`` (what Spark's ``show`` prints for doubles)."""
    if x != x:
        return "NaN"
    if x in (float("inf"), float("-inf")):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "-0.0" if np.copysign(1.0, x) < 0 else "0.0"
    if 1e-3 <= abs(x) < 1e7:
        return np.format_float_positional(float(x), unique=True, trim="0")
    s = np.format_float_scientific(float(x), unique=True, trim="0", exp_digits=1)
    m, e = s.split("e")
    return f"{m}E{int(e)}"


@dataclass
class Column:
    name: str
    kind: str
    data: np.ndarray
    missing: Optional[np.ndarray] = None  # bool mask, numeric columns only
    meta: Optional[dict] = None  # e.g. vocabulary of an indexed column, vector size
    # device copies of this column's data (models.base.features_tensor, features.hybrid): one
    # host->device transfer per column and device, shared by every fit / predict on the column;
    # a row subset (take_rows / filter / split) is a new Column with an empty cache
    cache: Optional[dict] = field(default=None, repr=False, compare=False)

    def __post_init__(self):
        if self.kind not in KINDS:
            raise ValueError(f"unknown column kind {self.kind}")
        if self.cache is None:
            self.cache = {}

    def __len__(self):
        return int(self.data.shape[0])

    def take_rows(self, idx) -> "Column":
        miss = None if self.missing is None else self.missing[idx]
        return Column(self.name, self.kind, self.data[idx], miss, self.meta)

    def spark_type(self) -> str:
        return {"int": "integer", "long": "long", "double": "double",
                "string": "string", "vector": "vector"}[self.kind]

    def cell_str(self, i: int) -> str:
        v = self.data[i]
        if self.missing is not None and self.missing[i]:
            return "null"
        if self.kind in ("int", "long"):
            return str(int(v))
        if self.kind == "double":
            return java_double_str(float(v))
        if self.kind == "string":
            return "null" if v is None else str(v)
        # vector: Spark prints sparse vectors as (size,[idx],[vals]) when sparse is smaller
        vec = np.asarray(v)
        nz = np.nonzero(vec)[0]
        if 2 * len(nz) + 1 < len(vec):
            idx = ",".join(str(int(j)) for j in nz)
            vals = ",".join(java_double_str(float(vec[j])) for j in nz)
            return f"({len(vec)},[{idx}],[{vals}])"
        return "[" + ",".join(java_double_str(float(a)) for a in vec) + "]"


class DeviceColumn(Column):
    """A column resident in device memory (the columnar HIP ETL).

    * numeric (``int``/``long``/``double``): ``tensor`` [N] (fp64 / int64), ``missing_t`` bool [N]
      or None;
    * ``string``: ``tensor`` = dictionary codes int64 [N] (-1 = null) into ``vocab`` (host list of
      the distinct strings), plus ``numeric_t`` (fp64 value of every field that parses as a
      number, NaN otherwise — what ``CastToDouble`` needs);
    * ``vector``: ``hybrid`` (:class:`har.features.hybrid.HybridMatrix`: one-hot indices + dense
      columns), never densified on the device unless a model asks for it.

    ``data`` / ``missing`` materialize the host (NumPy) form lazily — only for printing
    (``show``, ``describe`` output, saved CSVs).  Row subsets (``take_rows``: splits, folds,
    filters) index the device tensors."""

    def __init__(self, name: str, kind: str, tensor=None, missing_t=None, meta: Optional[dict] = None,
                 vocab: Optional[List[str]] = None, numeric_t=None, hybrid=None):
        if kind not in KINDS:
            raise ValueError(f"unknown column kind {kind}")
        self.name, self.kind, self.meta = name, kind, meta
        self.tensor, self.missing_t, self.vocab, self.numeric_t, self.hybrid = tensor, missing_t, vocab, numeric_t, hybrid
        self.cache = {}
        self._host = None
        self._host_missing = False

    @property
    def device(self):
        return self.hybrid.device if self.kind == "vector" else self.tensor.device

    def __len__(self):
        return self.hybrid.n_rows if self.kind == "vector" else int(self.tensor.shape[0])

    @property
    def data(self):
        if self._host is None:
            if self.kind == "vector":
                self._host = self.hybrid.to_dense().cpu().numpy()
            elif self.kind == "string":
                codes = self.tensor.cpu().numpy()
                table = np.asarray(list(self.vocab) + [None], dtype=object)
                self._host = table[np.where(codes < 0, len(self.vocab), codes)]
            else:
                v = self.tensor.cpu().numpy()
                self._host = v.astype(np.int64) if self.kind in ("int", "long") else v.astype(np.float64)
        return self._host

    @property
    def missing(self):
        if self._host_missing is False:
            m = None
            if self.missing_t is not None:
                mh = self.missing_t.cpu().numpy()
                m = mh if mh.any() else None
            self._host_missing = m
        return self._host_missing

    def take_rows(self, idx) -> "DeviceColumn":
        import torch

        it = idx if isinstance(idx, torch.Tensor) else torch.as_tensor(np.asarray(idx, dtype=np.int64))
        it = it.to(self.device)
        if self.kind == "vector":
            return DeviceColumn(self.name, "vector", meta=self.meta, hybrid=self.hybrid.take(it))
        return DeviceColumn(self.name, self.kind, self.tensor[it], None if self.missing_t is None else self.missing_t[it],
                            self.meta, self.vocab, None if self.numeric_t is None else self.numeric_t[it])


class Table:
    """Ordered set of equally long columns."""

    def __init__(self, columns: Iterable[Column] = ()):
        self._cols: "OrderedDict[str, Column]" = OrderedDict()
        n = None
        for c in columns:
            if n is None:
                n = len(c)
            elif len(c) != n:
                raise ValueError(f"column {c.name} has {len(c)} rows, expected {n}")
            self._cols[c.name] = c
        self._n = 0 if n is None else n

    # -- basic accessors -------------------------------------------------
    @property
    def columns(self) -> List[str]:
        return list(self._cols.keys())

    @property
    def dtypes(self):
        return [(c.name, c.spark_type() if c.kind != "int" else "int") for c in self._cols.values()]

    def __getitem__(self, name: str) -> Column:
        key = self._resolve(name)
        return self._cols[key]

    def __contains__(self, name: str) -> bool:
        try:
            self._resolve(name)
            return True
        except KeyError:
            return False

    def _resolve(self, name: str) -> str:
        if name in self._cols:
            return name
        low = name.lower()  # Spark column resolution is case-insensitive by default
        for k in self._cols:
            if k.lower() == low:
                return k
        raise KeyError(name)

    def count(self) -> int:
        return self._n

    __len__ = count

    # -- relational ops ----------------------------------------------------
    def select(self, names: Sequence[str]) -> "Table":
        return Table([self[n] for n in names])

    def drop(self, names: Sequence[str]) -> "Table":
        drop = {n.lower() for n in names}
        return Table([c for c in self._cols.values() if c.name.lower() not in drop])

    def with_column(self, col: Column) -> "Table":
        cols = [c for c in self._cols.values() if c.name != col.name] + [col]
        if self._cols and col.name in self._cols:
            cols = [col if c.name == col.name else c for c in self._cols.values()]
        return Table(cols)

    def take_rows(self, idx) -> "Table":
        return Table([c.take_rows(idx) for c in self._cols.values()])

    def filter(self, mask) -> "Table":
        return self.take_rows(np.nonzero(np.asarray(mask))[0])

    def head(self, n: int) -> "Table":
        return self.take_rows(np.arange(min(n, self._n)))

    def take(self, n: int):
        cols = list(self._cols.values())
        return [tuple(c.data[i] for c in cols) for i in range(min(n, self._n))]

    def order_by(self, name: str, ascending: bool = True) -> "Table":
        c = self[name]
        key = c.data if c.kind != "vector" else None
        if c.kind == "vector":  # Spark orders vectors lexicographically on values
            keys = [tuple(r) for r in c.data]
            order = sorted(range(self._n), key=lambda i: keys[i], reverse=not ascending)
            return self.take_rows(np.asarray(order, dtype=np.int64))
        order = np.argsort(key, kind="stable")
        if not ascending:
            order = np.argsort(-key if c.kind != "string" else key, kind="stable")
            if c.kind == "string":
                order = order[::-1]
        return self.take_rows(order)

    def group_count(self, name: str) -> "Table":
        """``groupBy(name).count().orderBy(col("count").desc())`` (main.py:35-38)."""
        c = self[name]
        if isinstance(c, DeviceColumn) and c.kind == "string":  # value_counts kernel over the codes
            from .device_ops import value_counts

            counts_all = value_counts(c.tensor, len(c.vocab))
            present = np.nonzero(counts_all > 0)[0]
            vals = np.asarray([c.vocab[i] for i in present], dtype=object)
            counts = counts_all[present]
            order = np.lexsort((vals.astype(str), -counts))
            return Table([Column(name.lower() if name != c.name else c.name, "string", vals[order]),
                          Column("count", "long", counts[order].astype(np.int64))])
        vals, counts = np.unique(c.data.astype(str) if c.kind == "string" else c.data, return_counts=True)
        order = np.lexsort((vals, -counts))
        return Table([Column(name.lower() if name != c.name else c.name, c.kind if c.kind != "string" else "string",
                             vals[order].astype(object) if c.kind == "string" else vals[order]),
                      Column("count", "long", counts[order].astype(np.int64))])

    # -- Spark-style text output ------------------------------------------------
    def print_schema(self, out=None) -> str:
        lines = ["root"]
        for c in self._cols.values():
            nullable = "false" if (c.meta or {}).get("nullable") is False else "true"
            lines.append(f" |-- {c.name}: {c.spark_type()} (nullable = {nullable})")
        s = "\n".join(lines) + "\n"
        if out is not None:
            print(s, file=out)
        return s

    def show(self, n: int = 20, truncate=20, out=None) -> str:
        k = min(n, self._n)
        if any(isinstance(c, DeviceColumn) for c in self._cols.values()):  # fetch only the shown rows
            head = self.head(k)
            host = Table([Column(c.name, c.kind, c.data, c.missing, c.meta) for c in head._cols.values()])
            shown = host.show(k, truncate)
            if self._n > k:
                shown += f"only showing top {k} row{'s' if k != 1 else ''}\n"
            if out is not None:
                print(shown, file=out)
            return shown
        cols = list(self._cols.values())
        trunc = 20 if truncate is True else (0 if truncate is False else int(truncate))
        cells = []
        for c in cols:
            col_cells = []
            for i in range(k):
                s = c.cell_str(i)
                if trunc > 0 and len(s) > trunc:
                    s = s[: trunc - 3] + "..." if trunc >= 4 else s[:trunc]
                col_cells.append(s)
            cells.append(col_cells)
        widths = [max(3, len(c.name), *(len(s) for s in cc)) for c, cc in zip(cols, cells)]
        sep = "+" + "+".join("-" * w for w in widths) + "+"
        lines = [sep, "|" + "|".join(c.name.rjust(w) for c, w in zip(cols, widths)) + "|", sep]
        for i in range(k):
            lines.append("|" + "|".join(cc[i].rjust(w) for cc, w in zip(cells, widths)) + "|")
        lines.append(sep)
        if self._n > k:
            lines.append(f"only showing top {k} row{'s' if k != 1 else ''}")
        s = "\n".join(lines) + "\n"
        if out is not None:
            print(s, file=out)
        return s

    def describe(self, names: Optional[Sequence[str]] = None) -> Dict[str, List[str]]:
        """count/mean/stddev(sample)/min/max per numeric column, as strings (Spark ``describe``)."""
        names = names or [c.name for c in self._cols.values() if c.kind in ("int", "long", "double")]
        out: Dict[str, List[str]] = {"summary": ["count", "mean", "stddev", "min", "max"]}
        dev_cols = [self[n] for n in names if isinstance(self[n], DeviceColumn)]
        if dev_cols and len(dev_cols) == len(names):
            from .device_ops import describe_device

            cnt, mean, std, mn, mx = describe_device(dev_cols)
            for j, c in enumerate(dev_cols):
                if c.kind in ("int", "long"):
                    lo, hi = str(int(mn[j])), str(int(mx[j]))
                else:
                    lo, hi = java_double_str(float(mn[j])), java_double_str(float(mx[j]))
                out[c.name] = [str(int(cnt[j])), java_double_str(float(mean[j])),
                               java_double_str(float(std[j])) if cnt[j] > 1 else "NaN", lo, hi]
            return out
        for name in names:
            c = self[name]
            x = c.data.astype(np.float64)
            ok = ~np.isnan(x) if c.missing is None else ~c.missing
            x = x[ok]
            cnt = len(x)
            mean = float(x.mean()) if cnt else float("nan")
            std = float(x.std(ddof=1)) if cnt > 1 else float("nan")
            if c.kind in ("int", "long"):
                mn, mx = str(int(x.min())), str(int(x.max()))
            else:
                mn, mx = java_double_str(float(x.min())), java_double_str(float(x.max()))
            out[c.name] = [str(cnt), java_double_str(mean), java_double_str(std), mn, mx]
        return out

    # -- numeric export ---------------------------------------------------------
    def numeric_matrix(self, names: Sequence[str], dtype=np.float32) -> np.ndarray:
        return np.stack([self[n].data.astype(dtype) for n in names], axis=1) if names else \
            np.zeros((self._n, 0), dtype=dtype)

    def __repr__(self):
        return f"Table({self._n} rows, cols={self.columns})"


def describe_text(desc: Dict[str, List[str]]) -> str:
    """``describe().toPandas().transpose()`` printed by pandas (main.py:43)."""
    import pandas as pd

    df = pd.DataFrame(desc)
    return str(df.transpose())
