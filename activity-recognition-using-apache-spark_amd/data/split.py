"""Seeded train/test split and k-fold assignment.

``random_split(table, [0.7, 0.3], seed=2018)`` is the equivalent of
``df.randomSplit([0.7, 0.3], seed = 2018)`` (``Main/main.py:80``): every row draws
one Philox uniform keyed by (seed, global row id) and lands in the bucket of
the normalized cumulative weights.  The result is exact-size-random (Bernoulli
per row, like Spark) and identical on 1 or 8 ranks.  Spark's own split is a
function of its partitioning and XORShift state and cannot be reproduced
outside Spark; the test/train sizes are statistically equivalent.

``kfold_ids(n, k, seed)`` is CrossValidator's ``MLUtils.kFold``: each row draws
one uniform and falls into fold ``floor(u * k)``.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from ..ops import rng
from .table import Table


def split_ids(n_rows: int, weights: Sequence[float], seed: int, row_offset: int = 0) -> np.ndarray:
    rows = np.arange(row_offset, row_offset + n_rows, dtype=np.uint64)
    return rng.assign_buckets(seed, rng.STREAM_SPLIT, rows, weights)


def random_split(table: Table, weights: Sequence[float], seed: int = 0) -> List[Table]:
    ids = split_ids(table.count(), weights, seed)
    return [table.take_rows(np.nonzero(ids == b)[0]) for b in range(len(weights))]


def kfold_ids(n_rows: int, k: int, seed: int, row_offset: int = 0) -> np.ndarray:
    rows = np.arange(row_offset, row_offset + n_rows, dtype=np.uint64)
    return rng.assign_buckets(seed, rng.STREAM_KFOLD, rows, [1.0] * k)


def kfold(table: Table, k: int, seed: int = 0):
    """List of (training, validation) tables like ``MLUtils.kFold``."""
    ids = kfold_ids(table.count(), k, seed)
    return [(table.take_rows(np.nonzero(ids != f)[0]), table.take_rows(np.nonzero(ids == f)[0]))
            for f in range(k)]
