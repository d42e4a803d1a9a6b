"""Hybrid (one-hot index + dense) device layout of an assembled feature vector.

The reference assembles three one-hot blocks (934 + 1401 + 755 columns from the
``*PEAK`` StringIndexer/OneHotEncoder stages) and 10 numeric columns into one
3,100-dim sparse ``features`` vector (``Main/main.py:51-66``, ``result.txt:110``:
``(3100,[0,934,2335,...])``).  Spark keeps it sparse; a dense device copy would
make every logistic-regression evaluation read 3,090 zeros per row.

``HybridMatrix`` keeps, per row, the global column id of the single 1 in each
one-hot block (``-1`` when the row is the dropped last category) plus the dense
columns as a small ``[N, Fd]`` float matrix.  It is derived ON THE DEVICE from
the dense matrix and the assembler's block structure (``VectorAssembler`` column
metadata), so it is valid for any row subset of the table (splits, folds, DP
shards).  A ``CSC`` row list per one-hot column (rows sorted by column) gives the
logistic-regression gradient kernel a fixed summation order (deterministic).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import torch


@dataclass
class HybridMatrix:
    dense: torch.Tensor        # [N, Fd] float32
    dense_cols: torch.Tensor   # [Fd] int32 global column ids
    cat: torch.Tensor          # [N, C] int32 global column id of the row's one-hot entry, -1 = none
    blocks: List[Tuple[int, int]]  # (offset, width) of every one-hot block
    n_features: int

    @property
    def n_rows(self) -> int:
        return int(self.dense.shape[0])

    @property
    def device(self):
        return self.dense.device

    def rows(self, lo: int, hi: int) -> "HybridMatrix":
        """Rows [lo, hi) — memoized per range (the matrix is immutable), so a fit's derived device
        index (the CSC row lists cached on the matrix) is built once per shard, not once per fit."""
        if lo == 0 and hi == self.n_rows:
            return self
        memo = self.__dict__.setdefault("_row_shards", {})
        if (lo, hi) not in memo:
            memo[(lo, hi)] = HybridMatrix(self.dense[lo:hi].contiguous(), self.dense_cols,
                                          self.cat[lo:hi].contiguous(), self.blocks, self.n_features)
        return memo[(lo, hi)]

    def take(self, idx: torch.Tensor) -> "HybridMatrix":
        return HybridMatrix(self.dense[idx].contiguous(), self.dense_cols, self.cat[idx].contiguous(), self.blocks,
                            self.n_features)

    def to_dense(self) -> torch.Tensor:
        X = torch.zeros(self.n_rows, self.n_features, dtype=torch.float32, device=self.device)
        if self.dense.shape[1]:
            X[:, self.dense_cols.long()] = self.dense
        for c in range(self.cat.shape[1]):
            col = self.cat[:, c].long()
            ok = col >= 0
            X[torch.nonzero(ok).squeeze(1), col[ok]] = 1.0
        return X

    def csc(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """(offsets [F+2] int32, rows int32): the rows holding each one-hot column, ascending."""
        N, C = self.cat.shape
        F = self.n_features
        dev = self.device
        rows = torch.arange(N, device=dev, dtype=torch.int64).repeat_interleave(C)
        cols = self.cat.reshape(-1).long()
        ok = cols >= 0
        key = cols[ok] * max(N, 1) + rows[ok]
        key, _ = torch.sort(key)
        csc_rows = (key % max(N, 1)).to(torch.int32).contiguous()
        counts = torch.bincount(key // max(N, 1), minlength=F + 1)[: F + 1]
        off = torch.zeros(F + 2, dtype=torch.int64, device=dev)
        off[1:] = torch.cumsum(counts, 0)
        return off.to(torch.int32).contiguous(), csc_rows

    def col_map(self) -> torch.Tensor:
        """[F+1] int32: dense index j (>= 0), -1 for the intercept slot F, -2 for one-hot columns."""
        F = self.n_features
        m = torch.full((F + 1,), -2, dtype=torch.int32, device=self.device)
        if self.dense_cols.numel():
            m[self.dense_cols.long()] = torch.arange(self.dense_cols.numel(), dtype=torch.int32, device=self.device)
        m[F] = -1
        return m


def onehot_blocks(structure: Optional[Sequence[dict]]) -> List[Tuple[int, int]]:
    return [(int(b["offset"]), int(b["width"])) for b in (structure or []) if b.get("kind") == "onehot"]


def from_dense(X: torch.Tensor, blocks: Sequence[Tuple[int, int]]) -> Optional[HybridMatrix]:
    """Split ``X`` into one-hot indices + dense columns; None if a declared block is not one-hot."""
    N, F = X.shape
    dev = X.device
    in_block = torch.zeros(F, dtype=torch.bool, device=dev)
    cats = []
    for off, w in blocks:
        blk = X[:, off:off + w]
        if w == 0:
            continue
        vmax, arg = blk.max(dim=1)
        rs = blk.sum(dim=1)
        valid = ((blk == 0) | (blk == 1)).all() & ((rs == 0) | (rs == 1)).all()
        if not bool(valid):
            return None
        cats.append(torch.where(vmax > 0, arg + off, torch.full_like(arg, -1)).to(torch.int32))
        in_block[off:off + w] = True
    dense_cols = torch.nonzero(~in_block).squeeze(1).to(torch.int32).contiguous()
    dense = X[:, dense_cols.long()].contiguous()
    cat = torch.stack(cats, 1).contiguous() if cats else torch.zeros(N, 0, dtype=torch.int32, device=dev)
    return HybridMatrix(dense.float(), dense_cols, cat, [tuple(b) for b in blocks], F)


def hybrid_features(table, col: str, device) -> HybridMatrix:
    """Cached device HybridMatrix of a ``vector`` column (one-hot blocks from its assembler
    metadata; a plain dense matrix when the column has none)."""
    from ..data.table import DeviceColumn
    from ..models.base import features_tensor

    c = table[col]
    key = ("hybrid", str(device))
    hit = c.cache.get(key) if c.cache is not None else None
    if hit is not None:
        return hit
    if isinstance(c, DeviceColumn) and c.kind == "vector" and str(c.hybrid.device) == str(torch.device(device)):
        return c.hybrid  # assembled on the device (features.encode.VectorAssembler)
    X = features_tensor(table, col, device)
    hm = from_dense(X, onehot_blocks((c.meta or {}).get("structure")))
    if hm is None:
        hm = from_dense(X, [])
    if c.cache is not None:
        c.cache[key] = hm
    return hm


def tree_hybrid(table, col: str, device) -> Optional[HybridMatrix]:
    """The HybridMatrix of ``col`` when it has one-hot blocks (the device assembler's layout, or its
    assembler metadata), else None — a plain numeric column is not copied into a hybrid form."""
    from ..data.table import DeviceColumn

    c = table[col]
    if c.kind != "vector":
        return None
    if isinstance(c, DeviceColumn):
        hm = c.hybrid
        if str(hm.device) == str(torch.device(device)) and hm.cat.shape[1] > 0:
            return hm
    if not onehot_blocks((c.meta or {}).get("structure")):
        return None
    hm = hybrid_features(table, col, device)
    return hm if hm.cat.shape[1] > 0 else None
