"""Device-resident CSV ingest: the columnar HIP ETL front end.

Replaces Spark's CSV data source with schema inference
(``sqlContext.read.format('com.databricks.spark.csv').options(header='true',
inferschema='true').load(path)``, ``Main/main.py:18-20``) and the
``countByValue`` pass of ``StringIndexer.fit`` (``Main/main.py:55-61``).

Flow (bytes are copied to HBM once, everything else stays on the device):

1. ``csv_count_newlines`` — one workgroup per 4 KiB chunk counts ``'\\n'``;
   an exclusive ``cumsum`` of the chunk counts gives each chunk's offset.
2. ``csv_newline_pos`` — recount + workgroup prefix scan writes the global
   position of every newline.  Line spans (CR stripped, blank lines dropped)
   are built with device tensor ops.
3. ``csv_parse_rows`` — one lane per data row: RFC-4180 field split, field
   class flags (non-empty / int literal / float literal / quoted), fp64 value,
   FNV-1a hash of the raw bytes and the byte span of every field; columnar
   ``[ncols, nrows]`` outputs.
4. Schema inference = device reductions over the flag planes, with the rule of
   the host parser (``har.data.csv_io``): all non-empty fields int literals ->
   ``int`` (``long`` beyond int32), all float literals -> ``double``, else
   ``string``.
5. Dictionary encoding (``dictionary_encode``): ``torch.unique`` over the 64-bit
   hashes with counts -> frequency-descending codes on the device; only one
   representative span per distinct value is decoded on the host (WISDM has
   <= 1,402 distinct strings per column).  Ties in frequency break by ascending
   string value, the rule of ``har.features.encode.StringIndexer``.  Two
   distinct strings colliding in 64-bit FNV-1a are not separated (probability
   ~n^2/2^65 — negligible for any vocabulary this pipeline sees).

``to_table()`` materializes the host :class:`~har.data.table.Table`, identical
to the host parser's (tested in ``tests/test_data.py``).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..ops import _native
from .table import Column, Table

CHUNK = 4096  # bytes per workgroup of csv_count_newlines / csv_newline_pos
INT32_MAX = 2 ** 31 - 1
INT32_MIN = -(2 ** 31)
F_NONEMPTY, F_INT, F_FLOAT, F_QUOTED, F_INEXACT = 1, 2, 4, 8, 16


def _unquote(raw: bytes, quoted: bool) -> str:
    s = raw.decode("utf-8")
    return s.replace('""', '"') if quoted else s


class DeviceCsv:
    """Parsed CSV resident in HBM: per-column kind, fp64 values, hashes, flags, spans."""

    def __init__(self, raw: bytes, buf: torch.Tensor, names: List[str], kinds: List[str], vals: torch.Tensor,
                 hashes: torch.Tensor, flags: torch.Tensor, fstart: torch.Tensor, flen: torch.Tensor):
        self.raw = raw              # host copy of the bytes (string decoding of representatives only)
        self.buf = buf              # uint8 [nbytes] on the device
        self.names = names
        self.kinds = kinds
        self.vals = vals            # fp64 [ncols, nrows]
        self.hashes = hashes        # int64 view of uint64 FNV-1a [ncols, nrows]
        self.flags = flags          # uint8 [ncols, nrows]
        self.fstart = fstart        # int64 [ncols, nrows]
        self.flen = flen            # int32 [ncols, nrows]

    @property
    def nrows(self) -> int:
        return int(self.vals.shape[1])

    @property
    def ncols(self) -> int:
        return len(self.names)

    def col_index(self, name: str) -> int:
        return self.names.index(name)

    def missing(self, j: int) -> torch.Tensor:
        """bool [nrows] device mask: empty numeric field, or unquoted empty string."""
        f = self.flags[j]
        if self.kinds[j] == "string":
            return (f & (F_NONEMPTY | F_QUOTED)) == 0
        return (f & F_FLOAT) == 0

    def numeric(self, names: Optional[List[str]] = None, dtype=torch.float32) -> torch.Tensor:
        """Device matrix [nrows, len(names)] of numeric columns (NaN where missing)."""
        names = names or [n for n, k in zip(self.names, self.kinds) if k != "string"]
        idx = [self.col_index(n) for n in names]
        for n, j in zip(names, idx):
            if self.kinds[j] == "string":
                raise ValueError(f"column {n} is a string column")
        return self.vals[idx].t().to(dtype).contiguous()

    def dictionary_encode(self, name: str) -> Tuple[torch.Tensor, List[str], torch.Tensor]:
        """Frequency-descending dictionary codes of a string column.

        Returns ``(codes int64 [nrows] on the device (-1 for missing), vocabulary,
        counts int64 [len(vocabulary)])``."""
        j = self.col_index(name)
        miss = self.missing(j)
        h = self.hashes[j]
        present = ~miss
        hp = h[present]
        uniq, inv, cnt = torch.unique(hp, return_inverse=True, return_counts=True)
        # one representative row per distinct hash: the first occurrence
        rows = torch.nonzero(present).squeeze(1)
        first = torch.full((uniq.numel(),), rows.numel(), dtype=torch.int64, device=h.device)
        first.scatter_reduce_(0, inv, torch.arange(rows.numel(), device=h.device), reduce="amin")
        rep = rows[first]
        st = self.fstart[j][rep].cpu().numpy()
        ln = self.flen[j][rep].cpu().numpy()
        qt = ((self.flags[j][rep] & F_QUOTED) != 0).cpu().numpy()
        vocab = [_unquote(self.raw[s:s + n], q) for s, n, q in zip(st, ln, qt)]
        counts = cnt.cpu().numpy()
        order = sorted(range(len(vocab)), key=lambda i: (-int(counts[i]), vocab[i]))
        rank = np.empty(len(order), dtype=np.int64)
        rank[np.asarray(order, dtype=np.int64)] = np.arange(len(order))
        rank_t = torch.from_numpy(rank).to(h.device)
        codes = torch.full((self.nrows,), -1, dtype=torch.int64, device=h.device)
        codes[present] = rank_t[inv]
        return codes, [vocab[i] for i in order], torch.from_numpy(counts[np.asarray(order, dtype=np.int64)])

    def to_device_table(self) -> Table:
        """Table of :class:`DeviceColumn` s: numeric planes stay in HBM (fp64 / int64 + missing
        mask), string columns become device dictionary codes + host vocabulary (frequency
        order is decided later by StringIndexer) with their fp64 parse kept for CastToDouble."""
        from .table import DeviceColumn

        cols = []
        for j, (name, kind) in enumerate(zip(self.names, self.kinds)):
            f = self.flags[j]
            if kind in ("int", "long"):
                miss = (f & F_FLOAT) == 0
                v = torch.where(miss, torch.zeros_like(self.vals[j]), self.vals[j]).to(torch.int64)
                cols.append(DeviceColumn(name, kind, v, miss))
            elif kind == "double":
                cols.append(DeviceColumn(name, "double", self.vals[j], (f & F_FLOAT) == 0))
            else:
                codes, vocab = self.dictionary_codes(name)
                num = torch.where((f & F_FLOAT) != 0, self.vals[j], torch.full_like(self.vals[j], float("nan")))
                cols.append(DeviceColumn(name, "string", codes, None, None, vocab, num))
        return Table(cols)

    def dictionary_codes(self, name: str) -> Tuple[torch.Tensor, List[str]]:
        """Device dictionary codes (first-occurrence order, -1 = missing) and the vocabulary:
        ``torch.unique`` over the 64-bit hashes, one representative span per value decoded."""
        j = self.col_index(name)
        miss = self.missing(j)
        h = self.hashes[j]
        present = ~miss
        hp = h[present]
        uniq, inv = torch.unique(hp, return_inverse=True)
        rows = torch.nonzero(present).squeeze(1)
        first = torch.full((uniq.numel(),), rows.numel(), dtype=torch.int64, device=h.device)
        first.scatter_reduce_(0, inv, torch.arange(rows.numel(), device=h.device), reduce="amin")
        rep = rows[first]
        st = self.fstart[j][rep].cpu().numpy()
        ln = self.flen[j][rep].cpu().numpy()
        qt = ((self.flags[j][rep] & F_QUOTED) != 0).cpu().numpy()
        vocab = [_unquote(self.raw[a:a + b], q) for a, b, q in zip(st, ln, qt)]
        codes = torch.full((self.nrows,), -1, dtype=torch.int64, device=h.device)
        codes[present] = inv
        return codes, vocab

    def to_table(self) -> Table:
        cols = []
        flags = self.flags.cpu().numpy()
        vals = self.vals.cpu().numpy()
        for j, (name, kind) in enumerate(zip(self.names, self.kinds)):
            f = flags[j]
            if kind in ("int", "long"):
                miss = (f & F_FLOAT) == 0
                data = np.where(miss, 0, vals[j]).astype(np.int64)
                cols.append(Column(name, kind, data, miss if miss.any() else None))
            elif kind == "double":
                miss = (f & F_FLOAT) == 0
                cols.append(Column(name, "double", vals[j].copy(), miss if miss.any() else None))
            else:
                codes, vocab, _ = self.dictionary_encode(name)
                c = codes.cpu().numpy()
                table = np.asarray(vocab + [None], dtype=object)
                cols.append(Column(name, "string", table[np.where(c < 0, len(vocab), c)]))
        return Table(cols)


def _line_spans(buf: torch.Tensor, start: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Device [b, e) spans of the non-empty lines (CR stripped) of ``buf[start:]``."""
    mod = _native.kernels()
    n = buf.numel()
    dev = buf.device
    blocks = (n + CHUNK - 1) // CHUNK
    counts = torch.zeros(max(1, blocks), dtype=torch.int32, device=dev)
    stream = _native.stream_ptr(dev)
    mod.csv_count_newlines(buf.data_ptr(), n, counts.data_ptr(), stream)
    csum = torch.cumsum(counts.to(torch.int64), 0)
    total = int(csum[-1])  # one host sync: sizes the position buffer
    block_off = (csum - counts.to(torch.int64)).contiguous()
    pos = torch.empty(max(1, total), dtype=torch.int64, device=dev)
    mod.csv_newline_pos(buf.data_ptr(), n, block_off.data_ptr(), pos.data_ptr(), stream)
    pos = pos[:total]
    starts = torch.cat([torch.tensor([start], dtype=torch.int64, device=dev), pos + 1])
    ends = torch.cat([pos, torch.tensor([n], dtype=torch.int64, device=dev)])
    # strip CR and drop blank lines (and the empty tail after a final newline)
    last = torch.clamp(ends - 1, min=0)
    cr = (ends > starts) & (buf[last] == ord("\r"))
    ends = ends - cr.to(torch.int64)
    keep = ends > starts
    return starts[keep].contiguous(), ends[keep].contiguous()


def _split_header(line: bytes) -> List[str]:
    import csv
    import io

    row = next(csv.reader(io.StringIO(line.decode("utf-8"))))
    return [c.strip() for c in row]


def read_csv_device(path: str, device="cuda", header: bool = True) -> DeviceCsv:
    """Parse a CSV file on the GPU.  ``to_table()`` gives the host Table."""
    with open(path, "rb") as f:
        raw = f.read()
    return parse_csv_device(raw, device=device, header=header)


def parse_csv_device(raw: bytes, device="cuda", header: bool = True) -> DeviceCsv:
    dev = torch.device(device)
    if dev.type != "cuda":
        raise ValueError("parse_csv_device needs a GPU device; use har.data.csv_io.read_csv on the host")
    mod = _native.kernels()
    start = 3 if raw[:3] == b"\xef\xbb\xbf" else 0
    host = torch.frombuffer(bytearray(raw), dtype=torch.uint8) if raw else torch.empty(0, dtype=torch.uint8)
    buf = host.pin_memory().to(dev, non_blocking=True) if host.numel() else torch.zeros(1, dtype=torch.uint8,
                                                                                         device=dev)
    if not raw:
        e = torch.empty(0, 0, device=dev)
        return DeviceCsv(raw, buf, [], [], e.double(), e.long(), e.to(torch.uint8), e.long(), e.int())
    starts, ends = _line_spans(buf, start)
    nlines = starts.numel()
    if nlines == 0:
        e = torch.empty(0, 0, device=dev)
        return DeviceCsv(raw, buf, [], [], e.double(), e.long(), e.to(torch.uint8), e.long(), e.int())
    b0, e0 = int(starts[0]), int(ends[0])
    first = _split_header(raw[b0:e0])
    if header:
        names = first
        starts, ends = starts[1:].contiguous(), ends[1:].contiguous()
    else:
        names = [f"_c{i}" for i in range(len(first))]
    nrows, ncols = starts.numel(), len(names)
    vals = torch.empty(ncols, nrows, dtype=torch.float64, device=dev)
    hashes = torch.empty(ncols, nrows, dtype=torch.int64, device=dev)
    flags = torch.empty(ncols, nrows, dtype=torch.uint8, device=dev)
    fstart = torch.empty(ncols, nrows, dtype=torch.int64, device=dev)
    flen = torch.empty(ncols, nrows, dtype=torch.int32, device=dev)
    if nrows:
        mod.csv_parse_rows(buf.data_ptr(), starts.data_ptr(), ends.data_ptr(), nrows, ncols, vals.data_ptr(),
                           hashes.data_ptr(), flags.data_ptr(), fstart.data_ptr(), flen.data_ptr(),
                           _native.stream_ptr(dev))
    kinds, n_inexact = _infer_kinds(vals, flags)
    if n_inexact:
        _fix_inexact(raw, vals, flags, fstart, flen)
    return DeviceCsv(raw, buf, names, kinds, vals, hashes, flags, fstart, flen)


def _fix_inexact(raw: bytes, vals: torch.Tensor, flags: torch.Tensor, fstart: torch.Tensor, flen: torch.Tensor):
    """Fields the kernel's fast path cannot round exactly (mantissa > 2^53 or |exp| > 22, bit
    F_INEXACT) are re-parsed on the host with ``float`` (strtod) — rare, so few bytes move."""
    idx = torch.nonzero(((flags & F_INEXACT) != 0).reshape(-1)).squeeze(1)
    st = fstart.reshape(-1)[idx].cpu().numpy()
    ln = flen.reshape(-1)[idx].cpu().numpy()
    fixed = torch.tensor([float(raw[a:a + b].decode("ascii")) for a, b in zip(st, ln)], dtype=torch.float64)
    vals.view(-1)[idx] = fixed.to(vals.device)


def _infer_kinds(vals: torch.Tensor, flags: torch.Tensor):
    """Per-column type votes as device reductions (one host transfer of [ncols, 4])."""
    ne = (flags & F_NONEMPTY) != 0
    isint = (flags & F_INT) != 0
    isflt = (flags & F_FLOAT) != 0
    any_ne = ne.any(1)
    non_float = (ne & ~isflt).any(1)
    non_int = (ne & ~isint).any(1)
    big = vals.abs() > 9.2e18  # does not fit a Java long -> the column is a double
    fits32 = (vals <= INT32_MAX) & (vals >= INT32_MIN)
    overflow32 = (isint & ~fits32).any(1)
    non_int = non_int | (isint & big).any(1)
    inexact = ((flags & F_INEXACT) != 0).sum(1)
    votes = torch.stack([any_ne, non_float, non_int, overflow32, inexact.bool()], 1).cpu().numpy()
    kinds = []
    for a, nf, ni, ov, _ in votes:
        if not a or nf:
            kinds.append("string")
        elif not ni:
            kinds.append("long" if ov else "int")
        else:
            kinds.append("double")
    return kinds, int(votes[:, 4].sum())


def read_numeric_device(path: str, columns: List[str], device="cuda") -> Dict[str, torch.Tensor]:
    """Convenience: parse on the GPU and return the named numeric columns (fp32, NaN missing)."""
    d = read_csv_device(path, device)
    return {c: d.numeric([c])[:, 0] for c in columns}
