"""Raw accelerometer ingest -> the WISDM *transformed* table, on the device.

The reference starts from WISDM's pre-windowed table (``Main/main.py:16-20``,
``wisdm_data.csv:1``: ``UID, USER, X0..Z9, XAVG.., XPEAK.., XABSDEV.., XSTDDEV..,
RESULTANT, ACTIVITY``).  The transform that produced it (Kwapisz et al. 2010: 10-s
windows, per axis 10-bin distribution / average / time between peaks / average
absolute deviation / standard deviation, average resultant) is not in the
reference.  This module runs it on raw samples so ``main.py --raw`` covers the whole
pipeline from sensor rows:

1. read ``user,activity,timestamp,x,y,z`` rows — a CSV with that header, or the
   WISDM v1.1 raw text layout (no header, ``;`` line terminators) — with the native
   host CSV parser;
2. segment the stream into maximal runs of one (user, activity) in file order, and
   place windows of ``round(hz * window_sec)`` samples every
   ``round(window * (1 - overlap))`` samples inside each run (a window never spans
   two users or activities);
3. featurize every window with the HIP window kernel (``window.hip``: LDS-staged
   samples, wave reductions), or its PyTorch oracle on the CPU; under
   ``torch.distributed`` each rank featurizes the windows that START in its
   contiguous shard of the samples, fetching the ``window - 1`` samples past its end
   from the next rank (``parallel.stream.exchange_halo``), and the rows are
   all-gathered;
4. emit the 46 WISDM columns with their names and types (``*PEAK`` as strings, ``?``
   when a window has fewer than two peaks — the missing marker of the original
   table), so ``features.wisdm.prepare`` and the rest of ``main.py`` run unchanged.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from ..data.table import Column, Table
from .window import NBINS, window_features, window_features_torch

AXES = ("X", "Y", "Z")
WISDM43 = ([f"{a}{i}" for a in AXES for i in range(NBINS)] + [a + "AVG" for a in AXES] + [a + "PEAK" for a in AXES]
           + [a + "ABSDEV" for a in AXES] + [a + "STDDEV" for a in AXES] + ["RESULTANT"])
ACTIVITIES = ("Walking", "Jogging", "Upstairs", "Downstairs", "Sitting", "Standing")


def read_raw(path: str):
    """(user int64 [S], activity object [S], timestamp int64 [S], xyz float32 [S, 3])."""
    from ..data.csv_io import parse_csv_bytes

    with open(path, "rb") as f:
        buf = f.read()
    first = buf.split(b"\n", 1)[0].strip().lower()
    header = first.startswith(b"user")
    if b";" in buf[:4096]:  # WISDM raw text: "33,Jogging,49105962326000,-0.69,12.68,0.50;"
        buf = buf.replace(b";", b"")
    t = parse_csv_bytes(buf, header=header)
    cols = t.columns
    if len(cols) < 6:
        raise ValueError(f"{path}: expected user,activity,timestamp,x,y,z columns, got {cols}")
    c = [t[n] for n in cols[:6]]
    ok = np.ones(t.count(), dtype=bool)
    for col in (c[0], c[2], c[3], c[4], c[5]):
        if col.kind == "string":
            raise ValueError(f"{path}: column {col.name} is not numeric")
        if col.missing is not None:
            ok &= ~col.missing
    xyz = np.stack([c[3].data, c[4].data, c[5].data], 1).astype(np.float32)
    ok &= np.isfinite(xyz).all(1)
    act = np.asarray([str(v) for v in c[1].data], dtype=object)
    return c[0].data.astype(np.int64)[ok], act[ok], c[2].data.astype(np.int64)[ok], xyz[ok]


def window_starts(user: np.ndarray, activity: np.ndarray, window: int, stride: int) -> Tuple[np.ndarray, np.ndarray]:
    """(start sample of every window, index of its segment's first sample); windows stay inside
    maximal runs of one (user, activity)."""
    n = len(user)
    if n == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    _, acode = np.unique(activity.astype(str), return_inverse=True)
    change = np.ones(n, dtype=bool)
    change[1:] = (user[1:] != user[:-1]) | (acode[1:] != acode[:-1])
    seg_lo = np.nonzero(change)[0]
    seg_hi = np.append(seg_lo[1:], n)
    nwin = np.where(seg_hi - seg_lo >= window, (seg_hi - seg_lo - window) // stride + 1, 0)
    seg_of = np.repeat(np.arange(len(seg_lo)), nwin)
    k = np.arange(int(nwin.sum())) - np.repeat(np.cumsum(nwin) - nwin, nwin)
    return seg_lo[seg_of] + k * stride, seg_lo[seg_of]


def featurize_starts(xyz: torch.Tensor, starts: torch.Tensor, window: int, hz: float) -> torch.Tensor:
    """[n, 43] WISDM features of the windows at ``starts`` (sample indices into ``xyz`` [S, 3])."""
    if starts.numel() == 0:
        return torch.zeros(0, len(WISDM43), dtype=torch.float32, device=xyz.device)
    idx = (starts.view(-1, 1) + torch.arange(window, device=xyz.device).view(1, -1)).reshape(-1)
    win = xyz.index_select(0, idx).contiguous()                 # windows back to back: stride == window
    f = window_features(win, window, window, hz) if win.is_cuda else window_features_torch(win, window, window, hz)
    return f[:, :len(WISDM43)]


def _featurize_dp(ctx, xyz_host: np.ndarray, starts: np.ndarray, window: int, hz: float, device) -> torch.Tensor:
    """Rank r featurizes the windows starting in its contiguous sample shard; the last window of a
    shard may run into the next rank's samples: one halo exchange of window - 1 samples."""
    from ..parallel import comm
    from ..parallel.stream import exchange_halo, shard_lengths

    S = xyz_host.shape[0]
    lo, hi = (S * ctx.rank) // ctx.world_size, (S * (ctx.rank + 1)) // ctx.world_size
    local = torch.as_tensor(xyz_host[lo:hi]).to(device)
    lens = shard_lengths(ctx, local.shape[0], local.device)
    ext = torch.cat([local, exchange_halo(ctx, local, window - 1, lens)], 0)
    mine = starts[(starts >= lo) & (starts < hi)] - lo
    f = featurize_starts(ext, torch.as_tensor(mine, device=device), window, hz)
    counts = [int(((starts >= (S * r) // ctx.world_size) & (starts < (S * (r + 1)) // ctx.world_size)).sum())
              for r in range(ctx.world_size)]
    pad = torch.zeros(max(counts), f.shape[1], dtype=f.dtype, device=f.device)
    pad[: f.shape[0]] = f
    allf = torch.zeros(ctx.world_size * pad.shape[0], f.shape[1], dtype=f.dtype, device=f.device)
    comm.all_gather_into_tensor(allf, pad, group=ctx.group)
    allf = allf.view(ctx.world_size, -1, f.shape[1])
    return torch.cat([allf[r, :counts[r]] for r in range(ctx.world_size)], 0)


def raw_to_table(path: str, hz: float = 20.0, window_sec: float = 10.0, overlap: float = 0.0, device=None,
                 ctx=None) -> Table:
    """Raw rows -> the WISDM transformed table (one row per window, columns of ``wisdm_data.csv:1``)."""
    user, act, ts, xyz = read_raw(path)
    window = int(round(hz * window_sec))
    stride = max(1, int(round(window * (1.0 - overlap))))
    if window < 3:
        raise ValueError("window must hold at least 3 samples")
    starts, _ = window_starts(user, act, window, stride)
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if ctx is not None and ctx.is_distributed:
        F = _featurize_dp(ctx, xyz, starts, window, hz, dev)
    else:
        F = featurize_starts(torch.as_tensor(xyz).to(dev), torch.as_tensor(starts, device=dev), window, hz)
    F = F.double().cpu().numpy()
    n = len(starts)
    cols = [Column("UID", "int", np.arange(n, dtype=np.int64)), Column("USER", "int", user[starts])]
    for j, name in enumerate(WISDM43):
        if name.endswith("PEAK"):  # WISDM: integer milliseconds, '?' when < 2 peaks
            v = F[:, j]
            s = np.asarray(["?" if not np.isfinite(p) else str(int(round(p))) for p in v], dtype=object)
            cols.append(Column(name, "string", s))
        else:
            cols.append(Column(name, "double", F[:, j].copy()))
    cols.append(Column("ACTIVITY", "string", np.asarray(act[starts], dtype=object)))
    return Table(cols)


def write_synthetic_raw(path: str, n_windows: int = 400, users: int = 6, seed: int = 2018, hz: float = 20.0,
                        window_sec: float = 10.0, wisdm_txt: bool = False) -> dict:
    """A raw ``user,activity,timestamp,x,y,z`` file from the synthetic stream generator
    (``data.synth``: class-conditional dynamics, activity runs of 8 windows); activity runs are
    dealt to ``users`` round robin and every (user, activity) run is recorded contiguously."""
    from ..data.synth import StreamSpec, generate_stream

    spec = StreamSpec(num_classes=6, axes=3, hz=hz, window=int(round(hz * window_sec)), seed=seed)
    s, y = generate_stream(n_windows, spec)
    W = spec.window
    runs = np.arange(n_windows) // spec.run_windows
    user_of_window = 1 + runs % users
    rows = []
    step_ns = int(round(1e9 / hz))
    for w in range(n_windows):
        u, a = int(user_of_window[w]), ACTIVITIES[int(y[w])]
        for i in range(W):
            x0, x1, x2 = s[w * W + i].tolist()
            rows.append(f"{u},{a},{(w * W + i) * step_ns},{x0:.6g},{x1:.6g},{x2:.6g}")
    with open(path, "w") as f:
        if wisdm_txt:
            f.write(";\n".join(rows) + ";\n")
        else:
            f.write("user,activity,timestamp,x,y,z\n" + "\n".join(rows) + "\n")
    return {"samples": n_windows * W, "window": W, "labels": y.numpy()}
