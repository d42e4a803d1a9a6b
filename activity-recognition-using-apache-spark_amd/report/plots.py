"""EDA plots (``Main/main.py:686-710``, ``Main/matplot.py``): a 10% sample of the
numeric columns, one pandas hexbin per ordered column pair
(``Fig <x>_<y>.png``) and a scatter matrix (``Scatter_Matrix.png``).

Differences: runs headless (Agg backend, no ``get_ipython``), uses the current
pandas ``plotting.scatter_matrix`` and a plain style, and writes ``Fig x_y.png``
(the reference's ``Fig: x_y.png`` name is invalid on Windows, where its colon
was mangled).  Sampling is Philox-seeded, so reruns produce the same figures.
"""
from __future__ import annotations

import os
from typing import List, Sequence

import numpy as np

from ..data.table import Table
from ..ops import rng


def sample_numeric(table: Table, cols: Sequence[str], fraction: float = 0.1, seed: int = 0):
    import pandas as pd

    u = rng.uniform(seed, rng.STREAM_SAMPLE, np.arange(table.count(), dtype=np.uint64))
    rows = np.nonzero(u < fraction)[0]
    return pd.DataFrame({c: table[c].data[rows].astype(np.float64) for c in cols})


def write_plots(table: Table, cols: Sequence[str], out_dir: str, fraction: float = 0.1, seed: int = 0,
                hexbin: bool = True, scatter: bool = True) -> List[str]:
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    os.makedirs(out_dir, exist_ok=True)
    df = sample_numeric(table, cols, fraction, seed)
    written = []
    n = len(df.columns)
    if hexbin:
        for i in range(n):
            for j in range(n):
                ax = df.plot.hexbin(x=i, y=j, sharex=False, gridsize=25)
                p = os.path.join(out_dir, f"Fig {ax.xaxis.get_label_text()}_{ax.yaxis.get_label_text()}.png")
                plt.savefig(p)
                plt.close("all")
                written.append(p)
    if scatter:
        written.append(_pair_grid(df, os.path.join(out_dir, "Scatter_Matrix.png"), plt))
    return written


def _pair_grid(df, path: str, plt) -> str:
    """n x n pair grid drawn directly with matplotlib: histograms on the diagonal,
    translucent scatters elsewhere; only the outer row / column carry axis names
    (horizontal on the left edge, vertical along the bottom) and no tick labels."""
    names = list(df.columns)
    n = len(names)
    fig, grid = plt.subplots(n, n, figsize=(16, 16), squeeze=False)
    vals = [df[c].to_numpy() for c in names]
    for r in range(n):
        for c in range(n):
            ax = grid[r][c]
            if r == c:
                ax.hist(vals[c], bins=20, color="tab:blue")
            else:
                ax.scatter(vals[c], vals[r], s=2, alpha=0.2, color="tab:blue")
            ax.set_xticks([])
            ax.set_yticks([])
            if c == 0:
                ax.set_ylabel(names[r], rotation="horizontal", horizontalalignment="right")
            if r == n - 1:
                ax.set_xlabel(names[c], rotation="vertical")
    fig.subplots_adjust(wspace=0, hspace=0)
    fig.savefig(path)
    plt.close(fig)
    return path
