"""Counter-based Philox4x32-10 randomness keyed by (seed, stream, global row id).

Replaces Spark's XORShiftRandom + per-partition BernoulliCellSampler used by
``df.randomSplit([0.7, 0.3], seed=2018)`` (``Main/main.py:80``), the k-fold
sampler inside ``CrossValidator`` (``Main/main.py:209``) and RandomForest's
Poisson(1) ``BaggedPoint`` weights (``Main/main.py:478``).  Because every draw is
a pure function of the *global* row id, splits, folds and bootstraps are
identical for every world size and every shard layout.

The same function is implemented in ``csrc/kernels/rng.hip`` for device use; the
NumPy version here is the oracle and the CPU path.
"""
from __future__ import annotations

import math

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = 0x9E3779B9
W1 = 0xBB67AE85
TAG = 0x48415221  # "HAR!" — 4th counter word
MASK32 = np.uint64(0xFFFFFFFF)

# stream ids (documented so HIP and NumPy agree)
STREAM_SPLIT = 0
STREAM_KFOLD = 1
STREAM_SAMPLE = 2
STREAM_INIT = 3
STREAM_FINDSPLITS = 4  # findSplits row sample (Bernoulli, keyed by global row id)
STREAM_BOOTSTRAP_BASE = 0x1000  # + tree id
STREAM_FEATURE_SUBSET = 0x7F000000  # per (tree,node) in counter


def philox4x32(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    """Return uint32 array [len(idx), 4] of Philox4x32-10 outputs."""
    idx = np.asarray(idx, dtype=np.uint64)
    c0 = idx & MASK32
    c1 = idx >> np.uint64(32)
    c2 = np.full_like(c0, np.uint64(stream & 0xFFFFFFFF))
    c3 = np.full_like(c0, np.uint64(TAG))
    k0 = seed & 0xFFFFFFFF
    k1 = (seed >> 32) & 0xFFFFFFFF
    for r in range(10):
        if r:
            k0 = (k0 + W0) & 0xFFFFFFFF
            k1 = (k1 + W1) & 0xFFFFFFFF
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ np.uint64(k0)), lo1, (hi0 ^ c3 ^ np.uint64(k1)), lo0
    return np.stack([c0, c1, c2, c3], axis=-1).astype(np.uint32)


def uniform_u32(seed: int, stream: int, idx) -> np.ndarray:
    return philox4x32(seed, stream, idx)[:, 0]


def uniform(seed: int, stream: int, idx) -> np.ndarray:
    """float64 uniforms in [0, 1) with 32-bit resolution (exact on host and device)."""
    return uniform_u32(seed, stream, idx).astype(np.float64) * (1.0 / 4294967296.0)


def bucket_thresholds(weights) -> np.ndarray:
    """Normalized cumulative weights as uint32 thresholds (Spark normalizes the
    randomSplit weights the same way).  Row goes to bucket b iff
    thr[b-1] <= u32 < thr[b]; the last bucket takes everything above."""
    w = np.asarray(weights, dtype=np.float64)
    if np.any(w < 0) or w.sum() <= 0:
        raise ValueError("split weights must be non-negative with positive sum")
    cum = np.cumsum(w / w.sum())
    thr = np.minimum(np.floor(cum * 4294967296.0), 4294967295.0).astype(np.uint64)
    thr[-1] = 1 << 32  # sentinel: everything
    return thr


def assign_buckets(seed: int, stream: int, row_ids, weights) -> np.ndarray:
    u = uniform_u32(seed, stream, row_ids).astype(np.uint64)
    thr = bucket_thresholds(weights)
    return np.searchsorted(thr, u, side="right").astype(np.int64)


def poisson_thresholds(rate: float = 1.0, kmax: int = 15) -> np.ndarray:
    """uint32 CDF thresholds of Poisson(rate): draw = #{k : u >= thr[k]} (rate 1: Spark's
    bootstrap with replacement at subsamplingRate 1)."""
    cdf, p, out = 0.0, math.exp(-float(rate)), []
    for k in range(kmax):
        cdf += p
        p = p * float(rate) / (k + 1)
        out.append(min(int(math.floor(cdf * 4294967296.0)), 4294967295))
    return np.asarray(out, dtype=np.uint64)


def bernoulli_thresholds(rate: float) -> np.ndarray:
    """Sampling without replacement at ``rate`` (Spark: one tree, subsamplingRate < 1): one
    threshold, draw = 1 when u >= (1 - rate) * 2^32."""
    return np.asarray([min(int(math.floor((1.0 - float(rate)) * 4294967296.0)), 4294967295)], dtype=np.uint64)


def _poisson1_thresholds(kmax: int = 15) -> np.ndarray:
    return poisson_thresholds(1.0, kmax)


POISSON1_THR = _poisson1_thresholds()


def bootstrap_weights(seed: int, tree_ids, n_rows: int, row_offset: int = 0, thresholds=None) -> np.ndarray:
    """Per-(tree, global row) bootstrap counts from a CDF threshold table (``poisson_thresholds``
    / ``bernoulli_thresholds``), shape [len(tree_ids), n_rows], uint8; None table = all ones."""
    if thresholds is None:
        return np.ones((len(tree_ids), n_rows), dtype=np.uint8)
    rows = np.arange(row_offset, row_offset + n_rows, dtype=np.uint64)
    out = np.empty((len(tree_ids), n_rows), dtype=np.uint8)
    for i, t in enumerate(tree_ids):
        u = uniform_u32(seed, STREAM_BOOTSTRAP_BASE + int(t), rows).astype(np.uint64)
        out[i] = np.searchsorted(thresholds, u, side="right")
    return out


def poisson1_weights(seed: int, tree_ids, n_rows: int, row_offset: int = 0) -> np.ndarray:
    """Poisson(1) bootstrap counts, shape [len(tree_ids), n_rows], uint8."""
    rows = np.arange(row_offset, row_offset + n_rows, dtype=np.uint64)
    out = np.empty((len(tree_ids), n_rows), dtype=np.uint8)
    for i, t in enumerate(tree_ids):
        u = uniform_u32(seed, STREAM_BOOTSTRAP_BASE + int(t), rows).astype(np.uint64)
        out[i] = np.searchsorted(POISSON1_THR, u, side="right")
    return out


def feature_subsets(seed: int, trees, nodes, n_features: int, m: int) -> np.ndarray:
    """Floyd's sampling of ``m`` distinct features out of ``n_features`` for each
    (tree, node) pair (vectorized over pairs).  Draw i of pair (t, n) uses
    counter ``t<<32 | n<<8 | i`` (so m <= 256, node < 2^24).  Returns int32
    [P, m], each row sorted ascending.  ``csrc/kernels/tree_level.hip`` implements the
    identical procedure per node on device."""
    trees = np.asarray(trees, dtype=np.uint64).reshape(-1)
    nodes = np.asarray(nodes, dtype=np.uint64).reshape(-1)
    P = trees.shape[0]
    if m >= n_features:
        return np.tile(np.arange(n_features, dtype=np.int32), (P, 1))
    assert m <= 256
    base = (trees << np.uint64(32)) | (nodes << np.uint64(8))
    ctr = (base[:, None] + np.arange(m, dtype=np.uint64)[None, :]).reshape(-1)
    draws = philox4x32(seed, STREAM_FEATURE_SUBSET, ctr)[:, 0].reshape(P, m).astype(np.int64)
    chosen = np.empty((P, m), dtype=np.int64)
    for i in range(m):
        j = n_features - m + i
        t = draws[:, i] % (j + 1)
        dup = (chosen[:, :i] == t[:, None]).any(axis=1) if i else np.zeros(P, dtype=bool)
        chosen[:, i] = np.where(dup, j, t)
    chosen.sort(axis=1)
    return chosen.astype(np.int32)


_THR_CACHE = {}


def device_buckets(seed: int, stream: int, row0: int, n: int, weights, device):
    """``assign_buckets`` on the GPU (HIP kernel ``har_philox_buckets``); int32 [n]."""
    import torch

    from . import _native

    key = (tuple(float(w) for w in weights), str(torch.device(device)))
    thr_t = _THR_CACHE.get(key)
    if thr_t is None:  # (a pageable 16-byte upload per call waited on the stream: cached per weights)
        thr = bucket_thresholds(weights)[:-1].astype(np.uint32)
        thr_t = _THR_CACHE[key] = torch.from_numpy(thr.view(np.int32)).to(device)
    out = torch.empty(n, dtype=torch.int32, device=device)
    _native.kernels().philox_buckets(seed, stream, row0, n, thr_t.data_ptr(), thr_t.numel(), out.data_ptr(),
                                     _native.stream_ptr())
    return out


def device_poisson1(seed: int, tree0: int, ntrees: int, row0: int, n: int, device):
    """``poisson1_weights`` on the GPU (HIP kernel ``har_poisson_bootstrap``); uint8 [ntrees, n]."""
    import torch

    from . import _native

    out = torch.empty(ntrees, n, dtype=torch.uint8, device=device)
    _native.kernels().poisson_bootstrap(seed, tree0, ntrees, row0, n, out.data_ptr(), _native.stream_ptr())
    return out
