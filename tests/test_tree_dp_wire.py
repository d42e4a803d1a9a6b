"""The DP forest's packed wire format (ops.tree.dp_wire_plan + csrc/kernels/tree_dp.hip): present
classes only, 8 / 16 / 32-bit integer fields by node weight, word-balanced owner ranges.  The integer
sum of packed words over ranks must unpack to the exact sum of the ranks' fp32 histograms."""
import numpy as np
import pytest
import torch

from har.ops import tree as T


def _random_level(A, K, mb, P, seed):
    """P ranks' integer histograms of A nodes whose global class counts span all three widths."""
    g = np.random.default_rng(seed)
    scale = g.choice([3, 100, 3000, 40000, 200000], size=A)
    present = g.random((A, K)) < 0.4
    present[np.arange(A), g.integers(0, K, A)] = True
    hist = np.zeros((P, A, mb, K), np.int64)
    for a in range(A):
        for k in np.nonzero(present[a])[0]:
            # rank parts of the class's count, spread over the (feature, bin) cells
            tot = int(g.integers(1, scale[a] + 1))
            cells = g.integers(0, mb, tot if tot < 5000 else 5000)
            w = np.full(len(cells), tot // len(cells))
            w[: tot - w.sum()] += 1
            ranks = g.integers(0, P, len(cells))
            np.add.at(hist, (ranks, a, cells, k), w)
    cc = hist.sum(0).sum(1)  # [A, K] global class counts
    return hist, cc


def _pack_numpy(store, cls, kp, bw, woff, P, wmax):
    """Host mirror of dp_pack_kernel."""
    A, mb, K = store.shape
    out = np.zeros(P * wmax, np.int64)
    for a in range(A):
        per, sh = 4 // bw[a], 8 * bw[a]
        seq = store[a][:, cls[a, :kp[a]]].reshape(-1)
        for i, v in enumerate(seq):
            out[woff[a] + i // per] += int(v) << (sh * (i % per)) if bw[a] < 4 else int(v)
    return out


def test_dp_wire_plan_layout_cpu():
    A, K, mb, P = 37, 6, 10, 4
    hist, cc = _random_level(A, K, mb, P, seed=5)
    cls, kp, bw, woff, bounds, wmax = T.dp_wire_plan(torch.from_numpy(cc).float(), mb, P)
    cls, kp, bw, woff = cls.numpy(), kp.numpy(), bw.numpy(), woff.numpy()
    assert bounds[0] == 0 and bounds[-1] == A and all(bounds[q] <= bounds[q + 1] for q in range(P))
    w = cc.sum(1)
    assert np.array_equal(bw, np.where(w < 256, 1, np.where(w < 65536, 2, 4)))
    assert np.array_equal(kp, (cc > 0).sum(1))
    for a in range(A):  # present classes ascending at the front
        assert list(cls[a, :kp[a]]) == list(np.nonzero(cc[a] > 0)[0])
    # node word ranges: inside their owner's row, disjoint, and covering mb * kp fields
    used = np.zeros(P * wmax, bool)
    for q in range(P):
        for a in range(bounds[q], bounds[q + 1]):
            nw = -(-mb * kp[a] // (4 // bw[a]))
            lo = woff[a]
            assert q * wmax <= lo and lo + nw <= (q + 1) * wmax
            assert not used[lo:lo + nw].any()
            used[lo:lo + nw] = True
    # the packed integer sum over ranks decodes field by field to the summed histogram
    tot = sum(_pack_numpy(hist[p], cls, kp, bw, woff, P, wmax) for p in range(P))
    summed = hist.sum(0)
    for a in range(A):
        per, sh = 4 // bw[a], 8 * bw[a]
        n = mb * kp[a]
        vals = [(int(tot[woff[a] + i // per]) >> (sh * (i % per))) & ((1 << sh) - 1) if bw[a] < 4
                else int(tot[woff[a] + i]) for i in range(n)]
        assert np.array_equal(np.array(vals).reshape(mb, kp[a]), summed[a][:, cls[a, :kp[a]]])
    # the dense fp32 store would be A * mb * K * 4 bytes per rank
    assert P * wmax * 4 < A * mb * K * 4


@pytest.mark.gpu
def test_dp_pack_unpack_gpu_sum_exact(cuda):
    from har.ops import _native

    A, K, mb, P = 53, 12, 13 * 32, 3
    hist, cc = _random_level(A, K, mb, P, seed=9)
    slot = mb * K
    cls, kp, bw, woff, bounds, wmax = T.dp_wire_plan(torch.from_numpy(cc).float().to(cuda), mb, P)
    mod, st = _native.kernels(), _native.stream_ptr()
    tot = torch.zeros(P * wmax, dtype=torch.int32, device=cuda)
    for p in range(P):
        store = torch.from_numpy(hist[p].reshape(-1)).float().to(cuda)
        out = torch.full((P * wmax,), 0, dtype=torch.int32, device=cuda)
        mod.tree_dp_pack(store.data_ptr(), A, slot, mb, K, cls.data_ptr(), kp.data_ptr(), bw.data_ptr(),
                         woff.data_ptr(), out.data_ptr(), st)
        tot += out  # the integer SUM a reduce-scatter performs
    summed = torch.from_numpy(hist.sum(0)).float().to(cuda)
    for r in range(P):
        a0, a1 = bounds[r], bounds[r + 1]
        if a1 == a0:
            continue
        loc = torch.full(((a1 - a0) * slot,), float("nan"), device=cuda)
        row = tot[r * wmax:(r + 1) * wmax].contiguous()
        mod.tree_dp_unpack(row.data_ptr(), a0, a1 - a0, slot, mb, K, cls.data_ptr(), kp.data_ptr(), bw.data_ptr(),
                           woff.data_ptr(), r * wmax, loc.data_ptr(), st)
        torch.cuda.synchronize()
        assert torch.equal(loc.view(a1 - a0, mb, K), summed[a0:a1]), f"rank {r} unpack differs"
