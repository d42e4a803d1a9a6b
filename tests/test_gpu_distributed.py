"""Data-parallel forests on the device level loop: several ranks share the one GPU of the test box
(gloo carries the collectives, staged through the host; RCCL runs the same calls on device
buffers).  The DP fit must grow the single-process forest bit for bit and read nothing back to
the host inside the level loop (models/tree.py `_levels_device_frontier`: every collective is sized
by the level's host-known node bound)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(n=12000, f=12, k=4, seed=0):
    g = torch.Generator().manual_seed(seed)
    mu = torch.randn(k, f, generator=g) * 1.2
    y = torch.randint(0, k, (n,), generator=g)
    return mu[y] + torch.randn(n, f, generator=g), y


def _estimator(kind):
    from har.models.tree import DecisionTreeClassifier, RandomForestClassifier

    if kind == "dt":
        return DecisionTreeClassifier(maxDepth=7, seed=3)
    return RandomForestClassifier(numTrees=12, maxDepth=6, seed=5)


def _count_level_reads(fn):
    """Run fn with Tensor.cpu / .item / .tolist / .numpy counted while the level loop runs."""
    from har.models import tree as tr

    names = ("cpu", "item", "tolist", "numpy")
    real = {n: getattr(torch.Tensor, n) for n in names}
    real_loop = tr._levels_device_frontier
    state = {"in_loop": False, "reads": 0}

    def wrap(n):
        def f(self, *a, **kw):
            if state["in_loop"]:
                state["reads"] += 1
            return real[n](self, *a, **kw)
        return f

    def loop(*a, **kw):
        state["in_loop"] = True
        try:
            return real_loop(*a, **kw)
        finally:
            state["in_loop"] = False

    for n in names:
        setattr(torch.Tensor, n, wrap(n))
    tr._levels_device_frontier = loop
    try:
        out = fn()
    finally:
        for n in names:
            setattr(torch.Tensor, n, real[n])
        tr._levels_device_frontier = real_loop
    return out, state["reads"]


def _worker(rank, world, port, out_dir, kind, reduction):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from har.models import tree as tr
    from har.ops import tree as T
    from har.parallel import data_parallel as dp
    from har.parallel import dist as hd

    ctx = hd.init(backend="gloo", device="cuda")
    X, y = _data()
    thr = T.find_thresholds(X.numpy(), 32)
    Xs, ys, off = dp.shard(X, y, ctx)
    Xs, ys = Xs.to(ctx.device), ys.to(ctx.device)
    est = _estimator(kind)
    kw = dict(owner=dp.NodeOwner(ctx)) if reduction == "owner" else dict(allreduce=dp.allreduce_sum(ctx))
    syncs0 = tr.LEVEL_SYNCS
    m, reads = _count_level_reads(lambda: est.fit_tensors(Xs, ys, 4, row_offset=off, thresholds=thr, **kw))
    a = m.arrs
    torch.save({"feature": a.feature.cpu(), "threshold": a.threshold.cpu(), "stats": a.stats.cpu(),
                "reads": torch.tensor([reads, tr.LEVEL_SYNCS - syncs0])}, os.path.join(out_dir, f"{rank}.pt"))
    hd.shutdown(ctx)


@pytest.mark.parametrize("kind,reduction,world", [("rf", "owner", 2), ("rf", "allreduce", 2), ("dt", "owner", 3),
                                                  ("rf", "owner", 4), ("rf", "owner", 8)])
def test_dp_device_forest_equals_single_with_one_read_per_level(cuda, kind, reduction, world):
    from har.ops import tree as T

    d = tempfile.mkdtemp()
    mp.spawn(_worker, args=(world, _free_port(), d, kind, reduction), nprocs=world, join=True)
    outs = [torch.load(os.path.join(d, f"{r}.pt"), weights_only=True) for r in range(world)]
    X, y = _data()
    thr = T.find_thresholds(X.numpy(), 32)
    m = _estimator(kind).fit_tensors(X.to(cuda), y.to(cuda), 4, thresholds=thr)
    a = m.arrs
    for o in outs:
        # per level one 16-byte count record (+ the roots') and, on the packed owner path, one
        # (2P + 1)-int layout header (ops.tree.dp_wire_plan) are read back: the collectives are sized
        # by the real node counts and present classes; nothing else leaves the device inside the loop
        assert o["reads"][1] <= m.arrs.max_depth + 1 and o["reads"][0] <= 3 * (m.arrs.max_depth + 1), o["reads"]
        assert torch.equal(o["feature"], a.feature.cpu())
        assert torch.equal(o["threshold"], a.threshold.cpu())
        assert torch.equal(o["stats"], a.stats.cpu())
