"""Multi-process data parallelism on the gloo backend (same code path as RCCL):
DP results must equal single-process results (SURVEY.md §4 'Distributed without
a cluster')."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(n=1200, f=12, k=4, seed=0):
    g = torch.Generator().manual_seed(seed)
    mu = torch.randn(k, f, generator=g) * 1.5
    y = torch.randint(0, k, (n,), generator=g)
    return mu[y] + torch.randn(n, f, generator=g), y


def _stream(n=3001, seed=4):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, 3, generator=g).cumsum(0) * 0.1


def _worker(rank, world, port, out_dir, what):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from har.parallel import data_parallel as dp
    from har.parallel import dist as hd

    ctx = hd.init(device="cpu")
    X, y = _data()
    Xs, ys, off = dp.shard(X, y, ctx)
    if what == "lr":
        import torch.distributed as tdist

        from har.models.logreg import FitSpec, LogisticRegression

        n_coll = [0]
        real = tdist.all_reduce

        def counting(*a, **kw):  # every collective of the fit goes through all_reduce
            n_coll[0] += 1
            return real(*a, **kw)

        tdist.all_reduce = counting
        try:
            ms = dp.fit_logreg_dp(LogisticRegression(maxIter=15), Xs, ys,
                                  [FitSpec(None, 0.1, 0.0), FitSpec(None, 0.05, 0.3)], 4, ctx)
        finally:
            tdist.all_reduce = real
        res = torch.stack([m.coefficientMatrix for m in ms])
        torch.save(torch.tensor([n_coll[0], ms[0].summary["n_evals"]]), os.path.join(out_dir, f"lrcoll_{rank}.pt"))
    elif what in ("rf", "rf_allreduce"):
        from har.models.tree import RandomForestClassifier

        m = dp.fit_forest_dp(RandomForestClassifier(numTrees=8, maxDepth=4, seed=5), Xs, ys, 4, off, ctx,
                             reduction="owner" if what == "rf" else "allreduce")
        res = m.predict_raw(X)
    elif what == "rf_tree":
        from har.models.tree import RandomForestClassifier
        from har.ops import tree as T

        thr = T.find_thresholds(X.numpy(), 32)
        m = dp.fit_forest_tree_parallel(RandomForestClassifier(numTrees=7, maxDepth=4, seed=5), X, y, 4, ctx,
                                        thresholds=thr)
        res = m.predict_raw(X)
    elif what == "stream":
        from har.features.window import WindowFeaturizer
        from har.parallel.stream import sharded_window_features

        S = _stream()
        # unequal shards, cuts not on a window / stride boundary, every shard longer than the halo
        cuts = [0] + [int(3001 * (q + 0.37 * (q % 2)) / world) for q in range(1, world)] + [3001]
        local = S[cuts[rank]:cuts[rank + 1]]
        feats, first = sharded_window_features(ctx, local, WindowFeaturizer(hz=20.0, seconds=10.0, overlap=0.5))
        res = torch.cat([torch.tensor([[float(first)] * feats.shape[1]]), feats])
    elif what == "stream_short":
        from har.features.window import WindowFeaturizer
        from har.parallel.stream import sharded_window_features

        S = _stream()
        local = S[:2900] if rank == 0 else S[2900:]  # rank 1: 101 samples < halo of 199
        try:
            sharded_window_features(ctx, local, WindowFeaturizer(hz=20.0, seconds=10.0, overlap=0.5))
            res = torch.tensor([0.0])
        except ValueError:
            res = torch.tensor([1.0])  # every rank must raise (none may block in the p2p exchange)
    else:
        from har.models.mlp import MLPEngine

        os.environ["HAR_MLP_SHARDED_OPT"] = "0" if what == "mlp_ar" else "1"
        per = 128 // world
        eng = MLPEngine([12, 32, 4], per, "cpu", lr=1e-2, seed=1, process_group=ctx.group, world_size=ctx.world_size)
        lo = rank * per
        for s in range(3):  # global batch 128 = world ranks x 128 / world rows
            b = slice(s * 128 + lo, s * 128 + lo + per)
            eng.train_step(X[b], y[b], 128)
        res = eng.P.clone()
    torch.save(res, os.path.join(out_dir, f"{what}_{rank}.pt"))
    hd.shutdown(ctx)


def _run(what, world=2):
    d = tempfile.mkdtemp()
    mp.spawn(_worker, args=(world, _free_port(), d, what), nprocs=world, join=True)
    return [torch.load(os.path.join(d, f"{what}_{r}.pt"), weights_only=True) for r in range(world)]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dp_logreg_equals_single(world):
    from har.models.logreg import FitSpec, LogisticRegression

    d = tempfile.mkdtemp()
    mp.spawn(_worker, args=(world, _free_port(), d, "lr"), nprocs=world, join=True)
    outs = [torch.load(os.path.join(d, f"lr_{r}.pt"), weights_only=True) for r in range(world)]
    for o in outs[1:]:
        torch.testing.assert_close(outs[0], o)
    for r in range(world):  # ONE all-reduce per objective evaluation (+ the summarizer's)
        n_coll, n_evals = torch.load(os.path.join(d, f"lrcoll_{r}.pt"), weights_only=True).tolist()
        assert n_evals > 5 and n_coll == n_evals + 1, (n_coll, n_evals)
    X, y = _data()
    ms = LogisticRegression(maxIter=15).fit_many(X, y, [FitSpec(None, 0.1, 0.0), FitSpec(None, 0.05, 0.3)], 4)
    torch.testing.assert_close(outs[0], torch.stack([m.coefficientMatrix for m in ms]), rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("what,world", [("rf", 2), ("rf", 3), ("rf", 4), ("rf", 8), ("rf_allreduce", 2),
                                        ("rf_allreduce", 8)])
def test_dp_forest_equals_single(what, world):
    """Owner-computes (reduce-scatter by node + all-gather of winners; world 3 leaves
    uneven node slices) and all-reduce histogram reductions both equal one process."""
    from har.models.tree import RandomForestClassifier
    from har.ops import tree as T

    outs = _run(what, world)
    for o in outs[1:]:
        torch.testing.assert_close(outs[0], o)
    X, y = _data()
    # single process with the thresholds the DP run used (rank 0 sample of both shards == all rows here)
    thr = T.find_thresholds(X.numpy(), 32)
    single = RandomForestClassifier(numTrees=8, maxDepth=4, seed=5).fit_tensors(X, y, 4, thresholds=thr)
    torch.testing.assert_close(outs[0], single.predict_raw(X))


@pytest.mark.parametrize("world", [2, 8])
def test_dp_mlp_equals_single(world):
    from har.models.mlp import MLPEngine

    outs = _run("mlp", world)
    for o in outs[1:]:
        torch.testing.assert_close(outs[0], o)
    X, y = _data()
    eng = MLPEngine([12, 32, 4], 128, "cpu", lr=1e-2, seed=1)
    for s in range(3):
        eng.train_step(X[s * 128:(s + 1) * 128], y[s * 128:(s + 1) * 128], 128)
    torch.testing.assert_close(outs[0], eng.P, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("world", [2, 8])
def test_dp_mlp_sharded_optimizer_matches_allreduce(world):
    """Sharded optimizer (reduce-scatter of G, Adam on the owned 1/N slice, all-gather of P) vs the
    all-reduce step: every rank bit-identical in both, and the two steps equal — bitwise at world 2
    (a two-rank sum is one commutative add in either collective), to rounding at world 8 (the
    reduce-scatter and the all-reduce may pair the rank partials in different orders)."""
    sh = _run("mlp", world)
    ar = _run("mlp_ar", world)
    for o in sh[1:]:
        assert torch.equal(sh[0], o)
    for o in ar[1:]:
        assert torch.equal(ar[0], o)
    if world == 2:
        assert torch.equal(sh[0], ar[0])
    else:
        torch.testing.assert_close(sh[0], ar[0], rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_stream_halo_equals_single(world):
    from har.features.window import WindowFeaturizer

    outs = _run("stream", world)
    full = WindowFeaturizer(hz=20.0, seconds=10.0, overlap=0.5).transform(_stream())
    firsts = [int(o[0, 0]) for o in outs]
    got = torch.cat([o[1:] for o in outs])
    assert firsts[0] == 0
    for q in range(1, world):  # contiguous window ids across the shards
        assert firsts[q] == firsts[q - 1] + outs[q - 1].shape[0] - 1
    torch.testing.assert_close(got, full, equal_nan=True)


def test_sharded_stream_short_shard_raises_on_every_rank():
    outs = _run("stream_short")
    assert [float(o[0]) for o in outs] == [1.0, 1.0]


def _main_worker(rank, world, port, out_dir, argv):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    import main

    main.main(argv + ["--out-dir", out_dir])


@pytest.mark.parametrize("world", [2, 8])
def test_main_data_parallel_matches_single(tmp_path, wisdm_csv, world):
    """``torchrun main.py`` (2 or 8 gloo ranks): every model fit data-parallel on row shards —
    LR (all-reduced objective), DT / RF (owner-computed levels), NaiveBayes (all-reduced
    moments) — gives the single-process metrics; rank 0 alone writes the artefacts."""
    import json

    import main

    argv = ["--data", wisdm_csv, "--device", "cpu", "--classifiers", "lr,dt,rf,nb"]
    mp.spawn(_main_worker, args=(world, _free_port(), str(tmp_path / "dp"), argv), nprocs=world, join=True)
    dp = json.loads((tmp_path / "dp" / "metrics.jsonl").read_text().splitlines()[-1])
    single = main.run(main.config_from_args(argv + ["--out-dir", str(tmp_path / "one")]))
    assert dp["world_size"] == world and single["world_size"] == 1
    for name in ("lr", "dt", "rf", "nb"):
        a, b = dp["models"][name], single["models"][name]
        tol = 0.0 if name in ("dt", "rf") else 2e-3  # LR / NB: fp32 sums in another order
        assert abs(a["accuracy"] - b["accuracy"]) <= tol, (name, a["accuracy"], b["accuracy"])
    rows = (tmp_path / "dp" / "additional_param.csv").read_text().splitlines()
    assert len(rows) == 5  # header + 4 models, written once (rank 0)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_tree_parallel_forest_equals_single(world):
    """Tree parallelism: ranks grow disjoint tree-id slices (7 trees over 2 or 3 ranks: uneven)
    over all rows; the all-gathered forest is the single-process forest."""
    from har.models.tree import RandomForestClassifier
    from har.ops import tree as T

    outs = _run("rf_tree", world)
    for o in outs[1:]:
        torch.testing.assert_close(outs[0], o)
    X, y = _data()
    thr = T.find_thresholds(X.numpy(), 32)
    single = RandomForestClassifier(numTrees=7, maxDepth=4, seed=5).fit_tensors(X, y, 4, thresholds=thr)
    torch.testing.assert_close(outs[0], single.predict_raw(X))


@pytest.mark.parametrize("config,extra", [("mlp", ["--batch", "512"]), ("rf", ["--rows", "3000", "--trees", "3"]),
                                          ("stream", ["--stream-pass", "--samples", "8000000", "--batch", "512"])])
def test_bench_contract_torchrun(config, extra):
    """The driver's N>1 launch (``torch.distributed.run ... bench.py --gpus N``) on 2 gloo ranks:
    exactly one JSON line (rank 0), whole-job aggregate value, dp2 config."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--config", config] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=root,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2" and rec["value"] > 0
    if config == "stream":  # full pass: both shards featurized (halo exchange across the cut), same step count
        assert rec["windows_featurized_per_pass"] >= 9990 and rec["mlp_steps_per_pass"] >= 9
    if config == "mlp":  # value = whole-job windows per second = global batch / step time
        assert abs(rec["value"] - rec["config"]["global_batch"] / (rec["ms_per_step"] * 1e-3)) <= 1e-6 * rec["value"]
        ph = rec["phase_ms"]  # the DP step's split: compute, the all-reduce of G, Adam
        assert ph["world"] == 2 and all(ph[k] >= 0 for k in ("compute", "allreduce", "adam")) and ph["allreduce"] > 0


def _bench_torchrun(world, args, timeout=900):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", str(world)] + args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=root,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_rf9_tree_parallel_world8():
    """``bench.py --config rf9 --rf-parallel tree`` under a gloo world of 8: one JSON line, every rank
    holds the whole 8 x --rows table and grows numTrees / 8 trees, and the only collective of a fit is
    ONE all-gather of the packed node arrays."""
    rec = _bench_torchrun(8, ["--steps", "1", "--warmup", "0", "--config", "rf9", "--rf-parallel", "tree",
                              "--rows", "200", "--trees", "16", "--depth", "4"])
    assert rec["n_gpus"] == 8 and rec["rf_parallel"] == "tree" and rec["config"]["global_batch"] == 1600
    coll = rec["collectives_per_step"]
    assert coll["all_gather"] == 1 and set(coll) == {"all_gather", "bytes"} and coll["bytes"] > 0


def test_rf_parallel_modes_same_forest_at_n1():
    """At N = 1 the tree-parallel and data-parallel entry points give the same forest."""
    from har.models.tree import RandomForestClassifier
    from har.ops import tree as T
    from har.parallel import data_parallel as dp
    from har.parallel.dist import DistContext

    X, y = _data()
    thr = T.find_thresholds(X.numpy(), 32)
    ctx = DistContext(rank=0, world_size=1, local_rank=0, device=torch.device("cpu"), backend="gloo")
    a = dp.fit_forest_tree_parallel(RandomForestClassifier(numTrees=6, maxDepth=4, seed=5), X, y, 4, ctx,
                                    thresholds=thr)
    b = RandomForestClassifier(numTrees=6, maxDepth=4, seed=5).fit_tensors(X, y, 4, thresholds=thr)
    torch.testing.assert_close(a.predict_raw(X), b.predict_raw(X))


def _forced_worker(rank, port, out_dir):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(k, None)
    os.environ.update(HAR_DIST_FORCE_PG="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    import torch.distributed as tdist

    from har.models.mlp import MLPEngine
    from har.parallel import comm
    from har.parallel import data_parallel as dp
    from har.parallel import dist as hd

    ctx = hd.init(device="cpu")
    res = {"forced": ctx.forced, "collective": ctx.collective, "backend": ctx.backend,
           "initialized": tdist.is_initialized(), "allreduce_fn": dp.allreduce_sum(ctx) is not None,
           "sum": hd.sum_over_ranks(ctx, 2.5)}
    X, y = _data()
    for sharded in ("1", "0"):
        os.environ["HAR_MLP_SHARDED_OPT"] = sharded
        a = MLPEngine([12, 32, 4], 128, "cpu", lr=1e-2, seed=1)
        b = MLPEngine([12, 32, 4], 128, "cpu", lr=1e-2, seed=1, process_group=ctx.group, world_size=1, force_dp=True)
        n = [0]
        real = (comm.reduce_scatter_tensor, comm.all_reduce)

        def rs(*x, **k):
            n[0] += 1
            return real[0](*x, **k)

        def ar(*x, **k):
            n[0] += 1
            return real[1](*x, **k)

        comm.reduce_scatter_tensor, comm.all_reduce = rs, ar
        try:
            for s in range(3):
                a.train_step(X[s * 128:(s + 1) * 128], y[s * 128:(s + 1) * 128], 128)
                b.train_step(X[s * 128:(s + 1) * 128], y[s * 128:(s + 1) * 128], 128)
        finally:
            comm.reduce_scatter_tensor, comm.all_reduce = real
        res[f"equal_{sharded}"] = bool(torch.equal(a.P, b.P) and torch.equal(a.m, b.m) and torch.equal(a.v, b.v))
        res[f"coll_{sharded}"] = n[0]
        res[f"dp_{sharded}"] = (b.dp, b.sharded)
    # unset: the form follows the parameter count (models/mlp.py SHARD_MIN_PARAMS)
    import har.models.mlp as mlp_mod

    os.environ.pop("HAR_MLP_SHARDED_OPT", None)
    small = MLPEngine([12, 32, 4], 128, "cpu", lr=1e-2, seed=1, process_group=ctx.group, world_size=1, force_dp=True)
    old_min = mlp_mod.SHARD_MIN_PARAMS
    mlp_mod.SHARD_MIN_PARAMS = 16
    try:
        big = MLPEngine([12, 32, 4], 128, "cpu", lr=1e-2, seed=1, process_group=ctx.group, world_size=1,
                        force_dp=True)
    finally:
        mlp_mod.SHARD_MIN_PARAMS = old_min
    res["auto"] = (small.sharded, big.sharded)
    torch.save(res, os.path.join(out_dir, "forced.pt"))
    hd.shutdown(ctx)


def test_forced_one_rank_group_runs_the_dp_paths():
    """HAR_DIST_FORCE_PG=1 at WORLD_SIZE 1: a 1-rank group (gloo here, RCCL on a GPU) is created, the
    DP paths issue their collectives on it, and the DP MLP step (sharded and all-reduce) equals the
    single-process step bit for bit."""
    d = tempfile.mkdtemp()
    mp.spawn(_forced_worker, args=(_free_port(), d), nprocs=1, join=True)
    r = torch.load(os.path.join(d, "forced.pt"), weights_only=True)
    assert r["forced"] and r["collective"] and r["backend"] == "gloo" and r["initialized"]
    assert r["allreduce_fn"] and r["sum"] == 2.5
    assert r["equal_1"] and r["equal_0"], r
    assert r["coll_1"] == 3 and r["coll_0"] == 3, r  # one gradient collective per step
    assert tuple(r["dp_1"]) == (True, True) and tuple(r["dp_0"]) == (True, False)
    assert tuple(r["auto"]) == (False, True)  # small gradient: one all-reduce; from SHARD_MIN_PARAMS: sharded
