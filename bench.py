#!/usr/bin/env python3
"""Benchmarks of the BASELINE.json configurations (default = the flagship).

Metric (BASELINE.json): "windows/sec (whole node) + test accuracy on WISDM 6-class
at 1/2/4/8 MI355X".  One process per GPU (``torch.distributed.run``), RCCL over
xGMI, weak scaling (fixed per-GPU work).  Every line is ONE JSON record.

``--config mlp``    (default; BASELINE config 3) WISDM-shaped 6-class 3-layer MLP, bf16
                    MFMA kernels, DP all-reduce of one flat gradient bucket per step.
                    Step = fwd + bwd + all-reduce + Adam on ``--batch`` windows per GPU.
                    Data: synthetic WISDM-shaped windows (43 features, 6 classes,
                    class-conditional Gaussians generated on device); random-init weights.
``--config rf``     (config 2) RandomForest 100 trees x depth 10, 32 bins, on
                    featurized synthetic 3-axis windows (43 WISDM features);
                    step = one whole forest fit (per level in DP: histograms reduce-scattered
                    by node owner, winners all-gathered; ``--rf-reduce allreduce`` for the
                    all-reduce variant).
``--config stream`` (config 4) raw synthetic 3-axis 20 Hz stream (1B samples per
                    8 GPUs, i.e. 125M per GPU resident in HBM) -> HIP window featurizer
                    -> MLP training step; step = featurize + train ``--batch`` windows.
``--config rf9``    (config 5) 12-class 9-axis IMU RandomForest, 500 trees.
``--config dt``     DecisionTree (every feature at every node) on config 2's windows; sibling
                   histogram subtraction on (``--no-subtract``: every node histogrammed directly).
``--config infer``  serving: windows/s classified by the trained config-3 MLP (an fp32 -> bf16 cast
                    kernel + the INFER instantiation of the training forward, logits + argmax); no
                    reference number exists.

``--config reference`` the reference's own four fits on the REAL WISDM table (3100-dim
                    StringIndexer/OneHot encoding, 70/30 split, seed 2018): LogisticRegression
                    (maxIter 20, reg 0.3), LR CrossValidator (3x3 grid x 5 folds, MAE objective as in
                    Main/main.py:175), DecisionTree depth 3, RandomForest 100 trees depth 4.
                    step = the four fits back to back; value = 4 x N_train / step seconds.

``vs_baseline`` is reported only against the SAME model on the SAME data: the
reference config divides by the reference run A's derived training throughput
(LR 418.6, LR-CV 29.2, DT 311.2, RF 185.3 windows/s; suite 88.4).
The reference has no MLP and no synthetic-stream configs, so those records carry
``vs_baseline: null``; they report the MLP's test accuracy on the real WISDM table
(same architecture, trained untimed after the throughput steps) and, at N=1, the
reference suite's same-model comparison in ``reference_suite``.

Usage: python bench.py --gpus N --steps K --warmup W [--config mlp|rf|stream|rf9]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
from har.config import DEFAULT_WISDM  # noqa: E402

METRIC = "windows/sec (whole node) + test accuracy on WISDM 6-class at 1/2/4/8 MI355X"
BASELINE_NOTE = "reference has no MLP / synthetic-stream benchmark: see reference_suite for same-model ratios"
N_FEATURES = 43
N_CLASSES = 6
WINDOW_SAMPLES = 200  # 10 s @ 20 Hz (WISDM v1.1 transformed windows)
WISDM_PRIOR = [2081, 1625, 632, 528, 306, 246]


def synthetic_windows(n: int, seed: int, device, class_seed: int = 2018):
    """Class-conditional Gaussian windows: x = mu[y] + noise; mu shared by all ranks."""
    g = torch.Generator(device="cpu").manual_seed(class_seed)
    mu = torch.randn(N_CLASSES, N_FEATURES, generator=g) * 0.6
    prior = torch.tensor(WISDM_PRIOR, dtype=torch.float64)
    gd = torch.Generator(device=device).manual_seed(seed)
    y = torch.multinomial(prior.to(device).float(), n, replacement=True, generator=gd)
    x = mu.to(device)[y] + torch.randn(n, N_FEATURES, device=device, generator=gd)
    return x, y


def timed(ctx, run, steps, warmup, dev):
    from har.parallel import dist as hdist

    for i in range(warmup):
        run(i)
    hdist.barrier(ctx)
    hdist.sync(dev)
    t0 = time.perf_counter()
    for i in range(steps):
        run(warmup + i)
    hdist.sync(dev)
    hdist.barrier(ctx)
    return hdist.max_over_ranks(ctx, time.perf_counter() - t0)


def settle_clocks(ctx, run, ms, dev):
    """Untimed training steps for ``ms`` of wall time before the warm-up steps (the same step the
    timed loop runs, so the model just trains longer): the timed window then starts at the clocks a
    running job holds instead of inside the power-state ramp of a GPU that was idle a moment ago
    (profiles/r4/bench_settle_ab.md: the driver's 20-step window read 0.0747-0.0758 ms per step
    without, 0.0674-0.0681 ms with >= 100 ms, the 500-step run 0.0689).  Ranks stop together (the
    elapsed time is agreed over the group after every 16 steps), so the DP steps' collectives pair
    up.  Returns the settle time spent (ms)."""
    from har.parallel import dist as hdist

    if ms <= 0 or dev.type != "cuda":
        return 0.0
    t0 = time.perf_counter()
    i = 1 << 20  # step indices past every warm-up / timed index (steps keyed on small i stay untouched)
    while True:
        for _ in range(16):
            run(i)
            i += 1
        torch.cuda.synchronize(dev)
        el = hdist.max_over_ranks(ctx, (time.perf_counter() - t0) * 1e3)
        if el >= ms:
            return el


def capture_steps(step, nslots, enable):
    """HIP-graph capture of one training step per batch slot (launch-bound inner loop)."""
    if not enable:
        return None
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(3):
            step(i)
    torch.cuda.current_stream().wait_stream(s)
    graphs = []
    for j in range(nslots):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step(j)
        graphs.append(g)
    return graphs


def bench_mlp(args, ctx):
    from har.models.mlp import MLPEngine, pad_input_bf16
    from har.parallel import dist as hdist

    dev, rank, world = ctx.device, ctx.rank, ctx.world_size
    B = args.batch
    layers = [N_FEATURES, args.hidden, args.hidden, N_CLASSES]
    eng = MLPEngine(layers, B, dev, lr=args.lr, seed=1234, process_group=ctx.group, world_size=world,
                    force_dp=ctx.forced)
    n_local = B * 8  # resident per-rank shard: 8 batches of windows
    X, y = synthetic_windows(n_local, seed=100 + rank, device=dev)
    Xin = pad_input_bf16(X, eng.layout.in_pad) if eng.native else X
    y32 = y.to(torch.int32).contiguous()
    nb = n_local // B
    global_batch = B * world

    def step(i):
        j = i % nb
        eng.train_step(Xin[j * B:(j + 1) * B], y32[j * B:(j + 1) * B], global_batch)

    # default eager at every N: the three-kernel step is GPU-bound; graph modes measured slower at
    # N = 1 (profiles/r3/bench_graph_modes.md: eager 0.0740-0.0757, whole-step 0.0801, segmented 0.0884,
    # one graph per 8-step cycle 0.0757 ms), and in DP the one flat all-reduce sits between the
    # reduction and Adam kernels
    mode = args.graph if args.graph >= 0 else 0
    graphs = None
    if eng.native and mode == 1:  # whole step (collective included) in one graph per slot
        graphs = capture_steps(step, nb, True)
        run = lambda i: graphs[i % nb].replay()  # noqa: E731
    elif eng.native and mode == 2:
        # segmented: graph(fwd+bwd+slab reduce) -> eager RCCL all-reduce of the flat fp32
        # gradient bucket -> graph(Adam); no collective inside a captured graph
        def grad(i):
            j = i % nb
            eng.grad_phase(Xin[j * B:(j + 1) * B], y32[j * B:(j + 1) * B], global_batch)

        gA = capture_steps(grad, nb, True)
        gB = capture_steps(lambda i: eng.apply_phase(), 1, True)[0]
        graphs = gA + [gB]

        def run(i):
            gA[i % nb].replay()
            eng.comm_phase()
            gB.replay()
            eng.gather_phase()
    else:
        run = step
    # the untimed WISDM accuracy run (a separate engine) goes first: the timed steps then start on a
    # GPU already out of its idle power state instead of ramping its clock inside a 20-step window
    extras = wisdm_accuracy_fields(args, ctx, hidden=(args.hidden, args.hidden))
    settle_ms = settle_clocks(ctx, run, args.settle_ms, dev)
    elapsed = timed(ctx, run, args.steps, args.warmup, dev)
    # accuracy of the model the timed steps trained, before the phase probe's extra steps move it
    Xt, yt = synthetic_windows(65536, seed=999, device=dev)
    acc = float((torch.argmax(eng.logits(Xt), dim=1) == yt).float().mean())
    phases = mlp_phase_times(ctx, eng, Xin, y32, B, nb, global_batch, n=max(10, min(50, args.steps)))
    rec = {"value": global_batch * args.steps / elapsed, "ms_per_step": elapsed * 1e3 / args.steps,
           "vs_baseline": None, "vs_baseline_note": BASELINE_NOTE,
           "data": "synthetic WISDM-shaped windows (43 features, 6 classes, class-conditional Gaussian); "
                   "random-init weights",
           "config": {"model": f"WISDM 6-class 3-layer MLP bf16 ({'-'.join(map(str, layers))})",
                      "global_batch": global_batch, "seq_len": None, "features": N_FEATURES,
                      "parallelism": f"dp{world}"},
           "synthetic_test_accuracy": hdist.mean_over_ranks(ctx, acc),
           "hip_graph": {0: "off", 1: "whole-step", 2: "segmented"}[mode if graphs else 0],
           "collectives_per_step": eng.collective_stats() if hasattr(eng, "collective_stats") else None,
           "phase_ms": phases, "settle_ms": settle_ms}
    rec.update(extras)
    return rec


def mlp_phase_times(ctx, eng, Xin, y32, B, nb, global_batch, n=50):
    """Per-phase time of the DP step, measured AFTER the timed loop on n extra (untimed) steps run
    as the phases of the N > 1 step: compute (forward + backward + slab reduction into the flat fp32
    gradient G), the gradient collective (``allreduce``: the RCCL reduce-scatter of G under the
    sharded optimizer, the all-reduce otherwise), Adam (on this rank's slice when sharded), and
    ``all_gather`` (sharded: the all-gather of P + the bf16 / fragment refresh).  Device time from
    HIP events around each phase on the compute stream (host clock on the CPU path); mean per step,
    max over ranks.  At N = 1 the collectives are absent (reported null, not as the HIP-event floor
    of an empty interval) and the N = 1 step fuses Adam into the reduction kernel, so compute + adam
    there is the split form of the timed step (one extra launch)."""
    from har.parallel import dist as hdist

    cuda = Xin.is_cuda
    tot = {"compute": 0.0, "allreduce": 0.0, "adam": 0.0, "all_gather": 0.0}
    phases = (lambda xb, yb: eng.grad_phase(xb, yb, global_batch), lambda xb, yb: eng.comm_phase(),
              lambda xb, yb: eng.apply_phase(), lambda xb, yb: eng.gather_phase())
    if cuda:
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(n)]
    for i in range(n):
        j = i % nb
        xb, yb = Xin[j * B:(j + 1) * B], y32[j * B:(j + 1) * B]
        if cuda:
            e = ev[i]
            e[0].record()
            for q, ph in enumerate(phases):
                ph(xb, yb)
                e[q + 1].record()
        else:
            t = [time.perf_counter()]
            for ph in phases:
                ph(xb, yb)
                t.append(time.perf_counter())
            for q, k in enumerate(tot):
                tot[k] += (t[q + 1] - t[q]) * 1e3
    if cuda:
        torch.cuda.synchronize()
        for e in ev:
            for q, k in enumerate(tot):
                tot[k] += e[q].elapsed_time(e[q + 1])
    out = {k: hdist.max_over_ranks(ctx, v / n) for k, v in tot.items()}
    # a collective the step does not issue is null, not the HIP-event floor of an empty interval
    # (N = 1 without a forced group: neither; the all-reduce form: no all-gather)
    if not getattr(eng, "dp", False):
        out["allreduce"] = out["all_gather"] = None
    elif not getattr(eng, "sharded", False):
        out["all_gather"] = None
    out.update(steps=n, clock="HIP events" if cuda else "host", world=ctx.world_size)
    return out


def wisdm_accuracy_fields(args, ctx, hidden):
    """Test accuracy of the bench's MLP architecture trained on the real WISDM table (untimed)."""
    from har.suite import wisdm_mlp_accuracy

    if args.no_wisdm:
        return {}
    r = wisdm_mlp_accuracy(ctx.device, args.wisdm, layers_hidden=hidden)
    return {"test_accuracy": r["accuracy"], "test_accuracy_data": "WISDM v1.1 transformed table, "
            f"{r['encoding']}, {r['split']}: {r['n_train']} train / {r['n_test']} test windows; same MLP "
            f"architecture ({'-'.join(map(str, r['layers']))}), {r['epochs']} epochs of batch {r['batch']}, "
            "a separate engine trained before the timed steps (untimed)", "wisdm_mlp_fit_s": r["fit_s"],
            "wisdm_mlp_first_fit_s": r["first_fit_s"]}


def bench_reference(args, ctx):
    """The reference's own four fits (LR, LR-CV, DT, RF) on the real WISDM table."""
    from har.suite import run_reference_suite

    steps, warmup = max(1, args.steps), max(0, args.warmup)
    r = run_reference_suite(ctx.device, args.wisdm, repeats=steps, warmup=warmup, ctx=ctx)
    models = r["models"]
    per_step = r["suite_fit_s"]
    return {"value": r["suite_train_windows_per_s"],
            "ms_per_step": per_step * 1e3, "vs_baseline": r["suite_vs_baseline"],
            "unit_note": "4 x N_train windows / (t_LR + t_LR-CV + t_DT + t_RF); median fit time per model",
            "data": f"WISDM v1.1 transformed table (tests/data/wisdm_data.csv), reference encoding "
                    f"({r['n_features']}-dim one-hot + numeric), 70/30 Philox split seed 2018: "
                    f"{r['n_train']} train / {r['n_test']} test windows",
            "config": {"model": "reference suite: LogisticRegression(maxIter 20, reg 0.3) + CrossValidator(LR 3x3 "
                                "grid, 5 folds, MAE) + DecisionTree(depth 3) + RandomForest(100 trees, depth 4)",
                       "global_batch": r["n_train"], "seq_len": None, "parallelism": f"dp{ctx.world_size}"},
            "dtype": "fp32", "test_accuracy": models["lr"]["accuracy"], "test_accuracy_data": "WISDM test split (LR)",
            "reference_suite": r}


def bench_infer(args, ctx):
    """Serving throughput: the MLP of config 3 (trained ``--train-steps`` steps first, untimed)
    classifies ``--batch`` fp32 feature windows per GPU per step: for the H = 256 network and
    batches that are multiples of 64, one vectorized fp32 -> bf16 cast kernel, then the INFER
    instantiation of the training step's forward (mlp_step.hip mlp_fwd3: logits and argmax out);
    other shapes run the fused forward+head kernel (mlp_fused.hip).  The reference has no measurable inference path
    (its "Prediction made in" timer is lazy-plan time, Main/main.py:121-123)."""
    from har.models.mlp import MLPEngine, pad_input_bf16
    from har.parallel import dist as hdist

    dev, rank, world = ctx.device, ctx.rank, ctx.world_size
    B = args.batch
    layers = [N_FEATURES, args.hidden, args.hidden, N_CLASSES]
    tb = 8192
    eng = MLPEngine(layers, tb, dev, lr=args.lr, seed=1234, process_group=ctx.group, world_size=world)
    Xtr, ytr = synthetic_windows(tb * 8, seed=100 + rank, device=dev)
    Xtr_b = pad_input_bf16(Xtr, eng.layout.in_pad) if eng.native else Xtr
    ytr32 = ytr.to(torch.int32)
    for i in range(args.train_steps):
        j = i % 8
        eng.train_step(Xtr_b[j * tb:(j + 1) * tb], ytr32[j * tb:(j + 1) * tb], tb * world)
    nb = 4
    X, y = synthetic_windows(B * nb, seed=500 + rank, device=dev)
    correct = torch.zeros((), dtype=torch.int64, device=dev)

    def step(i):
        j = i % nb
        xb = X[j * B:(j + 1) * B]
        if eng.native:
            _, pred = eng.infer_fused_f32(xb)  # raw fp32 features in: cast kernel + the step's INFER forward
        else:
            pred = torch.argmax(eng.logits(xb), 1)
        if i < nb:
            correct.add_((pred.long() == y[j * B:(j + 1) * B]).sum())

    settle_ms = settle_clocks(ctx, step, args.settle_ms, dev)
    elapsed = timed(ctx, step, args.steps, args.warmup, dev)
    acc = float(correct) / (B * min(nb, args.steps + args.warmup))
    return {"value": B * world * args.steps / elapsed, "ms_per_step": elapsed * 1e3 / args.steps,
            "vs_baseline": None,
            "data": "synthetic WISDM-shaped windows (43 features, 6 classes); MLP trained "
                    f"{args.train_steps} steps on synthetic windows first (untimed)",
            "config": {"model": f"WISDM 6-class 3-layer MLP bf16 inference ({'-'.join(map(str, layers))})",
                       "global_batch": B * world, "seq_len": None, "features": N_FEATURES,
                       "parallelism": f"dp{world}"},
            "test_accuracy": hdist.mean_over_ranks(ctx, acc), "test_accuracy_data": "held-out synthetic windows",
            "mode": "inference", "settle_ms": settle_ms}


def _featurized(n_windows, spec, dev, first_window):
    from har.data.synth import generate_stream
    from har.features.window import window_features

    s, y = generate_stream(n_windows, spec, dev, first_window=first_window)
    X = window_features(s, spec.window, spec.window, spec.hz)
    return torch.nan_to_num(X, nan=-1.0), y


def bench_rf(args, ctx, nine_axis=False, single_tree=False):
    from har.data.synth import StreamSpec
    from har.models import tree as tree_mod
    from har.models.tree import DecisionTreeClassifier, RandomForestClassifier
    from har.ops import tree as T
    from har.parallel import data_parallel as dp
    from har.parallel import dist as hdist

    dev, rank, world = ctx.device, ctx.rank, ctx.world_size
    K = 12 if nine_axis else N_CLASSES
    spec = StreamSpec(num_classes=K, axes=9 if nine_axis else 3, hz=50.0 if nine_axis else 20.0,
                      window=500 if nine_axis else 200, seed=2018)
    n_local = args.rows
    n_trees = args.trees or (500 if nine_axis else 100)
    # tree parallel (every rank: ALL n_local * N rows, n_trees / N trees, one all-gather) or data
    # parallel (rank's n_local rows, all trees, per-level reduce-scatter + all-gather); "auto" = tree
    # while the replicated table is small (its features fit every GPU many times over here)
    probe = RandomForestClassifier(numTrees=n_trees, parallelism=args.rf_parallel)
    from har.features.window import n_features

    n_feat = n_features(spec.axes) if nine_axis else N_FEATURES
    mode = "data" if single_tree else probe.resolve_parallelism(n_local * world, n_feat, world)
    if mode == "tree":  # the whole table, identical on every rank (windows keyed by global id)
        X, y = _featurized(n_local * world, spec, dev, first_window=0)
    else:
        X, y = _featurized(n_local, spec, dev, first_window=rank * n_local)
    if not nine_axis:
        X = X[:, :N_FEATURES].contiguous()  # the WISDM-43 feature set
    Xt, yt = _featurized(4096, spec, dev, first_window=10 ** 9)
    if not nine_axis:
        Xt = Xt[:, :N_FEATURES].contiguous()
    if single_tree:  # every feature at every node: sibling subtraction applies (--no-subtract: off)
        tree_mod.SIBLING_SUBTRACTION = not args.no_subtract
        tree_mod.SUBTRACT_MIN_PAIRS = 0  # measure the subtraction at every size
        est = DecisionTreeClassifier(maxDepth=args.depth, maxBins=32, device=dev)
    else:
        est = RandomForestClassifier(numTrees=n_trees, maxDepth=args.depth, maxBins=32, seed=7, device=dev,
                                     parallelism=mode)
    model = {}

    owner = dp.NodeOwner(ctx) if (mode == "data" and args.rf_reduce == "owner" and ctx.is_distributed) else None
    tp_stats = {}

    def run(i):
        # the whole fit is timed, findSplits included (sample all-gather + device sort + binning)
        if mode == "tree":
            thr = T.thresholds_for(X, 32, seed=7)  # the whole table is local: no collective
            model["m"] = dp.fit_forest_tree_parallel(est, X, y, K, ctx, thresholds=thr, stats=tp_stats)
            return
        thr = dp.global_thresholds(X, 32, ctx, seed=7)
        model["m"] = est.fit_tensors(X, y, K, allreduce=None if owner else dp.allreduce_sum(ctx),
                                     row_offset=rank * n_local, thresholds=thr, owner=owner)

    settle_ms = settle_clocks(ctx, run, args.settle_ms, dev)
    for st in (tp_stats, owner.stats if owner is not None else {}):  # per-fit collective counts: timed fits only
        for k in st:
            st[k] = 0
    elapsed = timed(ctx, run, args.steps, args.warmup, dev)
    acc = float((model["m"].predict(Xt) == yt).float().mean())
    rows = n_local * world
    if mode == "tree" and world > 1:
        coll = {k: v / (args.steps + args.warmup) for k, v in tp_stats.items()}
    elif owner is not None:
        coll = {k: v / (args.steps + args.warmup) for k, v in owner.stats.items()}
    else:
        coll = None
    if single_tree:
        name = (f"WISDM 6-class DecisionTree depth {args.depth} (all features, sibling subtraction "
                f"{'off' if args.no_subtract else 'on'})")
    elif nine_axis:
        name = f"Synthetic 12-class 9-axis IMU RandomForest {est.numTrees} trees depth {args.depth}"
    else:
        name = f"WISDM 6-class RandomForest {est.numTrees} trees depth {args.depth}"
    return {"value": rows * args.steps / elapsed, "ms_per_step": elapsed * 1e3 / args.steps,
            "vs_baseline": None, "vs_baseline_note": "reference RF is 100 trees x depth 4 on 3793 WISDM rows; "
                                                    "see --config reference",
            "data": f"synthetic {spec.axes}-axis {spec.hz:g} Hz streams featurized on device "
                    f"({X.shape[1]} features, {K} classes)",
            "config": {"model": name, "global_batch": rows, "seq_len": spec.window, "parallelism": f"dp{world}"},
            "test_accuracy": hdist.mean_over_ranks(ctx, acc), "test_accuracy_data": "held-out synthetic windows",
            "dtype": "fp32", "rf_parallel": mode, "settle_ms": settle_ms,
            "histogram_reduction": (args.rf_reduce if mode == "data" else "none (tree parallel)") if world > 1 else "none",
            "collectives_per_step": coll}


def bench_stream(args, ctx):
    from har.data.synth import StreamSpec, generate_stream
    from har.features.window import n_features, window_features, window_features_mlp
    from har.models.mlp import MLPEngine, pad_input_bf16
    from har.parallel import dist as hdist

    dev, rank, world = ctx.device, ctx.rank, ctx.world_size
    spec = StreamSpec(seed=2018)
    W = spec.window
    B = args.batch
    # 1B samples per 8-GPU node: 125M per GPU (weak scaling); --samples-per-gpu N holds N on every GPU
    # (1e9: config 4's whole 1B-sample stream, 12 GB of fp32 x/y/z, resident on ONE MI355X)
    samples_local = args.samples_per_gpu or args.samples // 8
    nw_local = samples_local // W
    stream = torch.empty(nw_local * W, 3, device=dev)
    labels = torch.empty(nw_local, dtype=torch.long, device=dev)
    chunk = 1 << 16
    for c0 in range(0, nw_local, chunk):  # generate the resident shard in chunks
        n = min(chunk, nw_local - c0)
        s, yl = generate_stream(n, spec, dev, first_window=rank * nw_local + c0)
        stream[c0 * W:(c0 + n) * W] = s
        labels[c0:c0 + n] = yl
    F = n_features(3)
    eng = MLPEngine([F, args.hidden, args.hidden, N_CLASSES], B, dev, lr=args.lr, seed=1234,
                    process_group=ctx.group, world_size=world)
    feat = torch.empty(B, F, device=dev)
    nb = nw_local // B
    y32 = labels.to(torch.int32)
    global_batch = B * world
    # feature standardization (Spark StandardScaler analogue): moments of a 16k-window sample of
    # every rank's shard, summed across ranks (untimed setup; HIP column-stats kernel on the GPU)
    from har.ops.stats import column_stats

    ns = min(nw_local, 16384)
    st = column_stats(torch.nan_to_num(window_features(stream[:ns * W], W, W, spec.hz), nan=-1.0))[:3].contiguous()
    if world > 1:
        from har.parallel import comm
        comm.all_reduce(st, group=ctx.group)
    mean = (st[1] / st[0]).float()
    var = (st[2] / st[0]).float() - mean * mean
    inv_std = torch.where(var > 1e-12, var.clamp_min(1e-12).rsqrt(), torch.ones_like(var))

    def featurize(s):
        X = torch.nan_to_num(window_features(s, W, W, spec.hz), nan=-1.0)
        return (X - mean) * inv_std

    xin = torch.empty(B, eng.layout.in_pad, dtype=torch.bfloat16, device=dev) if eng.native else None

    def step(i):
        j = i % nb
        s = stream[j * B * W:(j + 1) * B * W]
        if eng.native:  # one kernel: featurize + NaN fill + standardize + bf16 + pad
            window_features_mlp(s, W, W, spec.hz, mean, inv_std, eng.layout.in_pad, -1.0, out=xin)
            eng.train_step(xin, y32[j * B:(j + 1) * B], global_batch)
        else:
            feat.copy_(featurize(s))
            eng.train_step(pad_input_bf16(feat, eng.layout.in_pad), y32[j * B:(j + 1) * B], global_batch)

    if eng.native and args.stream_overlap:
        # software pipeline: step i trains on batch i (featurized during step i - 1) while a side
        # stream featurizes batch i + 1 into the other buffer (events order the buffer reuse), so the
        # memory-bound featurizer runs beside the MLP kernels instead of between them.  A timed window
        # of K steps still featurizes K batches and trains K batches.
        xb = [torch.empty_like(xin), torch.empty_like(xin)]
        fstream = torch.cuda.Stream(device=dev)
        ready = [torch.cuda.Event(), torch.cuda.Event()]
        consumed = [torch.cuda.Event(), torch.cuda.Event()]
        pending = {"i": None}

        def featurize_into(i):
            j, buf = i % nb, i % 2
            fstream.wait_event(consumed[buf])  # the train step that read this buffer has run
            with torch.cuda.stream(fstream):
                window_features_mlp(stream[j * B * W:(j + 1) * B * W], W, W, spec.hz, mean, inv_std,
                                    eng.layout.in_pad, -1.0, out=xb[buf])
                ready[buf].record(fstream)

        def step(i):  # noqa: F811
            if pending["i"] != i:  # not prefetched (the first step, or a jump in the step index)
                featurize_into(i)
            featurize_into(i + 1)
            pending["i"] = i + 1
            cur = torch.cuda.current_stream()
            cur.wait_event(ready[i % 2])
            j = i % nb
            eng.train_step(xb[i % 2], y32[j * B:(j + 1) * B], global_batch)
            consumed[i % 2].record(cur)

    def held_out_accuracy():
        # 8192 windows of the stream beyond every rank's shard, featurized the same way
        st_, yt = generate_stream(8192, spec, dev, first_window=10 ** 9)
        return hdist.mean_over_ranks(ctx, float((torch.argmax(eng.logits(featurize(st_)), 1) == yt).float().mean()))

    if args.stream_pass:
        rec = _stream_full_pass(args, ctx, spec, stream, labels, eng, mean, inv_std, samples_local)
        rec.update(test_accuracy=held_out_accuracy(),
                   test_accuracy_data="held-out synthetic stream (8192 windows past every shard), after the timed passes")
        return rec
    settle_ms = settle_clocks(ctx, step, args.settle_ms, dev)
    elapsed = timed(ctx, step, args.steps, args.warmup, dev)
    acc = held_out_accuracy()
    return {"value": global_batch * args.steps / elapsed, "ms_per_step": elapsed * 1e3 / args.steps,
            "vs_baseline": None, "vs_baseline_note": BASELINE_NOTE,
            "samples_per_s": global_batch * W * args.steps / elapsed,
            "data": f"synthetic 3-axis 20 Hz stream, {samples_local * world / 1e9:.2f}B samples resident "
                    f"({samples_local / 1e6:.0f}M per GPU), featurized + standardized on device each step",
            "config": {"model": f"raw stream -> window features ({F}) -> MLP bf16 "
                                f"({F}-{args.hidden}-{args.hidden}-{N_CLASSES})",
                       "global_batch": global_batch, "seq_len": W, "parallelism": f"dp{world}"},
            "test_accuracy": acc, "test_accuracy_data": "held-out synthetic stream", "settle_ms": settle_ms,
            "stream_overlap": bool(eng.native and args.stream_overlap)}


def _stream_full_pass(args, ctx, spec, stream, labels, eng, mean, inv_std, samples_local):
    """``--config stream --stream-pass``: one timed step = one FULL pass over every resident
    sample (1B per 8 GPUs): the rank's shard is featurized with 50%-overlapping windows — windows
    that straddle a shard cut take the right neighbour's first W-1 samples by one point-to-point
    halo exchange (parallel/stream.py) — straight into standardized bf16 MLP rows (window kernel
    MLP-input mode), then the MLP trains one epoch over them (every rank the same step count)."""
    import torch.distributed as tdist

    from har.features.window import WindowFeaturizer, n_features, window_features, window_features_mlp
    from har.models.mlp import pad_input_bf16
    from har.parallel import comm
    from har.parallel.stream import shard_offsets, sharded_window_features

    dev, world, B, W = ctx.device, ctx.world_size, args.batch, spec.window
    fz = WindowFeaturizer(hz=spec.hz, seconds=W / spec.hz, overlap=0.5)
    offset, total = shard_offsets(ctx, stream.shape[0], dev)
    xin_rows = {}

    def inputs(seg):
        if eng.native:  # one kernel: featurize + NaN fill + standardize + bf16 + pad
            return window_features_mlp(seg, fz.window, fz.stride, spec.hz, mean, inv_std, eng.layout.in_pad, -1.0)
        X = torch.nan_to_num(window_features(seg, fz.window, fz.stride, spec.hz), nan=-1.0)
        return pad_input_bf16((X - mean) * inv_std, eng.layout.in_pad)

    X0, _ = sharded_window_features(ctx, stream, fz, offset, total, transform=inputs)  # untimed: the owned count
    nbt = torch.tensor([X0.shape[0] // B], device=dev)
    del X0
    if world > 1:
        comm.all_reduce(nbt, op=tdist.ReduceOp.MIN, group=ctx.group)
    nb = int(nbt.item())  # MLP steps per pass (the same on every rank)
    gb = B * world

    def one_pass(i):
        X, first_w = sharded_window_features(ctx, stream, fz, offset, total, transform=inputs)
        xin_rows["n"] = X.shape[0]
        # window j starts at j * stride; its label is that of the generated segment it starts in (the
        # same windows every pass: the int32 label vector is built by the first (warm-up) pass only)
        y32 = xin_rows.get(("y", first_w))
        if y32 is None:
            lab = labels[(torch.arange(first_w, first_w + nb * B, device=dev) * fz.stride) // W - offset // W]
            y32 = xin_rows[("y", first_w)] = lab.to(torch.int32)
        for j in range(nb):
            # (the next batch's rows touched by this step's reduction launch: the epoch's 1.3 GB of rows
            # are not cache-resident, profiles/r6/mlp_cold_x_probe.txt)
            nxt = (X[(j + 1) * B:(j + 2) * B], y32[(j + 1) * B:(j + 2) * B]) if j + 1 < nb and eng.native else None
            eng.train_step(X[j * B:(j + 1) * B], y32[j * B:(j + 1) * B], gb, prefetch=nxt)

    settle_ms = settle_clocks(ctx, one_pass, args.settle_ms, dev)
    elapsed = timed(ctx, one_pass, args.steps, args.warmup, dev)
    trained = nb * gb
    return {"value": trained * args.steps / elapsed, "ms_per_step": elapsed * 1e3 / args.steps,
            "vs_baseline": None, "vs_baseline_note": BASELINE_NOTE,
            "samples_per_s": samples_local * world * args.steps / elapsed,
            "windows_featurized_per_pass": xin_rows.get("n", 0) * world, "mlp_steps_per_pass": nb,
            "data": f"synthetic 3-axis {spec.hz:g} Hz stream, {samples_local * world / 1e9:.2f}B samples resident "
                    f"({samples_local / 1e6:.0f}M per GPU); one step = one full pass: sharded featurization with "
                    f"{fz.window}-sample windows at stride {fz.stride} (halo exchange between ranks) + one MLP epoch",
            "config": {"model": f"raw stream full pass -> window features -> MLP bf16 "
                                f"({n_features(3)}-{args.hidden}-{args.hidden}-{N_CLASSES})",
                       "global_batch": gb, "seq_len": fz.window, "parallelism": f"dp{world}"},
            "samples_per_gpu": samples_local, "settle_ms": settle_ms}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="mlp", choices=["mlp", "rf", "stream", "rf9", "infer", "reference", "dt"])
    ap.add_argument("--wisdm", default=DEFAULT_WISDM, help="WISDM transformed CSV (accuracy / reference suite)")
    ap.add_argument("--no-wisdm", action="store_true", help="skip the WISDM accuracy / reference-suite extras")
    ap.add_argument("--train-steps", type=int, default=200, help="untimed MLP training steps before --config infer")
    ap.add_argument("--batch", type=int, default=65536, help="windows per GPU per step (MLP configs)")
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--graph", type=int, default=-1,
                    help="HIP graphs for the MLP step: 0 eager (default; in DP one flat all-reduce per step between "
                         "the reduction and Adam kernels), 1 whole step in one graph per batch slot, 2 graphs around "
                         "an eager RCCL all-reduce")
    ap.add_argument("--rows", type=int, default=60000, help="windows per GPU (forest configs)")
    ap.add_argument("--trees", type=int, default=0)
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--no-subtract", action="store_true", help="--config dt: histogram every node directly")
    ap.add_argument("--rf-reduce", default="owner", choices=["owner", "allreduce"],
                    help="DP forest histograms: reduce-scatter by node owner + all-gather of splits, or all-reduce")
    ap.add_argument("--rf-parallel", default="auto", choices=["auto", "data", "tree"],
                    help="forest configs over N GPUs: tree = every rank holds all N x --rows windows and grows "
                         "numTrees / N trees (one all-gather per fit); data = row shards with per-level histogram "
                         "reductions; auto = tree while the replicated table is small")
    ap.add_argument("--samples", type=int, default=1_000_000_000, help="stream samples per 8 GPUs")
    ap.add_argument("--samples-per-gpu", type=int, default=0,
                    help="--config stream: samples resident on EVERY GPU (overrides --samples / 8)")
    ap.add_argument("--stream-pass", action="store_true",
                    help="--config stream: time full passes over every resident sample (halo-sharded featurization "
                         "+ one MLP epoch) instead of per-batch steps")
    ap.add_argument("--out", type=str, default="")
    ap.add_argument("--stream-overlap", type=int, default=int(os.environ.get("HAR_STREAM_OVERLAP", "0")),
                    help="--config stream: featurize batch i+1 on a side stream while batch i trains (1) or "
                         "featurize then train in one stream (0)")
    ap.add_argument("--settle-ms", type=float, default=float(os.environ.get("HAR_BENCH_SETTLE_MS", "200")),
                    help="MLP configs: untimed training steps for this long before the warm-up (clock settle)")
    args = ap.parse_args()

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from har.parallel import dist as hdist

    ctx = hdist.init(expected_world=args.gpus)
    if args.config == "mlp":
        r = bench_mlp(args, ctx)
    elif args.config == "stream":
        r = bench_stream(args, ctx)
    elif args.config == "infer":
        r = bench_infer(args, ctx)
    elif args.config == "reference":
        r = bench_reference(args, ctx)
    else:
        r = bench_rf(args, ctx, nine_axis=args.config == "rf9", single_tree=args.config == "dt")
    rec = {"metric": METRIC, "value": r.pop("value"), "unit": "windows/s", "n_gpus": ctx.world_size,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": r.pop("ms_per_step"),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": r.pop("vs_baseline"),
           "dtype": r.pop("dtype", "bf16"), "data": r.pop("data"), "config": r.pop("config")}
    rec.update(r)
    if args.config == "mlp" and ctx.world_size == 1 and not args.no_wisdm:
        # same-model comparison against the reference's published fits, recorded with the headline run
        from har.suite import run_reference_suite

        rec["reference_suite"] = run_reference_suite(ctx.device, args.wisdm, repeats=3, warmup=1)
    rec["bench_config"] = args.config
    rec["dist_backend"] = ctx.backend  # None: one process, no group; "nccl" = RCCL
    if ctx.forced:
        rec["dist_forced_group"] = True  # HAR_DIST_FORCE_PG=1: a 1-rank RCCL group carried the DP collectives
    rec["device"] = torch.cuda.get_device_name(ctx.device) if ctx.device.type == "cuda" else "cpu"
    if ctx.rank == 0:
        line = json.dumps(rec)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    hdist.shutdown(ctx)


if __name__ == "__main__":
    main()
