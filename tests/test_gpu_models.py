"""GPU model paths (HIP kernels) vs the CPU oracles of the same algorithms."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _blobs(n=3000, f=20, k=6, seed=0):
    g = torch.Generator().manual_seed(seed)
    mu = torch.randn(k, f, generator=g) * 1.5
    y = torch.randint(0, k, (n,), generator=g)
    x = mu[y] + torch.randn(n, f, generator=g)
    return x, y


def test_philox_buckets_device_matches_host(cuda):
    from har.ops import rng

    n = 100_003
    host = rng.assign_buckets(2018, rng.STREAM_SPLIT, np.arange(5, 5 + n, dtype=np.uint64), [0.7, 0.3])
    dev = rng.device_buckets(2018, rng.STREAM_SPLIT, 5, n, [0.7, 0.3], cuda).cpu().numpy()
    assert np.array_equal(host, dev)


@pytest.mark.parametrize("n,k,seed", [(3853, 3, 2018), (3853, 5, 2018), (100_003, 5, 7), (17, 3, 1)])
def test_kfold_ids_device_matches_host(cuda, n, k, seed):
    """CrossValidator's device fold ids (rng.device_buckets on STREAM_KFOLD, equal weights) are the host
    kfold_ids bit for bit — GPU and CPU cross-validation score the same folds."""
    from har.data.split import kfold_ids
    from har.ops import rng

    dev = rng.device_buckets(seed, rng.STREAM_KFOLD, 0, n, [1.0] * k, cuda).cpu().numpy()
    assert np.array_equal(kfold_ids(n, k, seed), dev)


def test_poisson_device_matches_host(cuda):
    from har.ops import rng

    host = rng.poisson1_weights(7, range(3, 8), 20_000, row_offset=11)
    dev = rng.device_poisson1(7, 3, 5, 11, 20_000, cuda).cpu().numpy()
    assert np.array_equal(host, dev)
    assert abs(dev.mean() - 1.0) < 0.02


def test_hist_split_native_matches_torch(cuda):
    from har.ops import rng
    from har.ops import tree as T

    x, y = _blobs(2000, 30, 5)
    thr = T.find_thresholds(x.numpy(), 32)
    bins = torch.from_numpy(T.bin_features(x.numpy(), thr)).to(cuda)
    nbins = torch.tensor([len(t) + 1 for t in thr], dtype=torch.int32, device=cuda)
    # 3 nodes with overlapping random row subsets and weights
    g = torch.Generator().manual_seed(1)
    keys, rows = [], []
    for a in range(3):
        r = torch.randperm(2000, generator=g)[: 500 + 300 * a].sort().values
        rows.append(r)
        keys.append(torch.full_like(r, a))
    rows = torch.cat(rows).to(torch.int32).to(cuda)
    keys = torch.cat(keys).to(cuda)
    w = torch.randint(1, 3, (rows.numel(),), generator=g).float().to(cuda)
    counts = torch.bincount(keys, minlength=3).to(torch.int32)
    starts = (torch.cumsum(counts, 0) - counts).to(torch.int32)
    feats = torch.from_numpy(rng.feature_subsets(3, [0, 0, 1], [0, 1, 0], 30, 12)).to(cuda)
    y32 = y.to(torch.int32).to(cuda)
    nat = T.hist_split_native(bins, nbins, y32, rows, w, starts, counts, feats, 5, 32, 1.0, 0.0, T.GINI)
    ref = T.hist_split_torch(bins, nbins, y32, rows, w, keys, 3, feats, 5, 32, 1.0, 0.0, T.GINI)
    torch.testing.assert_close(nat.total, ref.total)
    torch.testing.assert_close(nat.gain, ref.gain, rtol=1e-5, atol=1e-6)
    assert torch.equal(nat.feat, ref.feat) and torch.equal(nat.bin, ref.bin)
    torch.testing.assert_close(nat.left, ref.left)
    # data-parallel form: histogram-only pass, (identity) all-reduce, split pass == fused kernel
    two = T.hist_split_native(bins, nbins, y32, rows, w, starts, counts, feats, 5, 32, 1.0, 0.0, T.GINI,
                              allreduce=lambda t: None)
    assert torch.equal(two.feat, nat.feat) and torch.equal(two.bin, nat.bin)
    torch.testing.assert_close(two.gain, nat.gain)
    torch.testing.assert_close(two.total, nat.total)

    # owner-computes form: this "rank" owns node slice [a0, a1); the split kernel runs on that
    # slice only (pointer-offset node / feature arrays) and the gathered rows must equal the
    # fused kernel's; the other rows stay zero (another rank's share)
    class SliceOwner:
        def __init__(self, a0, a1):
            self.a0, self.a1 = a0, a1

        def reduce_scatter(self, hist):
            return hist[self.a0:self.a1].clone(), self.a0, self.a1

        def all_gather(self, local, A):
            out = torch.zeros(A, *local.shape[1:], dtype=local.dtype, device=local.device)
            out[self.a0:self.a1] = local
            return out

    for a0, a1 in ((1, 3), (0, 1), (2, 3)):
        own = T.hist_split_native(bins, nbins, y32, rows, w, starts, counts, feats, 5, 32, 1.0, 0.0, T.GINI,
                                  owner=SliceOwner(a0, a1))
        assert torch.equal(own.feat[a0:a1], nat.feat[a0:a1]) and torch.equal(own.bin[a0:a1], nat.bin[a0:a1])
        torch.testing.assert_close(own.gain[a0:a1], nat.gain[a0:a1])
        torch.testing.assert_close(own.left[a0:a1], nat.left[a0:a1])
        torch.testing.assert_close(own.total[a0:a1], nat.total[a0:a1])


def test_forest_predict_native_matches_torch(cuda):
    from har.models.tree import RandomForestClassifier
    from har.ops import tree as T

    x, y = _blobs(1500, 16, 4, seed=2)
    m = RandomForestClassifier(numTrees=20, maxDepth=6, seed=3, device="cpu").fit_tensors(x, y, 4)
    a = m.arrs
    ref = T.forest_predict_torch(x, a.feature, a.threshold, a.left, a.right, a.stats, a.max_depth, True)
    ac = a.to(cuda)
    nat = T.forest_predict_native(x.to(cuda), ac.feature, ac.threshold, ac.left, ac.right, ac.stats, ac.max_depth,
                                  True)
    torch.testing.assert_close(nat.cpu(), ref, rtol=1e-5, atol=1e-5)


def test_decision_tree_gpu_equals_cpu(cuda):
    from har.models.tree import DecisionTreeClassifier

    x, y = _blobs(2500, 12, 6, seed=4)
    cpu = DecisionTreeClassifier(maxDepth=5, device="cpu").fit_tensors(x, y, 6)
    gpu = DecisionTreeClassifier(maxDepth=5, device=cuda).fit_tensors(x.to(cuda), y.to(cuda), 6)
    assert cpu.numNodes == gpu.numNodes
    assert torch.equal(cpu.arrs.feature, gpu.arrs.feature.cpu())
    assert torch.equal(cpu.predict(x), gpu.predict(x.to(cuda)).cpu())


def test_random_forest_gpu_accuracy(cuda):
    from har.models.tree import RandomForestClassifier

    xa, ya = _blobs(6000, 20, 6, seed=5)
    x, y, xt, yt = xa[:4000], ya[:4000], xa[4000:], ya[4000:]
    gpu = RandomForestClassifier(numTrees=50, maxDepth=8, seed=1, device=cuda).fit_tensors(x.to(cuda), y.to(cuda), 6)
    cpu = RandomForestClassifier(numTrees=50, maxDepth=8, seed=1, device="cpu").fit_tensors(x, y, 6)
    acc_g = float((gpu.predict(xt.to(cuda)).cpu() == yt).float().mean())
    acc_c = float((cpu.predict(xt) == yt).float().mean())
    assert acc_g > 0.8 and abs(acc_g - acc_c) < 0.03


def test_logreg_gpu_matches_cpu(cuda):
    from har.models.logreg import FitSpec, LogisticRegression

    x, y = _blobs(3000, 24, 6, seed=7)
    est = LogisticRegression(maxIter=50, regParam=0.1)
    specs = [FitSpec(None, 0.1, 0.0), FitSpec(None, 0.1, 0.5)]
    cpu = est.fit_many(x, y, specs, 6)
    gpu = est.fit_many(x.to(cuda), y.to(cuda), specs, 6)
    for c, g in zip(cpu, gpu):
        assert abs(c.summary["objective"] - g.summary["objective"]) < 1e-3
        agree = (c.predict(x) == g.predict(x.to(cuda)).cpu()).float().mean()
        assert agree > 0.99


def test_naive_bayes_gpu_matches_cpu(cuda):
    from har.models.naive_bayes import NaiveBayes

    x, y = _blobs(2000, 10, 4, seed=8)
    for mt, xx in (("gaussian", x), ("multinomial", x.abs())):
        c = NaiveBayes(modelType=mt).fit_tensors(xx, y, 4)
        g = NaiveBayes(modelType=mt).fit_tensors(xx.to(cuda), y.to(cuda), 4)
        torch.testing.assert_close(g.predict_raw(xx.to(cuda)).cpu(), c.predict_raw(xx), rtol=1e-4, atol=1e-3)


def test_naive_bayes_gpu_bitwise_deterministic(cuda):
    """NB class moments reduce split-K slabs in a fixed order (no float atomics): two fits of the
    same data give bit-identical parameters."""
    from har.models.naive_bayes import NaiveBayes

    x, y = _blobs(20000, 24, 5, seed=9)
    xg, yg = x.to(cuda), y.to(cuda)
    for mt, xx in (("gaussian", xg), ("multinomial", xg.abs())):
        a = NaiveBayes(modelType=mt).fit_tensors(xx, yg, 5)
        b = NaiveBayes(modelType=mt).fit_tensors(xx, yg, 5)
        assert torch.equal(a.theta, b.theta) and torch.equal(a.pi, b.pi)
        if a.sigma is not None:
            assert torch.equal(a.sigma, b.sigma)


def test_main_reference_run_gpu(cuda, tmp_path, wisdm_csv):
    import main

    s = main.run(main.config_from_args(["--data", wisdm_csv, "--out-dir", str(tmp_path), "--classifiers",
                                        "lr,lrcv,dt,rf", "--device", "cuda"]))
    m = s["models"]
    assert m["lr"]["accuracy"] >= 0.60 and m["lrcv"]["accuracy"] >= 0.70
    assert m["dt"]["accuracy"] >= 0.72 and m["rf"]["accuracy"] >= 0.62
    assert (tmp_path / "result.txt").exists() and (tmp_path / "additional_param.csv").exists()


def test_main_csv_device_matches_host_parse(cuda, tmp_path, wisdm_csv):
    """``main.py --csv-device``: the CSV is parsed and dictionary-encoded by the HIP kernels;
    the run must reproduce the host-parsed run's metrics exactly."""
    import main

    base = ["--data", wisdm_csv, "--classifiers", "lr,dt", "--device", "cuda"]
    a = main.run(main.config_from_args(base + ["--out-dir", str(tmp_path / "host")]))
    b = main.run(main.config_from_args(base + ["--out-dir", str(tmp_path / "dev"), "--csv-device"]))
    for name in ("lr", "dt"):
        assert a["models"][name]["accuracy"] == b["models"][name]["accuracy"]
        assert a["models"][name]["f1"] == b["models"][name]["f1"]


def test_dictionary_encode_device(cuda, wisdm_csv):
    from har.data.csv_device import read_csv_device
    from har.features.encode import StringIndexer
    from har.data.csv_io import read_csv

    d = read_csv_device(wisdm_csv, cuda)
    codes, vocab, counts = d.dictionary_encode("ACTIVITY")
    assert vocab == ["Walking", "Jogging", "Upstairs", "Downstairs", "Sitting", "Standing"]
    assert counts.tolist() == [2081, 1625, 632, 528, 306, 246]
    host = read_csv(wisdm_csv)
    sm = StringIndexer(inputCol="XPEAK", outputCol="i").fit(host)
    c2, v2, _ = d.dictionary_encode("XPEAK")
    assert v2 == list(sm.labels) and len(v2) == 935  # "?" included; frequency-desc, ties by value
    assert int(codes.min()) == 0 and codes.device.type == "cuda"


@pytest.mark.parametrize("F,m", [(165, 13), (3100, 56), (43, 7), (20, 20)])
def test_feature_subsets_device_matches_host(cuda, F, m):
    """tree_level.hip Floyd sampler == har.ops.rng.feature_subsets (the CPU oracle), bit for bit."""
    from har.ops import _native
    from har.ops import rng

    g = np.random.default_rng(F)
    trees = g.integers(0, 600, 5000)
    nodes = g.integers(0, 2047, 5000)
    host = rng.feature_subsets(7, trees, nodes, F, m)
    out = torch.empty(5000, m, dtype=torch.int32, device=cuda)
    tr = torch.as_tensor(trees, dtype=torch.int32, device=cuda)
    nd = torch.as_tensor(nodes, dtype=torch.int32, device=cuda)
    _native.kernels().tree_feature_subsets(7, tr.data_ptr(), nd.data_ptr(), 5000, F, m, out.data_ptr(), 0,
                                           _native.stream_ptr())
    assert np.array_equal(out.cpu().numpy(), host)


def test_random_forest_gpu_equals_cpu_builder(cuda):
    """The device level loop (HIP keys / partition / feature subsets) grows the forest of the
    CPU builder (PyTorch oracle) on integer-weighted bootstraps: identical top levels; deeper,
    a near-tie between two candidate splits may resolve differently (fp64 gains summed in a
    different order), so the forests' predictions are compared there."""
    from har.models.tree import RandomForestClassifier
    from har.ops import tree as T

    x, y = _blobs(3000, 24, 5, seed=3)
    thr = T.find_thresholds(x.numpy(), 32)
    c = RandomForestClassifier(numTrees=12, maxDepth=6, seed=4).fit_tensors(x, y, 5, thresholds=thr)
    g = RandomForestClassifier(numTrees=12, maxDepth=6, seed=4).fit_tensors(x.to(cuda), y.to(cuda), 5,
                                                                            thresholds=thr)
    assert torch.equal(g.arrs.feature[:, :7].cpu(), c.arrs.feature[:, :7])  # depth 0-2 of every tree
    torch.testing.assert_close(g.arrs.stats[:, :7].cpu(), c.arrs.stats[:, :7])
    same_node = float((g.arrs.feature.cpu() == c.arrs.feature).float().mean())
    agree = float((g.predict(x.to(cuda)).cpu() == c.predict(x)).float().mean())
    assert same_node > 0.97 and agree > 0.99, (same_node, agree)


def test_level_grouping_equals_sort_path(cuda, monkeypatch):
    """tree_level_group (counting sort: per-chunk counts, prefix, wave-stable scatter) feeds the
    histogram kernel the rows in exactly the order of the stable radix sort of the level keys, so
    the two device builders grow bit-identical forests (N not a multiple of the 1024-row chunk,
    deep trees so late levels have thousands of candidates)."""
    from har.models import tree as tree_mod
    from har.models.tree import RandomForestClassifier

    x, y = _blobs(5300, 16, 6, seed=7)
    xc, yc = x.to(cuda), y.to(cuda)
    fits = {}
    for force_sort in (True, False):
        monkeypatch.setattr(tree_mod, "FORCE_SORT_GROUPING", force_sort)
        fits[force_sort] = RandomForestClassifier(numTrees=40, maxDepth=12, seed=11).fit_tensors(xc, yc, 6)
    a, b = fits[True].arrs, fits[False].arrs
    for name in ("feature", "threshold", "left", "right", "stats"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    # the commit kernel sums the node weight sequentially, torch.sum may pair it differently
    torch.testing.assert_close(a.gain, b.gain)


def test_planned_levels_equal_node_blocks(cuda, monkeypatch):
    """Row-balanced levels (big nodes split into 2048-row chunk items whose LDS histograms merge
    into a slot, then a split pass over the merged nodes) grow bit-identically the forest of one
    workgroup per node: integer-valued weights make the merged histograms exact."""
    from har.models import tree as tree_mod
    from har.models.tree import RandomForestClassifier

    x, y = _blobs(9000, 20, 6, seed=9)
    xc, yc = x.to(cuda), y.to(cuda)
    fits = {}
    for node_blocks in (True, False):
        monkeypatch.setattr(tree_mod, "FORCE_NODE_BLOCKS", node_blocks)
        fits[node_blocks] = RandomForestClassifier(numTrees=30, maxDepth=9, seed=3).fit_tensors(xc, yc, 6)
    a, b = fits[True].arrs, fits[False].arrs
    for name in ("feature", "threshold", "left", "right", "stats", "gain"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name


@pytest.mark.parametrize("kind,depth", [("rf", 14), ("rf", 6), ("dt", 8)])
def test_device_count_levels_equal_synced_levels(cuda, monkeypatch, kind, depth):
    """Levels enqueued on device-side counts (grids / arrays sized by bounds, no D2H until the
    fit ends) grow the forest of levels that read their counts back every level, node for node.
    Depth 14 crosses the grouping's per-tree bound, so that fit switches to a synced level
    mid-way and back; the DT case samples every feature (m = F) with entropy."""
    from har.models import tree as tree_mod
    from har.models.tree import DecisionTreeClassifier, RandomForestClassifier

    x, y = _blobs(7000, 18, 6, seed=21)
    xc, yc = x.to(cuda), y.to(cuda)
    fits = {}
    for sync in (True, False):
        monkeypatch.setattr(tree_mod, "FORCE_LEVEL_SYNC", sync)
        if kind == "rf":
            est = RandomForestClassifier(numTrees=24, maxDepth=depth, seed=5)
        else:
            est = DecisionTreeClassifier(maxDepth=depth, impurity="entropy")
        fits[sync] = est.fit_tensors(xc, yc, 6)
    a, b = fits[True].arrs, fits[False].arrs
    assert np.array_equal(np.asarray(a.n_nodes), np.asarray(b.n_nodes))
    for name in ("feature", "threshold", "left", "right", "stats", "gain"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name


@pytest.mark.parametrize("kind", ["rf", "dt_sub"])
def test_fit_graph_replays_equal_eager_fits(cuda, monkeypatch, kind):
    """A fit signature seen twice is captured as ONE HIP graph (tree_init, device root frontier,
    every level) and replayed with new inputs copied into its static buffers: each replay grows
    exactly the forest an eager fit of the same data grows (two data sets, alternating)."""
    from har.models import tree as tree_mod
    from har.models.tree import DecisionTreeClassifier, RandomForestClassifier

    monkeypatch.setattr(tree_mod, "_fit_graphs", {})
    monkeypatch.setattr(tree_mod, "_fit_graph_seen", {})
    monkeypatch.setattr(tree_mod, "SUBTRACT_MIN_PAIRS", 0)
    data = [_blobs(6000, 20, 6, seed=s) for s in (41, 42)]
    data = [(x.to(cuda), y.to(cuda)) for x, y in data]

    def fit(x, y):
        if kind == "rf":
            return RandomForestClassifier(numTrees=16, maxDepth=8, seed=9).fit_tensors(x, y, 6).arrs
        return DecisionTreeClassifier(maxDepth=9).fit_tensors(x, y, 6).arrs

    monkeypatch.setattr(tree_mod, "FIT_GRAPHS", False)
    eager = [fit(*d) for d in data]
    monkeypatch.setattr(tree_mod, "FIT_GRAPHS", True)
    order = [0, 1, 0, 1]  # eager (first sighting), capture + replay, replay, replay
    got = [fit(*data[i]) for i in order]
    assert len(tree_mod._fit_graphs) == 1
    for i, a in zip(order, got):
        b = eager[i]
        assert np.array_equal(np.asarray(a.n_nodes), np.asarray(b.n_nodes))
        for name in ("feature", "threshold", "left", "right", "stats", "gain"):
            assert torch.equal(getattr(a, name), getattr(b, name)), (i, name)


@pytest.mark.parametrize("kind,F", [("dt", 24), ("dt", 200), ("rf_all", 30)])
def test_sibling_subtraction_equals_direct_histograms(cuda, monkeypatch, kind, F):
    """Trees that search every feature keep each level's node histograms and take the heavier
    sibling's as parent - lighter sibling (its rows skip the grouping and histogram passes); with
    integer-valued weights the subtraction is exact, so the forest equals the one built from
    direct histograms, bit for bit.  F = 200 splits the features over two LDS chunks; 9000 rows
    make the top nodes 2048-row chunked (merged) work items."""
    from har.models import tree as tree_mod
    from har.models.tree import DecisionTreeClassifier, RandomForestClassifier

    x, y = _blobs(9000, F, 6, seed=31)
    xc, yc = x.to(cuda), y.to(cuda)
    fits = {}
    monkeypatch.setattr(tree_mod, "SUBTRACT_MIN_PAIRS", 0)
    for sub in (False, True):
        monkeypatch.setattr(tree_mod, "SIBLING_SUBTRACTION", sub)
        if kind == "dt":
            est = DecisionTreeClassifier(maxDepth=9)
        else:
            est = RandomForestClassifier(numTrees=6, maxDepth=8, featureSubsetStrategy="all", seed=2)
        fits[sub] = est.fit_tensors(xc, yc, 6)
    a, b = fits[False].arrs, fits[True].arrs
    assert np.array_equal(np.asarray(a.n_nodes), np.asarray(b.n_nodes))
    for name in ("feature", "threshold", "left", "right", "stats", "gain"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name


@pytest.mark.parametrize("trees,rate", [(12, 0.6), (1, 0.4)])
def test_subsampled_forest_gpu_equals_cpu(cuda, trees, rate):
    """subsamplingRate on the device (tree_init: Poisson(rate) / Bernoulli(rate) from the CDF table)
    draws the host oracle's weights: identical root counts and top levels."""
    from har.models.tree import RandomForestClassifier
    from har.ops import tree as T

    x, y = _blobs(3000, 16, 5, seed=8)
    thr = T.find_thresholds(x.numpy(), 32)
    kw = dict(numTrees=trees, maxDepth=5, seed=6, subsamplingRate=rate)
    c = RandomForestClassifier(**kw).fit_tensors(x, y, 5, thresholds=thr)
    g = RandomForestClassifier(**kw).fit_tensors(x.to(cuda), y.to(cuda), 5, thresholds=thr)
    torch.testing.assert_close(g.arrs.stats[:, 0].cpu(), c.arrs.stats[:, 0], rtol=0, atol=0)
    assert torch.equal(g.arrs.feature[:, :3].cpu(), c.arrs.feature[:, :3])


@pytest.mark.parametrize("B,H", [(256, 256), (320, 256), (256, 128), (144, 128)])
def test_mlp_epoch_graph_equals_eager_fit(cuda, monkeypatch, B, H):
    """A single-GPU MultilayerPerceptronClassifier fit replays one captured HIP graph per epoch
    (static batch buffers, the shuffled rows gathered into them); it must train exactly the
    parameters of the eager step loop.  B = 256 / 320: the small batches main.py and the bench's
    WISDM accuracy run use (more backward slices than 4-tile slices would give); H = 128: main.py's
    43-128-128-6 on the fused forward + split-K backward (B = 144: not a multiple of 64)."""
    from har.models.mlp import MultilayerPerceptronClassifier

    g = torch.Generator().manual_seed(9)
    X = torch.randn(2500, 43, generator=g).to(cuda)
    y = torch.randint(0, 6, (2500,), generator=g).to(cuda)
    params = []
    for flag in ("1", "0"):
        monkeypatch.setenv("HAR_MLP_EPOCH_GRAPH", flag)
        est = MultilayerPerceptronClassifier(layers=[43, H, H, 6], maxIter=4, blockSize=B, stepSize=1e-3, seed=3,
                                             device=cuda)
        params.append(est.fit_tensors(X, y, num_classes=6).engine.P.clone())
    torch.cuda.synchronize()
    assert torch.equal(params[0], params[1])
