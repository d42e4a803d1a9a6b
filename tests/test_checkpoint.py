"""Checkpoint / resume / fault injection (SURVEY.md §5 failure handling).

A training process is hard-killed mid-run by ``HAR_FAULT_INJECT`` (exit code 17,
like a crashed rank); re-running the same command resumes from the newest
checkpoint and must produce exactly the model an uninterrupted run produces.
"""
import os
import subprocess
import sys

import pytest
import torch

from har.models.tree import RandomForestClassifier
from har.utils.checkpoint import FAULT_EXIT_CODE, Checkpointer

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r"""
import sys, torch
torch.set_num_threads(2)
from har.models.mlp import MultilayerPerceptronClassifier
from har.models.tree import RandomForestClassifier
kind, ckpt, out, dev = sys.argv[1:5]
g = torch.Generator().manual_seed(0)
mu = torch.randn(4, 12, generator=g) * 2
y = torch.randint(0, 4, (1024,), generator=g)
X = (mu[y] + torch.randn(1024, 12, generator=g)).to(dev)
y = y.to(dev)
ck = None if ckpt == "-" else ckpt
if kind == "mlp":
    m = MultilayerPerceptronClassifier(layers=[12, 32, 32, 4], maxIter=3, blockSize=128, stepSize=3e-3, seed=5,
                                       device=dev, checkpointDir=ck, checkpointInterval=4).fit_tensors(X, y)
    torch.save({"P": m.engine.P.detach().cpu()}, out)
else:
    rf = RandomForestClassifier(numTrees=12, maxDepth=4, seed=3, device=dev)
    m = rf.fit_tensors(X, y, 4, tree_wave=4, checkpoint_dir=ck)
    torch.save({"raw": m.predict_all(X)[0].detach().float().cpu()}, out)
"""


def _run(kind, ckpt, out, dev="cpu", fault=None):
    env = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
    env.pop("HAR_FAULT_INJECT", None)
    if fault is not None:
        env["HAR_FAULT_INJECT"] = str(fault)
    return subprocess.run([sys.executable, "-c", _SCRIPT, kind, ckpt, out, dev], env=env, capture_output=True,
                          text=True, timeout=300)


@pytest.mark.parametrize("kind,fault", [("mlp", 10), ("rf", 8)])
def test_fault_then_resume_matches_uninterrupted(tmp_path, kind, fault):
    ref = _run(kind, "-", str(tmp_path / "ref.pt"))
    assert ref.returncode == 0, ref.stderr
    ck = str(tmp_path / "ckpt")
    crashed = _run(kind, ck, str(tmp_path / "crash.pt"), fault=fault)
    assert crashed.returncode == FAULT_EXIT_CODE, crashed.stderr
    assert not os.path.exists(tmp_path / "crash.pt")
    assert Checkpointer(ck).latest() is not None  # something to resume from
    resumed = _run(kind, ck, str(tmp_path / "res.pt"))
    assert resumed.returncode == 0, resumed.stderr
    a = torch.load(tmp_path / "ref.pt", weights_only=True)
    b = torch.load(tmp_path / "res.pt", weights_only=True)
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_checkpointer_keeps_latest(tmp_path):
    c = Checkpointer(str(tmp_path), keep=2)
    for s in (1, 2, 3):
        c.save(s, {"x": torch.tensor([float(s)])}, {"tag": s})
    st, meta = c.latest()
    assert meta["step"] == 3 and float(st["x"][0]) == 3.0
    assert len([p for p in os.listdir(tmp_path) if p.endswith(".pt")]) == 2
    # non-zero ranks never write (replicated state has one writer)
    Checkpointer(str(tmp_path / "r1"), rank=1).save(9, {"x": torch.zeros(1)})
    assert Checkpointer(str(tmp_path / "r1")).latest() is None


def test_stale_checkpoint_of_another_fit_is_ignored(tmp_path):
    """A checkpoint written by a forest with other parameters (here: more trees, another seed)
    must not be resumed: the fit starts over and returns exactly the requested forest."""
    g = torch.Generator().manual_seed(2)
    y = torch.randint(0, 3, (600,), generator=g)
    X = torch.randn(3, 8, generator=g)[y] * 2 + torch.randn(600, 8, generator=g)
    ck = str(tmp_path / "ck")
    RandomForestClassifier(numTrees=9, maxDepth=3, seed=1, device="cpu").fit_tensors(X, y, 3, tree_wave=3,
                                                                                     checkpoint_dir=ck)
    assert Checkpointer(ck).latest() is not None
    with pytest.warns(UserWarning, match="different fit"):
        m = RandomForestClassifier(numTrees=6, maxDepth=3, seed=2, device="cpu").fit_tensors(
            X, y, 3, tree_wave=3, checkpoint_dir=ck)
    fresh = RandomForestClassifier(numTrees=6, maxDepth=3, seed=2, device="cpu").fit_tensors(X, y, 3)
    assert m.getNumTrees == 6
    assert torch.equal(m.predict_all(X)[0], fresh.predict_all(X)[0])


def test_rf_waves_equal_one_shot():
    g = torch.Generator().manual_seed(1)
    mu = torch.randn(3, 10, generator=g) * 2
    y = torch.randint(0, 3, (900,), generator=g)
    X = mu[y] + torch.randn(900, 10, generator=g)
    one = RandomForestClassifier(numTrees=10, maxDepth=5, seed=7, device="cpu").fit_tensors(X, y, 3)
    wav = RandomForestClassifier(numTrees=10, maxDepth=5, seed=7, device="cpu").fit_tensors(X, y, 3, tree_wave=3)
    assert torch.equal(one.predict_all(X)[0], wav.predict_all(X)[0])
    assert torch.equal(one.arrs.feature, wav.arrs.feature)


def test_rf_int32_slot_cap_waves_automatically(monkeypatch):
    """(tree, row) slots are int32 on the device: a forest whose lock-step build would exceed
    the slot limit grows in waves by itself, equal to the one-shot forest."""
    import har.models.tree as tree_mod

    assert tree_mod.max_lockstep_trees(4_300_000) == (2 ** 31 - 1) // 4_300_000
    assert tree_mod.max_lockstep_trees(2 ** 32) == 1
    g = torch.Generator().manual_seed(3)
    mu = torch.randn(3, 8, generator=g) * 2
    y = torch.randint(0, 3, (600,), generator=g)
    X = mu[y] + torch.randn(600, 8, generator=g)
    one = RandomForestClassifier(numTrees=7, maxDepth=4, seed=5, device="cpu").fit_tensors(X, y, 3)
    built = []
    real = tree_mod.ForestBuilder

    class Spy(real):
        def __init__(self, K, nt, *a, **kw):
            built.append(nt)
            super().__init__(K, nt, *a, **kw)

    monkeypatch.setattr(tree_mod, "LOCKSTEP_SLOT_LIMIT", 600 * 3)
    monkeypatch.setattr(tree_mod, "ForestBuilder", Spy)
    capped = RandomForestClassifier(numTrees=7, maxDepth=4, seed=5, device="cpu").fit_tensors(X, y, 3)
    assert built == [3, 3, 1]
    assert torch.equal(one.arrs.feature, capped.arrs.feature)
    assert torch.equal(one.predict_all(X)[0], capped.predict_all(X)[0])


@pytest.mark.gpu
@pytest.mark.parametrize("kind,fault", [("mlp", 10), ("rf", 8)])
def test_fault_then_resume_gpu(tmp_path, kind, fault):
    """Same as the CPU test through the HIP kernels: the native MLP step (device-side Adam
    step counter restored) and the waved GPU forest resume bit-for-bit."""
    ref = _run(kind, "-", str(tmp_path / "ref.pt"), dev="cuda")
    assert ref.returncode == 0, ref.stderr
    ck = str(tmp_path / "ckpt")
    assert _run(kind, ck, str(tmp_path / "c.pt"), dev="cuda", fault=fault).returncode == FAULT_EXIT_CODE
    res = _run(kind, ck, str(tmp_path / "res.pt"), dev="cuda")
    assert res.returncode == 0, res.stderr
    a = torch.load(tmp_path / "ref.pt", weights_only=True)
    b = torch.load(tmp_path / "res.pt", weights_only=True)
    for k in a:
        assert torch.equal(a[k], b[k]), k


@pytest.mark.gpu
def test_gpu_training_is_deterministic(cuda):
    """Split-K slabs + fixed-order reductions (no float atomics on the training path):
    two identical runs give bitwise-identical parameters / forests."""
    from har.models.mlp import MultilayerPerceptronClassifier

    g = torch.Generator().manual_seed(3)
    mu = torch.randn(6, 43, generator=g) * 2
    y = torch.randint(0, 6, (8192,), generator=g)
    X = (mu[y] + torch.randn(8192, 43, generator=g)).cuda()
    y = y.cuda()
    ps = []
    for _ in range(2):
        m = MultilayerPerceptronClassifier(layers=[43, 128, 128, 6], maxIter=2, blockSize=1024, seed=1,
                                           device="cuda").fit_tensors(X, y)
        ps.append(m.engine.P.detach().clone())
    assert torch.equal(ps[0], ps[1])
    fs = [RandomForestClassifier(numTrees=16, maxDepth=8, seed=2, device="cuda").fit_tensors(X, y, 6)
          for _ in range(2)]
    assert torch.equal(fs[0].arrs.feature, fs[1].arrs.feature)
    assert torch.equal(fs[0].arrs.threshold, fs[1].arrs.threshold)


_ELASTIC = r"""
import os, sys, torch
torch.set_num_threads(1)
from har.parallel import dist as hd
from har.models.mlp import MultilayerPerceptronClassifier
ckpt, out = sys.argv[1:3]
ctx = hd.init(device="cpu")
g = torch.Generator().manual_seed(0)
mu = torch.randn(4, 12, generator=g) * 2
y = torch.randint(0, 4, (1024,), generator=g)
X = mu[y] + torch.randn(1024, 12, generator=g)
per = 1024 // ctx.world_size
lo = ctx.rank * per
m = MultilayerPerceptronClassifier(layers=[12, 32, 32, 4], maxIter=3, blockSize=64, stepSize=3e-3, seed=5,
                                   device="cpu", checkpointDir=None if ckpt == "-" else ckpt,
                                   checkpointInterval=4).fit_tensors(X[lo:lo + per], y[lo:lo + per],
                                                                     process_group=ctx.group, rank=ctx.rank,
                                                                     world_size=ctx.world_size, num_classes=4)
if ctx.rank == 0:
    torch.save({"P": m.engine.P.detach().cpu(),
                "attempt": torch.tensor(int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")))}, out)
hd.shutdown(ctx)
"""


def _torchrun(tmp_path, ckpt, out, fault=None, restarts=0):
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    script = tmp_path / "elastic.py"
    script.write_text(_ELASTIC)
    env = dict(os.environ, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""), HAR_DIST_TIMEOUT_S="60")
    env.pop("HAR_FAULT_INJECT", None)
    if fault is not None:
        env["HAR_FAULT_INJECT"] = fault
    # dynamic (c10d) rendezvous: each restart forms a new round on the agent's store
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           f"--max-restarts={restarts}", "--rdzv-backend=c10d", f"--rdzv-endpoint=127.0.0.1:{port}",
           "--rdzv-id=har-elastic-test", "--monitor-interval=0.5", str(script), ckpt, out]
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)


def test_torchrun_rank_failure_restarts_and_resumes(tmp_path):
    """A DP rank crashes mid-fit (rank 1 at step 10 of 48, exit 17); torchrun's elastic agent
    tears the group down and restarts it (--max-restarts 1); both ranks resume from the newest
    checkpoint (step 8) and the final model equals an uninterrupted 2-rank fit bit for bit."""
    ref = _torchrun(tmp_path, "-", str(tmp_path / "ref.pt"))
    assert ref.returncode == 0, ref.stderr[-3000:]
    ck = str(tmp_path / "ckpt")
    res = _torchrun(tmp_path, ck, str(tmp_path / "res.pt"), fault="1:10", restarts=1)
    assert res.returncode == 0, res.stderr[-3000:]
    a = torch.load(tmp_path / "ref.pt", weights_only=True)
    b = torch.load(tmp_path / "res.pt", weights_only=True)
    assert int(b["attempt"]) == 1  # the run that finished is the restarted one
    assert torch.equal(a["P"], b["P"])
    # without a restart budget the same failure ends the job with an error instead of hanging
    fail = _torchrun(tmp_path, str(tmp_path / "ckpt2"), str(tmp_path / "fail.pt"), fault="1:10", restarts=0)
    assert fail.returncode != 0 and not os.path.exists(tmp_path / "fail.pt")


def _stall_worker(rank, port, out_dir):
    import time

    import torch.distributed as dist

    os.environ.update(RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from har.parallel import dist as hd

    ctx = hd.init(device="cpu", timeout_s=4)
    if rank == 1:
        time.sleep(10)  # a stalled rank: never reaches the collective in time
    t0 = time.time()
    err = ""
    try:
        dist.all_reduce(torch.ones(4))
    except Exception as e:  # gloo raises on the timeout (peer stalled / gone)
        err = type(e).__name__ + ": " + str(e)[:200]
    with open(os.path.join(out_dir, f"stall_{rank}.txt"), "w") as f:
        f.write(f"{time.time() - t0:.2f}\n{err}")
    os._exit(0)  # the group is broken: skip destroy_process_group


def test_stalled_rank_makes_peers_time_out(tmp_path):
    """Failure detection: a rank that stalls before a collective makes its peer's collective raise
    after the group timeout (HAR_DIST_TIMEOUT_S / init(timeout_s=...)) instead of hanging."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_stall_worker, args=(port, str(tmp_path)), nprocs=2, join=True)
    elapsed, err = (tmp_path / "stall_0.txt").read_text().split("\n", 1)
    assert err, "rank 0's all_reduce returned although rank 1 never joined"
    assert float(elapsed) < 9.0, elapsed  # raised by the 4 s timeout, not by rank 1 arriving at 10 s
