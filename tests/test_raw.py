"""Raw accelerometer rows -> WISDM transformed table -> main.py (features/raw.py).

The reference starts from the pre-windowed table (Main/main.py:16-20); ``main.py --raw``
starts from ``user,activity,timestamp,x,y,z`` rows, windows them inside (user, activity)
runs and featurizes them into the exact WISDM columns (``wisdm_data.csv:1``)."""
import json
import os

import numpy as np
import pytest
import torch

from har.features.raw import WISDM43, raw_to_table, read_raw, window_starts, write_synthetic_raw
from har.features.window import window_features_torch


def _as_matrix(t):
    cols = []
    for c in WISDM43:
        d = t[c].data
        cols.append(np.array([np.nan if v == "?" else float(v) for v in d]) if t[c].kind == "string"
                    else d.astype(np.float64))
    return np.stack(cols, 1)


def test_window_starts_respect_segments():
    user = np.array([1] * 10 + [2] * 7 + [2] * 9)
    act = np.array(["a"] * 10 + ["a"] * 7 + ["b"] * 9, dtype=object)
    st, seg = window_starts(user, act, 4, 2)
    # segments [0,10), [10,17), [17,26): windows of 4 every 2 samples inside each
    assert st.tolist() == [0, 2, 4, 6, 10, 12, 17, 19, 21]
    assert seg.tolist() == [0, 0, 0, 0, 10, 10, 17, 17, 17]


@pytest.mark.parametrize("overlap,txt", [(0.0, False), (0.5, True)])
def test_raw_table_matches_window_oracle(tmp_path, overlap, txt):
    p = str(tmp_path / ("raw.txt" if txt else "raw.csv"))
    write_synthetic_raw(p, n_windows=40, users=3, wisdm_txt=txt)
    t = raw_to_table(p, hz=20.0, window_sec=10.0, overlap=overlap)
    assert t.columns == ["UID", "USER"] + WISDM43 + ["ACTIVITY"]
    assert t["XPEAK"].kind == "string" and t["X0"].kind == "double" and t["ACTIVITY"].kind == "string"
    user, act, _, xyz = read_raw(p)
    st, _ = window_starts(user, act, 200, 100 if overlap else 200)
    assert t.count() == len(st) and (t.count() > 40 if overlap else t.count() == 40)
    ref = torch.cat([window_features_torch(torch.as_tensor(xyz[s:s + 200]), 200, 200, 20.0) for s in st])[:, :43]
    got = _as_matrix(t)
    peak = np.array([c.endswith("PEAK") for c in WISDM43])
    np.testing.assert_allclose(got[:, ~peak], ref.double().numpy()[:, ~peak], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(got[:, peak], ref.double().numpy()[:, peak], atol=0.5 + 1e-6)  # integer ms
    assert list(t["ACTIVITY"].data) == list(act[st])


def test_main_raw_end_to_end(tmp_path):
    import main

    p = str(tmp_path / "raw.csv")
    write_synthetic_raw(p, n_windows=160, users=5)
    out = tmp_path / "out"
    s = main.run(main.config_from_args(["--raw", p, "--out-dir", str(out), "--device", "cpu", "--classifiers",
                                        "lr,dt,rf", "--encoding", "numeric43"]))
    text = (out / "result.txt").read_text()
    assert "Raw stream" in text and "Classifier trained in" in text
    assert s["n_train"] + s["n_test"] == 160
    assert s["models"]["rf"]["accuracy"] > 0.5  # class-conditional synthetic dynamics are learnable
    rec = json.loads((out / "metrics.jsonl").read_text().splitlines()[-1])
    assert set(rec["models"]) == {"lr", "dt", "rf"}


@pytest.mark.gpu
def test_raw_table_gpu_equals_cpu(cuda, tmp_path):
    p = str(tmp_path / "raw.csv")
    write_synthetic_raw(p, n_windows=64, users=4)
    peak = np.array([c.endswith("PEAK") for c in WISDM43])
    for ov in (0.0, 0.5):
        a = _as_matrix(raw_to_table(p, overlap=ov, device=cuda))
        b = _as_matrix(raw_to_table(p, overlap=ov, device="cpu"))
        np.testing.assert_allclose(a[:, ~peak], b[:, ~peak], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(a[:, peak], b[:, peak], atol=1.0)  # integer ms, rounding ties may flip


def _dp_worker(rank, world, port, path, out):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from har.parallel import dist as hd

    ctx = hd.init(device="cpu")
    t = raw_to_table(path, overlap=0.5, ctx=ctx)
    np.save(os.path.join(out, f"r{rank}.npy"), _as_matrix(t))
    hd.shutdown(ctx)


@pytest.mark.parametrize("world", [2, 3])
def test_raw_featurization_sharded_with_halo_equals_single(tmp_path, world):
    """Ranks featurize the windows starting in their sample shard (halo = window - 1 samples
    from the next rank, batch_isend_irecv) and all-gather: the table every rank ends up with
    equals one process's."""
    import torch.multiprocessing as mp

    from test_distributed import _free_port

    p = str(tmp_path / "raw.csv")
    write_synthetic_raw(p, n_windows=30, users=3)
    mp.spawn(_dp_worker, args=(world, _free_port(), p, str(tmp_path)), nprocs=world, join=True)
    single = _as_matrix(raw_to_table(p, overlap=0.5))
    for r in range(world):
        np.testing.assert_allclose(np.load(tmp_path / f"r{r}.npy"), single, rtol=1e-6, atol=1e-6)
