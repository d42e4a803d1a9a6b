"""End-to-end: main.py artefacts, saved-model round trips, bench.py contract, build."""
import csv
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_main_reference_run_cpu(tmp_path, wisdm_csv):
    import main

    cfg = main.config_from_args(["--data", wisdm_csv, "--out-dir", str(tmp_path), "--device", "cpu",
                                 "--classifiers", "lr,dt,rf,lrcv", "--save-models", str(tmp_path / "models"),
                                 "--report"])
    s = main.run(cfg)
    m = s["models"]
    assert m["lr"]["accuracy"] >= 0.61 and m["dt"]["accuracy"] >= 0.72
    assert m["rf"]["accuracy"] >= 0.62 and m["lrcv"]["accuracy"] >= 0.70
    txt = (tmp_path / "result.txt").read_text()
    for banner in ("Loading Data Set...", "Data Schema----", "Activity Count----", "MODELING PIPELINE",
                   "Training Dataset Count : ", "CLASSIFICATION AND EVALUATION", "Binary Clasifier Area Under PR",
                   "MultiClass Weighted Precision", "Mean Absolute Error on test data", "Total Correct        ="):
        assert banner in txt
    with open(tmp_path / "additional_param.csv") as f:
        rows = list(csv.reader(f))
    assert rows[0] == ['Classifier', 'Count Total', 'Correct', 'Wrong', 'Ratio Wrong', 'Ratio Correct', 'F1 Score',
                       'Training Time', 'Testing Time', 'Accuracy']
    assert len(rows) == 4
    with open(tmp_path / "crossFold_additional_param.csv") as f:
        rows = list(csv.reader(f))
    assert rows[0][-3:] == ['Cross Validation Training Time', 'Cross Validation Testing Time', 'Cross Fold Accuracy']
    rec = json.loads((tmp_path / "metrics.jsonl").read_text().splitlines()[-1])
    assert rec["n_train"] + rec["n_test"] == 5418
    ph = rec["phases_s"]
    assert {"load_csv", "feature_pipeline", "random_split", "fit:lr", "predict:lr"} <= set(ph)
    assert abs(ph["fit:lr"] - rec["models"]["lr"]["train_s"]) < 2e-3
    # curated results (the reference's Results.xls / Graph.pdf / docs page, generated)
    rep = tmp_path / "report"
    with open(rep / "Results.csv") as f:
        res = list(csv.DictReader(f))
    assert [r["Classifier"] for r in res] == ["Logistic Regression", "Decision Tree", "Random Forest",
                                              "Logistic Regression (5-fold CV)"]
    assert int(res[0]["Correct"]) + int(res[0]["Wrong"]) == rec["n_test"]
    for png in ("prediction.png", "prediction_ratio.png", "accuracy.png", "lr_vs_lrcv.png", "training_time.png"):
        assert (rep / png).read_bytes()[:4] == b"\x89PNG"
    page = (rep / "index.html").read_text()
    assert "Results" in page and "data:image/png;base64," in page and "CLASSIFICATION AND EVALUATION" in page


def test_persist_roundtrip(tmp_path, wisdm_csv):
    from har.data.csv_io import read_csv
    from har.data.split import random_split
    from har.features import wisdm
    from har.models.logreg import LogisticRegression
    from har.models.mlp import MultilayerPerceptronClassifier
    from har.models.naive_bayes import NaiveBayes
    from har.models.tree import DecisionTreeClassifier, RandomForestClassifier
    from har.utils import persist

    raw = read_csv(wisdm_csv)
    data, pm, df = wisdm.prepare(raw, "numeric43")
    tr, te = random_split(df, [0.7, 0.3], 1)
    X = torch.as_tensor(te["features"].data)
    for est in (LogisticRegression(maxIter=5, device="cpu"), DecisionTreeClassifier(maxDepth=4, device="cpu"),
                RandomForestClassifier(numTrees=5, maxDepth=3, device="cpu"), NaiveBayes(modelType="gaussian"),
                MultilayerPerceptronClassifier(layers=[43, 32, 6], maxIter=1, device="cpu")):
        m = est.fit(tr)
        d = tmp_path / type(m).__name__
        persist.save(m, str(d), labels=df["label"].meta["vocab"])
        m2 = persist.load(str(d), device="cpu")
        torch.testing.assert_close(m2.predict_raw(X), m.predict_raw(X))
        md = json.loads((d / "metadata.json").read_text())
        assert md["class"] == type(m).__name__ and md["labels"][0] == "Walking"
    # pipeline: raw CSV rows -> identical features after reload
    persist.save(pm, str(tmp_path / "pipe"))
    pm2 = persist.load(str(tmp_path / "pipe"))
    np.testing.assert_array_equal(pm2.transform(data)["features"].data, df["features"].data)


def test_bench_contract_cpu():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--batch", "512"], capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in rec
    assert rec["n_gpus"] == 1 and rec["steps"] == 2 and rec["value"] > 0
    assert rec["config"]["parallelism"] == "dp1" and rec["scaling"] == "weak"


def test_native_build_uptodate():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import build_native

    if not os.path.exists(build_native.HIPCC):
        pytest.skip("no hipcc")
    build_native.build()
    assert not build_native.needs_build()
    import har._har_native as nat

    assert hasattr(nat, "gemm") and hasattr(nat, "tree_hist_split") and hasattr(nat, "csv_parse")


def test_yaml_configs_load():
    """Every configs/*.yaml is a valid RunConfig overlay (bench-only files hold a ``bench:`` block)."""
    import glob

    import yaml

    from har.config import config_from_args

    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs",
                                          "*.yaml")))
    assert len(files) >= 5
    for f in files:
        with open(f) as fh:
            d = yaml.safe_load(fh)
        if "bench" in d:
            assert d["bench"]["config"] in ("mlp", "rf", "stream", "rf9")
            continue
        cfg = config_from_args(["--preset-file", f])
        for k, v in d.items():
            assert getattr(cfg, k) == v


def test_predict_cli_from_saved_models(tmp_path, wisdm_csv):
    """predict.py re-encodes raw CSV rows with the saved PipelineModel and reproduces the
    saved model's predictions; unlabeled input (no ACTIVITY column) is served too."""
    import main
    import predict

    mdir = tmp_path / "models"
    main.run(main.config_from_args(["--data", wisdm_csv, "--out-dir", str(tmp_path / "out"), "--device", "cpu",
                                    "--preset", "all-numeric", "--classifiers", "dt,nb",
                                    "--save-models", str(mdir)]))
    rec = predict.main(["--models", str(mdir), "--model", "dt", "--data", wisdm_csv, "--device", "cpu",
                        "--out", str(tmp_path / "p.csv")])
    assert rec["rows"] == 5418 and rec["accuracy"] > 0.6 and rec["predict_windows_per_s"] > 0
    with open(tmp_path / "p.csv") as f:
        rows = list(csv.reader(f))
    assert rows[0] == ["row", "UID", "prediction", "label_name", "probability"] and len(rows) == 5419
    assert rows[1][3] in ("Walking", "Jogging", "Upstairs", "Downstairs", "Sitting", "Standing")
    # unlabeled serving input: drop ACTIVITY -> no metrics, same predictions
    lines = open(wisdm_csv).read().splitlines()
    hdr = lines[0].split(",")
    j = hdr.index("ACTIVITY")
    unl = tmp_path / "unlabeled.csv"
    unl.write_text("\n".join(",".join(c for k, c in enumerate(l.split(",")) if k != j) for l in lines[:201]) + "\n")
    rec2 = predict.main(["--models", str(mdir), "--model", "dt", "--data", str(unl), "--device", "cpu",
                         "--out", str(tmp_path / "q.csv")])
    assert rec2["rows"] == 200 and "accuracy" not in rec2
    with open(tmp_path / "q.csv") as f:
        q = list(csv.reader(f))
    assert [r[2] for r in q[1:]] == [r[2] for r in rows[1:201]]


def test_plots_hexbin_grid_and_scatter_matrix(tmp_path, wisdm_csv):
    """C29 (main.py:686-710): a seeded 10% sample, one hexbin PNG per ordered column pair
    ("Fig <x>_<y>.png") and Scatter_Matrix.png."""
    from har.data.csv_io import read_csv
    from har.report.plots import sample_numeric, write_plots

    t = read_csv(wisdm_csv)
    cols = ["YAVG", "ZAVG", "RESULTANT"]
    df = sample_numeric(t, cols, 0.1, seed=3)
    assert 400 < len(df) < 700 and list(df.columns) == cols
    written = write_plots(t, cols, str(tmp_path / "plot"), seed=3)
    names = sorted(os.path.basename(p) for p in written)
    assert "Scatter_Matrix.png" in names and "Fig YAVG_ZAVG.png" in names
    assert len([n for n in names if n.startswith("Fig ")]) == len(cols) ** 2
    assert all(os.path.getsize(p) > 1000 for p in written)


def test_warm_up_device_covers_every_classifier(wisdm_csv):
    """The device warm-up (suite.warm_up_device, run by main.py and the reference suite before any
    timer) fits every configured classifier — the CrossValidators included — on 256 rows and
    predicts through each model's own feature layout; on the CPU it must run the same code."""
    from har.config import RunConfig
    from har.models.base import labels_tensor, num_label_classes
    from har.suite import load_wisdm, warm_up_device

    cfg = RunConfig(cv_metric="mae")
    train, _, _ = load_wisdm(wisdm_csv, "reference", cfg.seed, device=torch.device("cpu"))
    warm_up_device(torch.device("cpu"), train, cfg, ["lr", "lrcv", "dt", "dtcv", "rf", "nb"])
    # the label tensor and class count are cached on the column (no device -> host read per fit)
    y = labels_tensor(train, "label", "cpu")
    assert labels_tensor(train, "label", "cpu") is y
    assert num_label_classes(train, "label", "cpu") == max(int(y.max()) + 1, len(train["label"].meta["vocab"]))
