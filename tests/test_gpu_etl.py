"""Device-resident ETL: the HIP CSV parser's table stays in HBM
(DeviceColumn) and describe / groupBy-count / StringIndexer / OneHotEncoder / VectorAssembler /
CastToDouble run on the device.  Every result must equal the host pipeline's."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("encoding", ["reference", "numeric43"])
def test_device_pipeline_equals_host(cuda, wisdm_csv, encoding):
    from har.data.csv_io import read_csv
    from har.data.split import random_split
    from har.data.table import DeviceColumn
    from har.features import wisdm
    from har.features.hybrid import hybrid_features

    host = read_csv(wisdm_csv)
    dev = read_csv(wisdm_csv, device=cuda)
    assert isinstance(dev["YAVG"], DeviceColumn) and isinstance(dev["XPEAK"], DeviceColumn)
    assert dev.dtypes == host.dtypes
    d1, m1, df1 = wisdm.prepare(host, encoding)
    d2, m2, df2 = wisdm.prepare(dev, encoding)
    f2 = df2["features"]
    assert isinstance(f2, DeviceColumn) and f2.kind == "vector"
    np.testing.assert_array_equal(f2.data, df1["features"].data)
    np.testing.assert_array_equal(df2["label"].data, df1["label"].data)
    if encoding == "reference":  # frequency-descending vocabularies (934 / 1401 / 755 one-hot widths)
        assert [s.labels for s in m2.stages if hasattr(s, "labels")] == \
               [s.labels for s in m1.stages if hasattr(s, "labels")]
        hm = hybrid_features(df2, "features", cuda)
        assert hm is f2.hybrid and hm.cat.shape[1] == 3 and hm.dense.shape[1] == 10
    # summaries computed on the device print the host numbers
    g1, g2 = d1.group_count("activity"), d2.group_count("activity")
    assert list(g2["activity"].data) == list(g1["activity"].data) and list(g2["count"].data) == list(g1["count"].data)
    num = [n for n, t in d1.dtypes if t in ("double", "int")]
    s1, s2 = d1.describe(num), d2.describe(num)
    for c in num:
        assert s2[c][0] == s1[c][0] and s2[c][3] == s1[c][3] and s2[c][4] == s1[c][4], c
        for k in (1, 2):
            assert abs(float(s2[c][k]) - float(s1[c][k])) <= 1e-9 * max(1.0, abs(float(s1[c][k]))), (c, k)
    tr1, te1 = random_split(df1, [0.7, 0.3], 2018)
    tr2, te2 = random_split(df2, [0.7, 0.3], 2018)
    assert tr2.count() == tr1.count() and isinstance(tr2["features"], DeviceColumn)
    np.testing.assert_array_equal(tr2["features"].data, tr1["features"].data)
    assert tr2.show(3) == tr1.show(3)


def test_main_reference_run_device_etl(cuda, wisdm_csv, tmp_path):
    import main

    s = main.run(main.config_from_args(["--data", wisdm_csv, "--out-dir", str(tmp_path), "--classifiers",
                                        "lr,dt,rf,nb", "--device", "cuda"]))
    h = main.run(main.config_from_args(["--data", wisdm_csv, "--out-dir", str(tmp_path / "h"), "--classifiers",
                                        "lr,dt,rf,nb", "--device", "cuda", "--no-csv-device"]))
    for k in ("lr", "dt", "rf", "nb"):
        assert abs(s["models"][k]["accuracy"] - h["models"][k]["accuracy"]) < 1e-9, k
    text = (tmp_path / "result.txt").read_text()
    assert "Walking" in text and "|   Walking| 2081|" in text
