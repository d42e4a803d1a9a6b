"""CSV ingest, schema inference, table ops, encoders, split — vs golden facts of
the reference run (result.txt)."""
import numpy as np
import pytest

from har.data.csv_io import parse_csv_bytes, parse_csv_text_python, read_csv
from har.data.split import kfold_ids, random_split, split_ids
from har.data.table import Column, Table, java_double_str
from har.features import wisdm
from har.features.encode import OneHotEncoder, Pipeline, StringIndexer, VectorAssembler
from har.ops import _native


def test_java_double_str():
    assert java_double_str(8.4) == "8.4"
    assert java_double_str(0.0) == "0.0"
    assert java_double_str(1550.0) == "1550.0"
    assert java_double_str(1e-5) == "1.0E-5"
    assert java_double_str(12345678.0) == "1.2345678E7"


SAMPLE = b'a,b,c,d,e\r\n1,2.5,x,"q,1",\r\n2,?,y,"he said ""hi""",3\r\n3,4,z,w,4\r\n'


@pytest.mark.parametrize("native", [False, True])
def test_csv_parse_semantics(native):
    if native and not _native.available():
        pytest.skip("native extension not built")
    t = parse_csv_bytes(SAMPLE, use_native=native)
    assert t.columns == ["a", "b", "c", "d", "e"]
    assert t["a"].kind == "int" and list(t["a"].data) == [1, 2, 3]
    assert t["b"].kind == "string"          # '?' makes the column a string (Spark inferSchema)
    assert list(t["d"].data) == ["q,1", 'he said "hi"', "w"]
    assert t["e"].kind == "int" and t["e"].missing is not None and t["e"].missing[0]


def test_native_matches_python_parser(wisdm_csv):
    if not _native.available():
        pytest.skip("native extension not built")
    a = read_csv(wisdm_csv, use_native=True)
    b = read_csv(wisdm_csv, use_native=False)
    assert a.columns == b.columns
    for c in a.columns:
        assert a[c].kind == b[c].kind
        if a[c].kind == "double":
            np.testing.assert_allclose(a[c].data, b[c].data)
        else:
            assert list(a[c].data) == list(b[c].data)


def test_wisdm_schema_and_golden_facts(wisdm_csv):
    t = read_csv(wisdm_csv)
    assert t.count() == 5418 and len(t.columns) == 46
    data = t.drop(wisdm.DROP_LIST)
    kinds = dict(data.dtypes)
    assert kinds["UID"] == "int" and kinds["XAVG"] == "int" and kinds["XPEAK"] == "string"
    assert kinds["YAVG"] == "double" and kinds["ACTIVITY"] == "string"
    gc = data.group_count("activity")
    assert list(gc["activity"].data) == ["Walking", "Jogging", "Upstairs", "Downstairs", "Sitting", "Standing"]
    assert list(gc["count"].data) == [2081, 1625, 632, 528, 306, 246]
    d = data.describe(["YAVG", "UID"])
    assert abs(float(d["YAVG"][1]) - 7.076515319306007) < 1e-9
    assert abs(float(d["YAVG"][2]) - 3.7527377344848674) < 1e-9
    assert d["UID"][3] == "1" and d["UID"][4] == "728"
    s = data.print_schema()
    assert " |-- XPEAK: string (nullable = true)" in s
    shown = data.show(5)
    assert "|UID|XAVG|YAVG|" in shown and "only showing top 5 rows" in shown


def test_reference_encoding_dims(wisdm_csv):
    t = read_csv(wisdm_csv)
    _, model, df = wisdm.prepare(t, "reference")
    f = df["features"]
    assert f.data.shape == (5418, 3100)
    offs = [b["offset"] for b in f.meta["structure"]]
    assert offs[:4] == [0, 934, 2335, 3090]
    assert df["label"].meta["vocab"] == ["Walking", "Jogging", "Upstairs", "Downstairs", "Sitting", "Standing"]
    assert (f.data[:, :3090].sum(1) <= 3).all()


def test_numeric43_encoding(wisdm_csv):
    t = read_csv(wisdm_csv)
    _, _, df = wisdm.prepare(t, "numeric43")
    X = df["features"].data
    assert X.shape == (5418, 43)
    assert (X[:, 33] == -1).sum() == 381  # XPEAK '?' count -> -1


def test_string_indexer_tie_break_and_invalid():
    t = Table([Column("c", "string", np.array(["b", "a", "b", "a", "c"], dtype=object))])
    m = StringIndexer("c", "ci").fit(t)
    assert m.labels == ["a", "b", "c"]  # ties by frequency break alphabetically
    t2 = Table([Column("c", "string", np.array(["a", "zz"], dtype=object))])
    with pytest.raises(ValueError):
        m.transform(t2)
    m.handleInvalid = "keep"
    assert list(m.transform(t2)["ci"].data) == [0, 3]


def test_onehot_droplast_and_assembler():
    t = Table([Column("c", "string", np.array(["x", "y", "x", "z"], dtype=object)),
               Column("n", "double", np.array([1.0, 2.0, 3.0, 4.0]))])
    pm = Pipeline([StringIndexer("c", "ci"), OneHotEncoder(["ci"], ["cv"]), VectorAssembler(["cv", "n"], "f")]).fit(t)
    f = pm.transform(t)["f"].data
    assert f.shape == (4, 3)  # 3 categories -> width 2 (dropLast) + 1 numeric
    np.testing.assert_array_equal(f[:, :2], [[1, 0], [0, 1], [1, 0], [0, 0]])


def test_split_deterministic_and_shard_invariant():
    n = 20000
    ids = split_ids(n, [0.7, 0.3], 2018)
    assert abs((ids == 0).mean() - 0.7) < 0.02
    # world-size invariance: a shard's split equals the slice of the global split
    lo = 7000
    np.testing.assert_array_equal(split_ids(n - lo, [0.7, 0.3], 2018, row_offset=lo), ids[lo:])
    f = kfold_ids(n, 5, 1)
    assert set(np.unique(f)) == {0, 1, 2, 3, 4} and abs((f == 2).mean() - 0.2) < 0.02


def test_random_split_wisdm_sizes(wisdm_csv):
    t = read_csv(wisdm_csv)
    tr, te = random_split(t, [0.7, 0.3], 2018)
    assert tr.count() + te.count() == 5418
    assert abs(tr.count() - 3793) < 120  # Spark's own draw gave 3793 / 1625


@pytest.mark.gpu
def test_device_csv_matches_host(cuda, wisdm_csv, tmp_path):
    from har.data.csv_device import read_csv_device

    for path in (wisdm_csv, None):
        if path is None:
            path = str(tmp_path / "s.csv")
            with open(path, "wb") as f:
                f.write(SAMPLE + b"4,5e2,zz,\"\",7\n\n")
        host = read_csv(path, use_native=True)  # native host parser: quoted "" is a present empty string
        dev = read_csv_device(path, cuda).to_table()
        assert dev.columns == host.columns and dev.count() == host.count()
        for c in host.columns:
            assert dev[c].kind == host[c].kind, c
            if host[c].kind == "double":
                np.testing.assert_array_equal(dev[c].data, host[c].data)
            else:
                assert list(dev[c].data) == list(host[c].data), c


@pytest.mark.gpu
def test_device_csv_edge_tokens_match_host(cuda, tmp_path):
    """'Infected' is a string (only the exact 'Infinity' is a number), and values outside the
    kernel's exact fast path (17+ significant digits, |exp| > 22) equal strtod bit for bit."""
    from har.data.csv_device import read_csv_device

    path = str(tmp_path / "edge.csv")
    with open(path, "wb") as f:
        f.write(b"a,b,c\n"
                b"1.2345678901234567891,Infected,3e-30\n"
                b"9007199254740993,Infinity,1.7976931348623157e308\n"
                b"-0.1000000000000000055511151231257827,-Infinity,4.9e-324\n")
    host = read_csv(path, use_native=True)
    dev = read_csv_device(path, cuda).to_table()
    for c in host.columns:
        assert dev[c].kind == host[c].kind, c
        if host[c].kind == "double":
            np.testing.assert_array_equal(dev[c].data, host[c].data)
        else:
            assert list(dev[c].data) == list(host[c].data), c
