"""Frame transform tests (reference: test/integration/functions/transform/
TransformFrameEncodeApplyTest, TransformFrameEncodeDecodeTest, TransformFrameEncodeColmapTest,
TransformFrameEncodeApplySubsetTest; data: src/test/scripts/functions/transform/input/homes3).

The reference compares encode vs apply outputs and decode(encode(F)) vs F; we do the same
on the reference's own homes3 data (read from the reference tree as plain CSV) and on
synthetic frames with missing values for impute/omit/bin, checked against numpy.
"""
import os
import shutil

import numpy as np
import pytest

from systemml_amd.api.executor import run
from systemml_amd.conf import DMLConfig
from systemml_amd.runtime.data import FrameBlock
from systemml_amd.runtime import transform as T

CFG = DMLConfig(gpu=False)
REF = "/root/reference/src/test/scripts/functions/transform"
HOMES = os.path.join(REF, "input", "homes3")
needs_ref = pytest.mark.skipif(not os.path.isdir(HOMES), reason="reference transform inputs not present")

SPECS = ["recode", "recode2", "dummy", "dummy2", "bin", "bin2", "impute", "impute2", "omit", "omit2",
         "recode_dummy", "recode_dummy2", "colmap1", "colmap2"]


@pytest.fixture(scope="module")
def homes(tmp_path_factory):
    d = tmp_path_factory.mktemp("homes")
    for f in ("homes.csv", "homes.csv.mtd"):
        shutil.copy(os.path.join(HOMES, f), d / f)
    return d


def _run(src, outputs=None, **args):
    return run(src, args=args, outputs=outputs or [], config=CFG)


@needs_ref
@pytest.mark.parametrize("spec", SPECS)
def test_encode_equals_apply(homes, spec):
    r = _run('''
F1 = read($DATA, data_type="frame", format="csv");
jspec = read($TFSPEC, data_type="scalar", value_type="string");
[X, M] = transformencode(target=F1, spec=jspec);
while(FALSE){}
X2 = transformapply(target=F1, spec=jspec, meta=M);
''', ["X", "X2", "M"], DATA=str(homes / "homes.csv"), TFSPEC=os.path.join(HOMES, f"homes.tfspec_{spec}.json"))
    X, X2 = r["X"].numpy(), r["X2"].numpy()
    np.testing.assert_array_equal(X, X2)
    assert not np.isnan(X).any()
    assert X.shape[0] == 148
    if "dummy" in spec or "colmap" in spec:
        # every dummy block has exactly one 1 per row
        width = {"dummy": 17, "dummy2": 17, "colmap1": 17, "colmap2": 17,
                 "recode_dummy": 14, "recode_dummy2": 14}[spec]
        assert X.shape[1] == width


@needs_ref
@pytest.mark.parametrize("spec", ["recode", "recode2", "dummy", "dummy2", "recode_dummy"])
def test_encode_decode_roundtrip(homes, spec):
    r = _run('''
F1 = read($DATA, data_type="frame", format="csv");
jspec = read($TFSPEC, data_type="scalar", value_type="string");
[X, M] = transformencode(target=F1, spec=jspec);
F2 = transformdecode(target=X, spec=jspec, meta=M);
''', ["F1", "F2"], DATA=str(homes / "homes.csv"), TFSPEC=os.path.join(HOMES, f"homes.tfspec_{spec}.json"))
    F1, F2 = r["F1"], r["F2"]
    assert F2.shape == F1.shape
    for j in range(F1.ncol()):
        a, b = F1.columns[j], F2.columns[j]
        if F2.schema[j] == "STRING":
            assert [str(x) for x in a] == [str(x) for x in b]
        else:
            np.testing.assert_allclose([float(x) for x in a], b)


@needs_ref
def test_colmap_script(homes, tmp_path):
    src = open(os.path.join(REF, "TransformFrameEncodeColmap1.dml")).read()
    out = tmp_path / "F2"
    _run(src, DATA=str(homes / "homes.csv"), TFSPEC=os.path.join(HOMES, "homes.tfspec_colmap1.json"),
         TFDATA=str(out), OFMT="csv")
    got = [l.split(",") for l in open(out).read().strip().split("\n")]
    ref = [l.split(",") for l in open(homes / "homes.csv").read().strip().split("\n")[1:]]
    assert len(got) == len(ref)
    for g, e in zip(got, ref):
        for a, b in zip(g, e):
            try:
                assert float(a) == float(b)
            except ValueError:
                assert a == b


@needs_ref
def test_apply_subset_script(homes, tmp_path):
    src = open(os.path.join(REF, "TransformFrameEncodeApplySubset1.dml")).read()
    _run(src, **{"1": str(homes / "homes.csv"), "2": str(tmp_path / "R")})
    assert open(tmp_path / "R").read().split() == ["1", "1", "148.0"]


def _frame():
    cols = [["a", "b", None, "a", "c", "a"],
            [1.0, None, 3.0, 4.0, 5.0, 6.0],
            ["x", "y", "y", None, "y", "x"],
            [10.0, 20.0, 30.0, 40.0, 50.0, 60.0]]
    return FrameBlock(cols, ["STRING", "DOUBLE", "STRING", "DOUBLE"], ["cat", "num", "cat2", "v"])


def test_impute_modes_and_recode():
    fr = _frame()
    spec = ('{ids: true, recode: [1, 3], impute: [{id: 1, method: global_mode}, '
            '{id: 2, method: global_mean}, {id: 3, method: constant, value: "y"}]}')
    X, M = T.encode(None, fr, spec)
    X = X.numpy()
    np.testing.assert_array_equal(X[:, 0], [1, 2, 1, 1, 3, 1])          # a=1,b=2,c=3; missing -> mode a
    np.testing.assert_allclose(X[1, 1], np.mean([1, 3, 4, 5, 6]))
    np.testing.assert_array_equal(X[:, 2], [1, 2, 2, 2, 2, 1])          # x=1,y=2; missing -> y
    assert M.col_meta[0]["ndistinct"] == 3 and M.col_meta[0]["mv"] == "a"


def test_omit_and_dummycode_order():
    fr = _frame()
    fr = FrameBlock([fr.columns[0], fr.columns[1], fr.columns[3]], ["STRING", "DOUBLE", "DOUBLE"], ["cat", "num", "v"])
    X, M = T.encode(None, fr, '{ids: true, dummycode: [1], omit: [1, 2]}')
    # rows with a missing cat / num are dropped, then cat expands into 3 one-hot columns
    np.testing.assert_array_equal(X.numpy(), [[1, 0, 0, 1, 10], [1, 0, 0, 4, 40], [0, 0, 1, 5, 50], [1, 0, 0, 6, 60]])


def test_omit_drops_missing_rows():
    fr = FrameBlock([[1.0, None, 3.0], [4.0, 5.0, None]], ["DOUBLE", "DOUBLE"], ["a", "b"])
    X, _ = T.encode(None, fr, '{"ids": true, "omit": [1]}')
    np.testing.assert_array_equal(X.numpy(), [[1, 4], [3, np.nan]])


def test_equi_width_bins():
    vals = np.array([0.0, 1.0, 2.5, 5.0, 7.5, 10.0])
    fr = FrameBlock([vals.tolist()], ["DOUBLE"], ["x"])
    X, M = T.encode(None, fr, '{"ids": true, "bin": [{"id": 1, "method": "equi-width", "numbins": 4}]}')
    np.testing.assert_array_equal(X.numpy().ravel(), [1, 1, 1, 2, 3, 4])
    assert M.col_meta[0]["ndistinct"] == 4
    # apply on new data with the same meta: bins clamp at the ends
    X2 = T.apply(None, FrameBlock([[-5.0, 3.0, 99.0]], ["DOUBLE"], ["x"]),
                 '{"ids": true, "bin": [{"id": 1, "method": "equi-width", "numbins": 4}]}', M)
    np.testing.assert_array_equal(X2.numpy().ravel(), [1, 2, 4])


def test_colmap_and_named_spec():
    fr = _frame()
    fr.columns[0] = ["a", "b", "a", "a", "c", "a"]
    X, M = T.encode(None, fr, '{"dummycode": ["cat", cat2]}')
    cm = T.colmap(None, M, '{"dummycode": ["cat", cat2]}').numpy()
    np.testing.assert_array_equal(cm, [[1, 1, 3], [2, 4, 4], [3, 5, 6], [4, 7, 7]])
    assert X.shape == (6, 7)
    np.testing.assert_array_equal(X[3, 4:6].numpy(), [0, 0])      # missing cat2 -> all-zero block


def test_transformmeta_reads_meta_directory(tmp_path):
    d = tmp_path / "meta"
    (d / "Recode").mkdir(parents=True)
    (d / "column.names").write_text("city,price\n")
    (d / "Recode" / "city.map").write_text('"ber",1,10\n"par",2,5\n')
    (d / "Recode" / "city.ndistinct").write_text("2\n")
    src = '''
F = as.frame(matrix(0, 1, 1))
M = transformmeta(spec="{ids: true, recode: [1]}", meta=$META)
X = matrix("2 7 1 9", rows=2, cols=2)
G = transformdecode(target=X, spec="{ids: true, recode: [1]}", meta=M)
'''
    r = _run(src, ["G"], META=str(d))
    G = r["G"]
    assert G.columns[0] == ["par", "ber"]
    assert G.columns[1] == [7.0, 9.0]


@needs_ref
def test_legacy_transform_and_apply_scripts(homes, tmp_path):
    from systemml_amd.api.mlcontext import SCRIPTS_DIR
    spec = os.path.join(HOMES, "homes.tfspec_recode_dummy.json")
    tdir = tmp_path / "tf"
    src = open(os.path.join(SCRIPTS_DIR, "algorithms", "transform.dml")).read()
    _run(src, DATA_PATH=str(homes / "homes.csv"), TRANSFORM_SPEC_PATH=spec, TRANSFORM_PATH=str(tdir),
         OUTPUT_NAMES=str(tmp_path / "names"), OUTPUT_DATA_PATH=str(tmp_path / "A.csv"))
    assert (tdir / "Recode" / "zipcode.map").exists() and (tdir / "column.names").exists()
    src2 = open(os.path.join(SCRIPTS_DIR, "algorithms", "apply-transform.dml")).read()
    _run(src2, DATA_PATH=str(homes / "homes.csv"), TRANSFORM_PATH=str(tdir), APPLY_TRANSFORM_PATH=str(tdir),
         OUTPUT_DATA_PATH=str(tmp_path / "B.csv"))
    A = np.loadtxt(tmp_path / "A.csv", delimiter=",")
    B = np.loadtxt(tmp_path / "B.csv", delimiter=",")
    assert A.shape == (148, 14)
    np.testing.assert_array_equal(A, B)
