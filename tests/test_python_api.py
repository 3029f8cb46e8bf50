"""Python API surface of the reference (src/main/python/systemml): `import systemml`,
random sampling, converters (incl. a caffemodel written here with a minimal protobuf
encoder — parity unpinned: no caffe model ships in the reference), getHopDAG."""
import struct

import numpy as np
import pytest


def test_systemml_package_exports():
    import systemml as sml
    for name in ("MLContext", "dml", "pydml", "dmlFromFile", "matrix", "eval", "solve", "full", "seq",
                 "load", "getHopDAG", "convertToMatrixBlock", "convertToNumPyArr", "convertToPandasDF",
                 "getNumCols", "convert_caffemodel", "convertImageToNumPyArr", "getDatasetMean"):
        assert hasattr(sml, name), name
    from systemml.mllearn import LogisticRegression, LinearRegression, SVM, NaiveBayes, Caffe2DML, Keras2DML  # noqa
    from systemml import random  # noqa: F401
    assert sml.setSparkContext(None) is None


def test_random_sampling_distributions():
    from systemml_amd import random as R
    n = R.normal(loc=3, scale=2, size=(400, 50), seed=11).toNumPy()
    assert n.shape == (400, 50) and abs(n.mean() - 3) < 0.05 and abs(n.std() - 2) < 0.05
    u = R.uniform(low=-1, high=4, size=(300, 30), seed=12).toNumPy()
    assert u.min() >= -1 and u.max() <= 4 and abs(u.mean() - 1.5) < 0.1
    p = R.poisson(lam=4, size=(500, 20), seed=13).toNumPy()
    assert np.all(p == np.round(p)) and abs(p.mean() - 4) < 0.1 and abs(p.var() - 4) < 0.4
    s = R.normal(loc=5, scale=1, size=(200, 100), sparsity=0.3, seed=14).toNumPy()
    nz = (s != 0).mean()
    assert 0.25 < nz < 0.35 and abs(s[s != 0].mean() - 5) < 0.1
    with pytest.raises(TypeError):
        R.uniform(size=(3,))


def test_converters_roundtrip_and_images():
    import scipy.sparse as sp
    from systemml_amd.api import converters as CV
    a = np.arange(12.0).reshape(3, 4)
    np.testing.assert_array_equal(CV.convertToNumPyArr(CV.convertToMatrixBlock(None, a)), a)
    s = sp.random(50, 40, density=0.02, format="csr", random_state=0)
    np.testing.assert_allclose(CV.convertToNumPyArr(CV.convertToMatrixBlock(s)), s.toarray())
    df = CV.convertToPandasDF(a)
    assert list(df.columns) == ["C1", "C2", "C3", "C4"]
    ldf = CV.convertToLabeledDF(None, a, np.array([1, 2, 1]))
    assert list(ldf.columns) == ["features", "label"] and ldf["label"].tolist() == [1, 2, 1]
    img = np.arange(2 * 3 * 3, dtype=float).reshape(2, 3, 3)       # H x W x C
    rows = CV.convertImageToNumPyArr(img, add_rotated_images=True, add_mirrored_images=True)
    assert rows.shape == (5, 18)
    np.testing.assert_array_equal(rows[0], np.transpose(img, (2, 0, 1)).ravel())
    bgr = CV.convertImageToNumPyArr(img, color_mode="BGR", mean=[1, 2, 3])
    np.testing.assert_array_equal(bgr[0], np.transpose(img[:, :, ::-1] - [1, 2, 3], (2, 0, 1)).ravel())
    assert CV.getDatasetMean("VGG_ILSVRC_19_2014").shape == (3,)


# ---------------------------------------------------------------------------- caffemodel
def _vint(n):
    out = b""
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out += bytes([b | 0x80])
        else:
            return out + bytes([b])


def _fld(fno, wt, payload):
    key = _vint((fno << 3) | wt)
    if wt == 2:
        return key + _vint(len(payload)) + payload
    return key + payload


def _blob(arr):
    shape = b"".join(_vint(d) for d in arr.shape)
    return _fld(7, 2, _fld(1, 2, shape)) + _fld(5, 2, arr.astype("<f4").tobytes())


def _layer(name, typ, blobs):
    body = _fld(1, 2, name.encode()) + _fld(2, 2, typ.encode())
    for b in blobs:
        body += _fld(7, 2, _blob(b))
    return _fld(100, 2, body)


def test_convert_caffemodel(tmp_path):
    from systemml_amd.api import converters as CV
    from systemml_amd.io.readers import read_matrix
    rng = np.random.default_rng(0)
    Wc, bc = rng.standard_normal((4, 1, 3, 3)), rng.standard_normal(4)
    Wf, bf = rng.standard_normal((2, 36)), rng.standard_normal(2)
    net = _fld(1, 2, b"toy") + _layer("conv1", "Convolution", [Wc, bc]) + _layer("relu1", "ReLU", []) + \
        _layer("fc1", "InnerProduct", [Wf, bf])
    model = tmp_path / "toy.caffemodel"
    model.write_bytes(net)
    layers = CV.read_caffemodel(str(model))
    assert [(n, t, len(b)) for n, t, b in layers] == [("conv1", "Convolution", 2), ("fc1", "InnerProduct", 2)]
    out = tmp_path / "w"
    CV.convert_caffemodel(None, None, str(model), str(out), format="csv")
    np.testing.assert_allclose(read_matrix(str(out / "conv1_weight.mtx")).numpy(),
                               Wc.reshape(4, -1).astype(np.float32), rtol=1e-6)
    np.testing.assert_allclose(read_matrix(str(out / "conv1_bias.mtx")).numpy(), bc.reshape(4, 1).astype(np.float32),
                               rtol=1e-6)
    np.testing.assert_allclose(read_matrix(str(out / "fc1_weight.mtx")).numpy(), Wf.T.astype(np.float32), rtol=1e-6)
    np.testing.assert_allclose(read_matrix(str(out / "fc1_bias.mtx")).numpy(), bf.reshape(1, 2).astype(np.float32),
                               rtol=1e-6)


def test_get_hop_dag_dot():
    import systemml as sml
    s = sml.dml("Y = t(X) %*% X\nz = sum(Y)").input(X=np.ones((5, 3))).output("Y", "z")
    dot = sml.getHopDAG(sml.MLContext(), s, with_subgraph=True)
    assert dot.startswith("digraph") and "tsmm" in dot and "cluster_0" in dot
    raw = sml.getHopDAG(sml.MLContext(), s, apply_rewrites=False)
    assert "tsmm" not in raw and " t " not in raw
