"""Compressed linear algebra (reference: test/integration/functions/compress/* compare
compressed vs uncompressed results of the same operations)."""
import numpy as np
import pytest
import torch

from systemml_amd.api.executor import run
from systemml_amd.api.mlcontext import SCRIPTS_DIR
from systemml_amd.conf import DMLConfig
from systemml_amd.ops import compress as CMP


def _data(n=6000, seed=0):
    rng = np.random.default_rng(seed)
    cat = rng.integers(0, 5, (n, 6)).astype(float)            # low-cardinality columns (compress)
    flags = (rng.random((n, 4)) < 0.3).astype(float)
    cont = rng.standard_normal((n, 2))                        # incompressible columns
    return np.hstack([cat, flags, cont, cat[:, :2] * 2 + 1])


def test_compress_roundtrip_and_ops():
    X = torch.from_numpy(_data())
    C = CMP.compress(X, force=True)
    assert CMP.is_compressed(C) and C.ratio() > 2
    assert torch.equal(C.decompress(), X)
    V = torch.randn(X.shape[1], 3, dtype=torch.float64)
    Y = torch.randn(X.shape[0], 2, dtype=torch.float64)
    torch.testing.assert_close(C.matmul(V), X @ V)
    torch.testing.assert_close(C.tmatmul(Y), X.t() @ Y)
    torch.testing.assert_close(C.colsums(), X.sum(0, keepdim=True))
    torch.testing.assert_close(C.rowsums(sq=True), (X * X).sum(1, keepdim=True))
    torch.testing.assert_close(C.scale(2.0).decompress(), 2 * X)


@pytest.mark.parametrize("mode", ["true", "auto"])
def test_compressed_linalg_in_dml(mode):
    X = _data(n=80000, seed=1)
    y = X @ np.linspace(-1, 1, X.shape[1]).reshape(-1, 1) + 0.01
    dense = DMLConfig(gpu=False)
    comp = DMLConfig(gpu=False, compressed_linalg=mode)
    src = open(f"{SCRIPTS_DIR}/algorithms/LinearRegCG.dml").read()
    args = dict(X="X", Y="y", B="B", icpt=0, reg=1e-6, tol=1e-12, maxi=100)
    r1 = run(src, args=args, inputs={"X": X, "y": y}, outputs=["beta"], config=dense, out=lambda s: None)
    r2 = run(src, args=args, inputs={"X": X, "y": y}, outputs=["beta"], config=comp, out=lambda s: None)
    np.testing.assert_allclose(r2["beta"].numpy(), r1["beta"].numpy(), rtol=1e-8, atol=1e-10)
    r3 = run("s = sum(X); cs = colSums(X); rs = rowSums(X); Z = X * 3; z = sum(Z ^ 2); e = sum(exp(X))",
             inputs={"X": X}, outputs=["s", "cs", "rs", "z", "e", "X"], config=comp)
    assert CMP.is_compressed(r3["X"])
    np.testing.assert_allclose(r3["s"], X.sum())
    np.testing.assert_allclose(r3["cs"].numpy().ravel(), X.sum(0))
    np.testing.assert_allclose(r3["rs"].numpy().ravel(), X.sum(1))
    np.testing.assert_allclose(r3["z"], (9 * X ** 2).sum())
    np.testing.assert_allclose(r3["e"], np.exp(X).sum())


def _sparse_sorted_data(n=20000, seed=2):
    """Columns where OLE / RLE win: mostly-zero flags (OLE) and sorted category runs (RLE)."""
    rng = np.random.default_rng(seed)
    flags = (rng.random((n, 3)) < 0.02) * rng.integers(1, 4, (n, 3))
    runs = np.sort(rng.integers(0, 6, (n, 2)), axis=0).astype(float)
    dense_cat = rng.integers(1, 5, (n, 2)).astype(float)
    return np.hstack([flags.astype(float), runs, dense_cat])


@pytest.mark.parametrize("kinds", [("ddc",), ("ole",), ("rle",), None])
def test_encodings_roundtrip_and_ops(kinds):
    """Every column-group encoding (reference ColGroupDDC / OLE / RLE) gives the dense results
    of decompress, X %*% V, t(X) %*% Y, row / column sums and scaling."""
    X = torch.from_numpy(_sparse_sorted_data())
    C = CMP.compress(X, force=True, kinds=kinds)
    assert CMP.is_compressed(C)
    if kinds is not None:
        assert set(C.kinds()) <= set(kinds) | {"unc"}, C.kinds()
    assert torch.equal(C.decompress(), X)
    V = torch.randn(X.shape[1], 3, dtype=torch.float64)
    Y = torch.randn(X.shape[0], 2, dtype=torch.float64)
    torch.testing.assert_close(C.matmul(V), X @ V)
    torch.testing.assert_close(C.tmatmul(Y), X.t() @ Y)
    torch.testing.assert_close(C.colsums(), X.sum(0, keepdim=True))
    torch.testing.assert_close(C.colsums(sq=True), (X * X).sum(0, keepdim=True))
    torch.testing.assert_close(C.rowsums(), X.sum(1, keepdim=True))
    torch.testing.assert_close(C.scale(-1.5).decompress(), -1.5 * X)
    assert torch.isnan(C.scale(float("inf")).decompress() if CMP.is_compressed(C.scale(float("inf")))
                       else C.scale(float("inf"))).any() == bool((X == 0).any())


def test_planner_picks_smallest_encoding():
    """Sparse flag columns plan as OLE, sorted runs as RLE, dense categories as DDC; the
    compressed size beats DDC-only coding."""
    X = torch.from_numpy(_sparse_sorted_data())
    C = CMP.compress(X, force=True)
    kinds = C.kinds()
    assert kinds.get("ole", 0) + kinds.get("rle", 0) >= 1, kinds
    assert C.nbytes() < CMP.compress(X, force=True, kinds=("ddc",)).nbytes()


@pytest.mark.gpu
@pytest.mark.parametrize("kinds", [("ddc",), ("ole",), ("rle",)])
def test_encodings_on_gpu(kinds):
    """The compressed operators run in HBM (dictionary products, gathers and scatter-adds on
    the MI355X) and agree with the dense fp64 results."""
    X = torch.from_numpy(_sparse_sorted_data(n=50000)).cuda()
    C = CMP.compress(X, force=True, kinds=kinds)
    assert CMP.is_compressed(C) and C.device.type == "cuda"
    assert torch.equal(C.decompress(), X)
    V = torch.randn(X.shape[1], 4, dtype=torch.float64, device="cuda")
    Y = torch.randn(X.shape[0], 3, dtype=torch.float64, device="cuda")
    torch.testing.assert_close(C.matmul(V), X @ V)
    torch.testing.assert_close(C.tmatmul(Y), X.t() @ Y)
    torch.testing.assert_close(C.rowsums(sq=True), (X * X).sum(1, keepdim=True))
