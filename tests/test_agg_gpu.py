"""Wide column sums on the generated column-aggregate kernel (ops/core.py agg -> ops/cell.py,
fp64 accumulation) against fp64 torch, including bf16-stored and ragged shapes.  Reference
test: test/integration/functions/aggregate/ColSumTest."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(2, 2048), (256, 12544), (77, 5001), (3000, 4096)])
@pytest.mark.parametrize("dt", [torch.float32, torch.float64, torch.bfloat16])
def test_wide_colsums_on_cell_kernel(shape, dt):
    from systemml_amd.conf import DMLConfig
    from systemml_amd.ops import core as C, kernels
    from systemml_amd.ops.backend import backend
    backend.configure(DMLConfig(gpu=True, precision="double" if dt == torch.float64 else "single"))
    g = torch.Generator().manual_seed(shape[0] + shape[1])
    X = torch.randn(shape, generator=g, dtype=torch.float64)
    Xd = X.to("cuda:0", dt)
    c0 = kernels.counters.get("cell", 0)
    got = C.agg("sum", "col", Xd)
    assert kernels.counters.get("cell", 0) == c0 + 1
    assert tuple(got.shape) == (1, shape[1])
    ref = Xd.double().cpu().sum(0, keepdim=True)
    tol = 1e-12 if dt == torch.float64 else 1e-5
    torch.testing.assert_close(got.double().cpu(), ref, rtol=tol, atol=tol * shape[0] ** 0.5)


# ----------------------------------------------------------------------------- ops/hip/agg.hip
def _ref(o, d, X):
    dim = None if d == "all" else (1 if d == "row" else 0)
    kw = {} if dim is None else {"dim": dim, "keepdim": True}
    if o == "sum":
        return X.sum(**kw)
    if o == "sumsq":
        return (X * X).sum(**kw)
    if o == "mean":
        return X.mean(**kw)
    if o == "prod":
        return X.prod(**kw)
    if o == "min":
        return X.amin(**kw) if dim is not None else X.min()
    if o == "max":
        return X.amax(**kw) if dim is not None else X.max()
    if o in ("var", "sd"):
        # DML: the variance of a single value is 0 (ops/core._var)
        n = X.numel() if dim is None else X.shape[dim]
        if n <= 1:
            return torch.zeros(X.sum(**kw).shape, dtype=X.dtype)
        v = X.var(**kw) if dim is not None else X.var()
        return v if o == "var" else v.sqrt()
    xf = torch.flip(X, dims=[1])
    idx = torch.argmax(xf, 1, keepdim=True) if o == "imax" else torch.argmin(xf, 1, keepdim=True)
    return (X.shape[1] - idx).double()


@pytest.mark.parametrize("o", ["sum", "sumsq", "mean", "min", "max", "prod", "var", "sd", "imax", "imin"])
@pytest.mark.parametrize("d", ["all", "row", "col"])
@pytest.mark.parametrize("shape", [(1, 1), (7, 3), (1000, 1), (300, 70), (40000, 5), (17, 1001)])
def test_agg_kernel_matches_fp64(o, d, shape):
    """Every aggregate x direction on agg.hip against fp64 torch on the same (fp32) values; the
    index aggregates return the last extreme column (ties forced by rounding to 1/8)."""
    if o in ("imax", "imin") and d != "row":
        pytest.skip("index aggregates are row-wise")
    from systemml_amd.conf import DMLConfig
    from systemml_amd.ops import core as C, kernels
    from systemml_amd.ops.backend import backend
    backend.configure(DMLConfig(gpu=True, precision="single"))
    g = torch.Generator().manual_seed(shape[0] * 31 + shape[1])
    X = torch.randn(shape, generator=g, dtype=torch.float64)
    if o == "prod":
        X = 1.0 + 0.01 * X
    if o in ("imax", "imin"):
        X = torch.round(X * 8) / 8
    Xd = X.to("cuda:0", torch.float32)
    before = kernels.counters.get("agg." + o, 0)
    got = C.agg(o, d, Xd)
    # sum / sumsq over all cells, and sumsq of large matrices, keep their existing kernels
    fused = (d == "all" and o in ("sum", "sumsq")) or (o == "sumsq" and X.numel() >= 1 << 16)
    if not fused:
        assert kernels.counters.get("agg." + o, 0) == before + 1
    ref = _ref(o, d, Xd.double().cpu())
    got = torch.as_tensor(got, dtype=torch.float64).cpu() if not isinstance(got, torch.Tensor) else got.double().cpu()
    if d != "all":
        assert tuple(got.shape) == tuple(ref.shape)
    tol = 1e-4 if fused else 2e-6              # those accumulate in fp32
    torch.testing.assert_close(got.reshape(ref.shape), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float64])
def test_agg_kernel_storage_types_and_nan(dt):
    from systemml_amd.conf import DMLConfig
    from systemml_amd.ops import core as C
    from systemml_amd.ops.backend import backend
    backend.configure(DMLConfig(gpu=True, precision="double" if dt == torch.float64 else "single"))
    X = torch.randn(513, 129, dtype=torch.float64)
    X[7, 5] = float("nan")
    Xd = X.to("cuda:0", dt)
    Xr = Xd.double().cpu()
    for o, d in (("max", "row"), ("min", "col"), ("var", "col"), ("mean", "row"), ("max", "all")):
        got = C.agg(o, d, Xd)
        got = torch.as_tensor(got, dtype=torch.float64) if not isinstance(got, torch.Tensor) else got.double().cpu()
        ref = _ref(o, d, Xr)
        tol = 1e-9 if dt == torch.float64 else 1e-6        # fp32 results for bf16 storage
        torch.testing.assert_close(got.reshape(ref.shape), ref, rtol=tol, atol=tol, equal_nan=True)


@pytest.mark.parametrize("o", ["sum", "sumsq", "mean"])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(5000, 64), (3001, 1000), (9, 128), (70000, 512)])
def test_column_aggregate_16b_loads(o, dt, shape):
    """agg.hip col_vec (16-B loads of 8 bf16 / 4 fp32 columns, fp64 accumulation) against fp64."""
    from systemml_amd.ops import kernels
    kernels.load(required=True)
    g = torch.Generator().manual_seed(shape[0] + shape[1])
    X = torch.randn(shape, generator=g, dtype=torch.float64).to("cuda:0", dt)
    got = kernels.agg(o, "col", X)
    Xr = X.double().cpu()
    ref = {"sum": Xr.sum(0), "sumsq": (Xr * Xr).sum(0), "mean": Xr.mean(0)}[o].reshape(1, -1)
    torch.testing.assert_close(got.double().cpu().reshape(ref.shape), ref, rtol=1e-6, atol=1e-6)   # fp32 result
