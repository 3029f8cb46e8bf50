"""Column-wise cumulative aggregates on the chunked HIP scan (ops/hip/scan.hip) against fp64
PyTorch references: both thread mappings (narrow D < 64, wide D >= 64), single- and multi-chunk
row counts, NaN propagation of cummin / cummax, and the DML builtins end to end.  Reference
tests: test/integration/functions/aggregate/FullCumsumTest / FullCumprodTest / FullCumminTest /
FullCummaxTest."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REF = {
    "cumsum": lambda x: torch.cumsum(x, 0),
    "cumprod": lambda x: torch.cumprod(x, 0),
    "cummin": lambda x: torch.cummin(x, 0).values,
    "cummax": lambda x: torch.cummax(x, 0).values,
}


@pytest.mark.parametrize("shape", [(1, 1), (7, 3), (1023, 1), (1025, 5), (50000, 2), (3000, 64), (4097, 129),
                                   (20000, 1000), (33, 70000)])
@pytest.mark.parametrize("op", list(REF))
@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
def test_cumagg_kernel(op, shape, dt):
    from systemml_amd.ops import kernels as Kn
    g = torch.Generator().manual_seed(shape[0] * 7 + shape[1])
    X = torch.rand(shape, generator=g, dtype=torch.float64)
    if op == "cumprod":          # factors near 1 keep long products finite
        X = 1.0 + (X - 0.5) * 1e-3
    elif op == "cumsum":
        X = X - 0.5
    ref = REF[op](X)
    c0 = Kn.counters.get(op, 0)
    got = Kn.cumagg(op, X.to("cuda:0", dt)).double().cpu()
    assert Kn.counters[op] == c0 + 1
    if op in ("cummin", "cummax"):
        assert torch.equal(got, REF[op](X.to(dt).double()))
        return
    tol = 1e-12 if dt == torch.float64 else 2e-5 * max(1.0, shape[0] ** 0.5 / 10)
    scale = ref.abs().max().item() + 1e-30 if op == "cumsum" else 1.0
    err = (got - ref).abs().max().item() / scale
    assert err < tol, err


@pytest.mark.parametrize("shape", [(3000, 2), (5000, 100)])
def test_cummin_cummax_propagate_nan(shape):
    from systemml_amd.ops import kernels as Kn
    X = torch.rand(shape, dtype=torch.float64)
    X[1500, 0] = float("nan")
    for op in ("cummin", "cummax", "cumsum"):
        got = Kn.cumagg(op, X.cuda()).cpu()
        ref = REF[op](X)
        assert torch.equal(torch.isnan(got), torch.isnan(ref)), op
        np.testing.assert_allclose(got[~torch.isnan(ref)], ref[~torch.isnan(ref)], rtol=1e-10)


def test_cumulative_builtins_run_on_the_scan_kernel():
    from systemml_amd.api.executor import run
    from systemml_amd.conf import DMLConfig
    from systemml_amd.ops import kernels as Kn
    src = "a = cumsum(X)\nb = cumprod(X)\nc = cummin(X)\nd = cummax(X)\n"
    X = np.random.default_rng(2).random((4000, 40)) + 0.5
    c0 = dict(Kn.counters)
    res = run(src, inputs={"X": X}, outputs=list("abcd"), config=DMLConfig(gpu=True, gpu_min_cells=0),
              out=lambda s: None)
    for k, f in zip("abcd", (np.cumsum, np.cumprod, np.minimum.accumulate, np.maximum.accumulate)):
        got = np.asarray(res[k].double().cpu() if isinstance(res[k], torch.Tensor) else res[k])
        np.testing.assert_allclose(got, f(X, axis=0), rtol=1e-9)
    for op in REF:
        assert Kn.counters.get(op, 0) > c0.get(op, 0), op
