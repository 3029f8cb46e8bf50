"""Numerics of the HIP row-streaming kernels vs a plain PyTorch fp64 reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from systemml_amd.ops import kernels
    from systemml_amd.ops.backend import backend
    from systemml_amd.conf import DMLConfig
    backend.configure(DMLConfig(precision="single"))
    kernels.load(required=True)
    return kernels


def _mk(n, d, dt, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.rand((n, d), generator=g, device="cuda", dtype=torch.float64) * 2 - 1
    return x.to(dt)


TOL = {torch.bfloat16: 2e-4, torch.float32: 2e-4, torch.float64: 1e-10}


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32, torch.float64])
@pytest.mark.parametrize("d", [1000, 512, 37, 1024])
@pytest.mark.parametrize("k", [1, 3, 4, 8])
def test_xv_xtg(K, dt, d, k):
    n = 20011
    x = _mk(n, d, dt)
    x64 = x.double()
    v = torch.randn((d, k), device="cuda", dtype=torch.float64)
    u = K.xv(x, v)
    ref = x64 @ v
    assert u is not None
    err = (u.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < TOL[dt], err
    g = torch.randn((n, k), device="cuda", dtype=torch.float64)
    r = K.xtg(x, g)
    ref2 = x64.t() @ g
    err2 = (r.double() - ref2).abs().max().item() / ref2.abs().max().item()
    assert err2 < TOL[dt], err2


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32, torch.float64])
@pytest.mark.parametrize("ctype", ["XtXv", "XtwXv", "XtXvy", "XtPSXv"])
@pytest.mark.parametrize("k", [1, 4, 5])
def test_mmchain(K, dt, ctype, k):
    n, d = 30000, 1000
    x = _mk(n, d, dt, seed=1)
    x64 = x.double()
    v = torch.randn((d, k), device="cuda", dtype=torch.float64)
    w = None
    u = x64 @ v
    if ctype == "XtXv":
        g = u
    elif ctype == "XtwXv":
        w = torch.rand((n, 1), device="cuda", dtype=torch.float64)
        g = w * u
    elif ctype == "XtXvy":
        w = torch.randn((n, k), device="cuda", dtype=torch.float64)
        g = u - w
    else:
        w = torch.softmax(torch.randn((n, k + 1), device="cuda", dtype=torch.float64), 1)[:, :k].contiguous()
        q = w * u
        g = q - w * q.sum(1, keepdim=True)
    ref = x64.t() @ g
    from systemml_amd.ops import core as C
    r = C.mmchain(ctype, x, v, w)   # dispatch: fused kernel, or XV + XTG passes where unsupported
    err = (r.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < TOL[dt] * 5, err


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_sumsq(K, dt):
    x = _mk(50000, 1000, dt, seed=2)
    x64 = x.double()
    r = K.sumsq(x, "row")
    assert (r.double() - (x64 * x64).sum(1, keepdim=True)).abs().max().item() < 1e-2
    c = K.sumsq(x, "col")
    ref = (x64 * x64).sum(0, keepdim=True)
    assert ((c.double() - ref).abs() / ref).max().item() < 1e-4
    a = K.sumsq(x, "all")
    assert abs(a - float((x64 * x64).sum())) / float((x64 * x64).sum()) < 1e-5


def test_dml_uses_fused_kernels(gpu_config):
    import numpy as np
    from systemml_amd.api.executor import run
    from systemml_amd.ops import kernels
    X = np.random.rand(10000, 50)
    w = np.random.rand(50, 1)
    before = kernels.counters.get("rowstream.mmchain.XtXv", 0)
    res = run("q = t(X) %*% (X %*% w)", inputs={"X": X, "w": w}, outputs=["q"], config=gpu_config)
    after = kernels.counters.get("rowstream.mmchain.XtXv", 0)
    assert after == before + 1
    np.testing.assert_allclose(res["q"].cpu().double().numpy(), X.T @ (X @ w), rtol=1e-4)
