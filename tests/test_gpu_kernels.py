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
    cnt = lambda: sum(v for k, v in kernels.counters.items() if k.endswith("mmchain.XtXv"))
    before = cnt()
    res = run("q = t(X) %*% (X %*% w)", inputs={"X": X, "w": w}, outputs=["q"], config=gpu_config)
    after = cnt()
    assert after == before + 1
    np.testing.assert_allclose(res["q"].cpu().double().numpy(), X.T @ (X @ w), rtol=1e-4)


# ---------------------------------------------------------------------------
# MFMA chain kernels (ops/hip/mfma_chain.hip): exact small-integer data first (catches any
# operand/accumulator layout slip, which would show up as a wrong element, not rounding),
# then random data against an fp64 reference.
# ---------------------------------------------------------------------------
@pytest.fixture
def mfma_all(K):
    """Route every eligible op (incl. the fused chains) through the MFMA kernel."""
    K.MFMA_ALL = True
    K.CHAIN4 = False
    yield
    K.MFMA_ALL = False
    K.CHAIN4 = True


def _ints(shape, lo, hi, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randint(lo, hi + 1, shape, generator=g, device="cuda").to(torch.float64)


@pytest.mark.parametrize("n", [1, 15, 17, 4099])
@pytest.mark.parametrize("d", [8, 136, 256, 264, 1000])
@pytest.mark.parametrize("k", [1, 2, 3, 4])
def test_mfma_exact_integer_layout(K, n, d, k, mfma_all):
    x = _ints((n, d), -3, 3, 10 + d).to(torch.bfloat16)
    x64 = x.double()
    v = _ints((d, k), -2, 2, 20 + k)
    g = _ints((n, k), -2, 2, 30 + n)
    c0 = dict(K.counters)
    u = K.xv(x, v)
    torch.testing.assert_close(u.double(), x64 @ v, rtol=0, atol=0)
    r = K.xtg(x, g)
    torch.testing.assert_close(r.double(), x64.t() @ g, rtol=0, atol=0)
    r2 = K.mmchain("XtXv", x, v)
    torch.testing.assert_close(r2.double(), x64.t() @ (x64 @ v), rtol=0, atol=0)
    r3 = K.mmchain("XtXvy", x, v, g)
    torch.testing.assert_close(r3.double(), x64.t() @ (x64 @ v - g), rtol=0, atol=0)
    assert K.counters.get("mfma.xv", 0) > c0.get("mfma.xv", 0)
    assert K.counters.get("mfma.xtg", 0) > c0.get("mfma.xtg", 0)
    assert K.counters.get("mfma.mmchain.XtXv", 0) > c0.get("mfma.mmchain.XtXv", 0)


@pytest.mark.parametrize("n", [1, 17, 4099])
@pytest.mark.parametrize("d", [8, 264, 1000, 1024])
@pytest.mark.parametrize("k", [5, 9, 16])
def test_wide_mfma_exact_integer_layout(K, n, d, k):
    """5..16-column products (wide_kernel: planes as separate MFMAs, columns in the tile's M / N
    dimension) are exact on small integers: any layout slip shows as a wrong element."""
    x = _ints((n, d), -3, 3, 40 + d).to(torch.bfloat16)
    x64 = x.double()
    v = _ints((d, k), -2, 2, 50 + k)
    g = _ints((n, k), -2, 2, 60 + n)
    c0 = dict(K.counters)
    torch.testing.assert_close(K.xv(x, v).double(), x64 @ v, rtol=0, atol=0)
    torch.testing.assert_close(K.xtg(x, g).double(), x64.t() @ g, rtol=0, atol=0)
    assert K.counters.get("mfma.xv_wide", 0) > c0.get("mfma.xv_wide", 0)
    assert K.counters.get("mfma.xtg_wide", 0) > c0.get("mfma.xtg_wide", 0)


@pytest.mark.parametrize("n", [1, 17, 4099])
@pytest.mark.parametrize("d", [8, 264, 1000])
@pytest.mark.parametrize("k", [5, 9, 16])
@pytest.mark.parametrize("ctype", ["XtXv", "XtwXv", "XtXvy", "XtPSXv"])
def test_wide_mfma_chains(K, n, d, k, ctype):
    """Fused wide chains t(X) %*% g(X %*% V) (one pass over X, 16-wave blocks at D > 768) on
    small integers: exact up to fp32 accumulation of the final products."""
    x = _ints((n, d), -2, 2, 70 + d).to(torch.bfloat16)
    x64 = x.double()
    v = _ints((d, k), -1, 1, 80 + k)
    u = x64 @ v
    w = None
    if ctype == "XtXv":
        g = u
    elif ctype == "XtwXv":
        w = _ints((n, 1), -2, 2, 90)
        g = w * u
    elif ctype == "XtXvy":
        w = _ints((n, k), -2, 2, 91)
        g = u - w
    else:
        w = _ints((n, k + 1), -1, 1, 92)[:, :k]          # strided view, like P[, 1:K]
        q = w * u
        g = q - w * q.sum(1, keepdim=True)
    ref = x64.t() @ g
    c0 = K.counters.get("mfma.mmchain_wide." + ctype, 0)
    r = K.mmchain(ctype, x, v, w)
    assert K.counters.get("mfma.mmchain_wide." + ctype, 0) == c0 + 1
    err = (r.double() - ref).abs().max().item() / max(ref.abs().max().item(), 1.0)
    assert err < 1e-6, err


@pytest.mark.parametrize("k", [6, 10, 16])
def test_wide_mfma_fp32_operands(K, k):
    """fp32 V / G are split into three bf16 planes: products match fp64 to fp32 accuracy, and
    `%*%` routes 10-column shapes (10-class MultiLogReg) to the wide kernel."""
    n, d = 30011, 1000
    x = _mk(n, d, torch.bfloat16, seed=7)
    x64 = x.double()
    v = torch.randn((d, k), device="cuda", dtype=torch.float64)
    g = torch.randn((n, k), device="cuda", dtype=torch.float64)
    u = K.try_mm(x, v, False)
    ref = x64 @ v
    assert (u.double() - ref).abs().max().item() / ref.abs().max().item() < 2e-6
    r = K.try_mm(x, g, True)
    ref2 = x64.t() @ g
    assert (r.double() - ref2).abs().max().item() / ref2.abs().max().item() < 2e-6


@pytest.mark.parametrize("ctype", ["XtXv", "XtwXv", "XtXvy", "XtPSXv"])
@pytest.mark.parametrize("k", [1, 2, 4])
def test_mfma_matches_rowstream(K, ctype, k, mfma_all):
    n, d = 50001, 1000
    x = _mk(n, d, torch.bfloat16, seed=7)
    x64 = x.double()
    v = torch.randn((d, k), device="cuda", dtype=torch.float64)
    w = None
    if ctype == "XtwXv":
        w = torch.rand((n, 1), device="cuda", dtype=torch.float64)
    elif ctype == "XtXvy":
        w = torch.randn((n, k), device="cuda", dtype=torch.float64)
    elif ctype == "XtPSXv":
        w = torch.softmax(torch.randn((n, k + 1), device="cuda", dtype=torch.float64), 1)[:, :k].contiguous()
    u = x64 @ v
    if ctype == "XtXv":
        g = u
    elif ctype == "XtwXv":
        g = w * u
    elif ctype == "XtXvy":
        g = u - w
    else:
        q = w * u
        g = q - w * q.sum(1, keepdim=True)
    ref = x64.t() @ g
    assert K._mfma_ok(x, k)
    r_m = K.mmchain(ctype, x, v, w)
    K.MFMA = False
    try:
        r_v = K.mmchain(ctype, x, v, w)
    finally:
        K.MFMA = True
    scale = ref.abs().max().item()
    err_m = (r_m.double() - ref).abs().max().item() / scale
    err_v = (r_v.double() - ref).abs().max().item() / scale
    # the split-bf16 MFMA path must be as accurate as the fp32 VALU path
    assert err_m < max(2e-5, 2 * err_v), (err_m, err_v)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("d", [1000, 512, 64])
@pytest.mark.parametrize("k", [4, 3, 2])
def test_smgrad_fused_softmax_gradient(K, dt, d, k):
    """Mode XTSMG: U = X V and t(X) (softmax([U, 0])[:, :k] - Y) in one pass vs fp64 torch."""
    n = 30011
    x = _mk(n, d, dt, seed=5)
    x64 = x.double()
    v = torch.randn((d, k), device="cuda", dtype=torch.float64) * 0.05
    lab = torch.randint(0, k + 1, (n,), device="cuda")
    y = torch.nn.functional.one_hot(lab, k + 1)[:, :k].double()
    r = K.smgrad(x, v, y)
    assert r is not None
    u, g = r
    u_ref = x64 @ v
    lt = torch.cat([u_ref, torch.zeros((n, 1), device="cuda", dtype=torch.float64)], 1)
    p = torch.softmax(lt, dim=1)[:, :k]
    g_ref = x64.t() @ (p - y)
    assert (u.double() - u_ref).abs().max().item() <= 2e-4 * u_ref.abs().max().item()
    assert (g.double() - g_ref).abs().max().item() <= 2e-4 * g_ref.abs().max().item()
    assert K.counters.get("rowstream.smgrad", 0) + K.counters.get("chain4.smgrad", 0) > 0


# ---------------------------------------------------------------------------
# Row-group chain kernels (ops/hip/chain4.hip): exact small-integer data through every mode,
# ragged row counts (partial groups / blocks) and D not a multiple of 64.
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("n", [1, 15, 17, 4099, 50001])
@pytest.mark.parametrize("d", [8, 136, 512, 520, 1000])
@pytest.mark.parametrize("k", [1, 2, 3, 4])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_chain4_exact_integer(K, n, d, k, dt):
    x = _ints((n, d), -3, 3, 11 + d).to(dt)
    x64 = x.double()
    v = _ints((d, k), -2, 2, 21 + k)
    g = _ints((n, k), -2, 2, 31 + n)
    w = _ints((n, 1), 0, 3, 41 + n)
    u64 = x64 @ v
    c0 = dict(K.counters)
    torch.testing.assert_close(K.mmchain("XtXv", x, v).double(), x64.t() @ u64, rtol=0, atol=0)
    torch.testing.assert_close(K.mmchain("XtXvy", x, v, g).double(), x64.t() @ (u64 - g), rtol=0, atol=0)
    torch.testing.assert_close(K.mmchain("XtwXv", x, v, w).double(), x64.t() @ (w * u64), rtol=0, atol=0)
    q = g * u64
    ref = x64.t() @ (q - g * q.sum(1, keepdim=True))
    torch.testing.assert_close(K.mmchain("XtPSXv", x, v, g).double(), ref, rtol=0, atol=0)
    used = sum(v_ - c0.get(k_, 0) for k_, v_ in K.counters.items() if k_.startswith("chain4."))
    if k > 1:
        assert used >= 3


@pytest.mark.parametrize("n", [2065, 4099, 300001])
@pytest.mark.parametrize("k", [1, 2, 3, 4])
def test_chain4_softmax_gradient(K, n, k):
    d = 1000
    x = _mk(n, d, torch.bfloat16, seed=5)
    x64 = x.double()
    g0 = torch.Generator(device="cuda").manual_seed(3)
    v = torch.randn((d, k), generator=g0, device="cuda", dtype=torch.float64) * 0.05
    y = (torch.rand((n, k), generator=g0, device="cuda") < 0.3).double()
    c0 = K.counters.get("chain4.smgrad", 0)
    U, G = K.smgrad(x, v.float(), y.float())
    assert K.counters.get("chain4.smgrad", 0) == c0 + 1
    u64 = x64 @ v
    lt = torch.cat([u64, torch.zeros((n, 1), device="cuda", dtype=torch.float64)], 1)
    p = torch.softmax(lt, 1)[:, :k]
    G64 = x64.t() @ (p - y)
    torch.testing.assert_close(U.double(), u64, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(G.double(), G64, rtol=2e-4, atol=2e-3 * G64.abs().max().item())


@pytest.mark.parametrize("ctype", ["XtPSXv", "XtwXv", "XtXvy"])
@pytest.mark.parametrize("n,d", [(70001, 1000), (4099, 512), (513, 136)])
def test_chain4m_matrix_core_matches_valu(K, ctype, n, d):
    """chain4m (both products on 4x4x4 bf16 MFMAs, V / G as exact three-plane bf16 splits) is as
    accurate as the fp32 VALU row-group kernel against an fp64 reference, on random data."""
    x = _mk(n, d, torch.bfloat16, seed=9)
    x64 = x.double()
    g0 = torch.Generator(device="cuda").manual_seed(4)
    v = torch.randn((d, 4), generator=g0, device="cuda") * 0.05
    w = torch.rand((n, 1 if ctype == "XtwXv" else 4), generator=g0, device="cuda")
    u = x64 @ v.double()
    w64 = w.double()
    if ctype == "XtPSXv":
        q = w64 * u
        ref = x64.t() @ (q - w64 * q.sum(1, keepdim=True))
    elif ctype == "XtwXv":
        ref = x64.t() @ (w64 * u)
    else:
        ref = x64.t() @ (u - w64)
    old = K.C4M
    try:
        c0 = K.counters.get("chain4m", 0)
        K.C4M = True
        r_m = K.mmchain(ctype, x, v, w)
        assert K.counters.get("chain4m", 0) == c0 + 1
        K.C4M = False
        r_v = K.mmchain(ctype, x, v, w)
    finally:
        K.C4M = old
    scale = ref.abs().max().item()
    err_m = (r_m.double() - ref).abs().max().item() / scale
    err_v = (r_v.double() - ref).abs().max().item() / scale
    assert err_m < max(2e-5, 2 * err_v), (err_m, err_v)


@pytest.mark.parametrize("n,d,k", [(70001, 1000, 4), (4099, 512, 3), (30011, 136, 2), (5003, 1000, 1)])
def test_chain4m_softmax_objective(K, n, d, k):
    """XTSMGO (compiler op smobj): probabilities, gradient and the two objective terms of the
    multinomial-logreg candidate point in one pass, vs an fp64 reference."""
    x = _mk(n, d, torch.bfloat16, seed=7)
    x64 = x.double()
    g0 = torch.Generator(device="cuda").manual_seed(6)
    v = torch.randn((d, k), generator=g0, device="cuda") * 0.05
    lab = torch.randint(0, k + 1, (n,), device="cuda", generator=g0)
    y = torch.nn.functional.one_hot(lab, k + 1).float()
    r = K.smobj(x, v, y)
    assert r is not None
    P, G, s1, s2 = r
    L = torch.cat([x64 @ v.double(), torch.zeros((n, 1), device="cuda", dtype=torch.float64)], 1)
    LT = L - L.max(1, keepdim=True).values
    E = torch.exp(LT)
    P64 = E / E.sum(1, keepdim=True)
    G64 = x64.t() @ (P64[:, :k] - y.double()[:, :k])
    torch.testing.assert_close(P.double(), P64, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(G.double(), G64, rtol=2e-4, atol=2e-4 * G64.abs().max().item())
    r1 = (y.double() * LT).sum().item()
    r2 = torch.log(E.sum(1)).sum().item()
    assert abs(s1 - r1) <= 1e-4 * max(1.0, abs(r1)), (s1, r1)
    assert abs(s2 - r2) <= 1e-4 * max(1.0, abs(r2)), (s2, r2)


@pytest.mark.parametrize("n,d,k", [(70001, 1000, 9), (4099, 512, 15), (30011, 136, 5), (2053, 1024, 7)])
def test_wide_softmax_objective_and_gradient(K, n, d, k):
    """Wide softmax modes (5..15 classes + the zero class, e.g. the 10-class MultiLogReg):
    XTSMGO probabilities / gradient / objective terms and XTSMG (U, gradient) vs fp64."""
    x = _mk(n, d, torch.bfloat16, seed=8)
    x64 = x.double()
    g0 = torch.Generator(device="cuda").manual_seed(9)
    v = torch.randn((d, k), generator=g0, device="cuda") * 0.05
    lab = torch.randint(0, k + 1, (n,), device="cuda", generator=g0)
    y = torch.nn.functional.one_hot(lab, k + 1).float()
    c0 = dict(K.counters)
    P, G, s1, s2 = K.smobj(x, v, y)
    U64 = x64 @ v.double()
    L = torch.cat([U64, torch.zeros((n, 1), device="cuda", dtype=torch.float64)], 1)
    LT = L - L.max(1, keepdim=True).values
    E = torch.exp(LT)
    P64 = E / E.sum(1, keepdim=True)
    G64 = x64.t() @ (P64[:, :k] - y.double()[:, :k])
    torch.testing.assert_close(P.double(), P64, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(G.double(), G64, rtol=2e-4, atol=2e-4 * G64.abs().max().item())
    r1 = (y.double() * LT).sum().item()
    r2 = torch.log(E.sum(1)).sum().item()
    assert abs(s1 - r1) <= 1e-4 * max(1.0, abs(r1)), (s1, r1)
    assert abs(s2 - r2) <= 1e-4 * max(1.0, abs(r2)), (s2, r2)
    U, G2 = K.smgrad(x, v, y[:, :k])
    torch.testing.assert_close(U.double(), U64, rtol=1e-5, atol=1e-5 * U64.abs().max().item())
    torch.testing.assert_close(G2.double(), G64, rtol=2e-4, atol=2e-4 * G64.abs().max().item())
    assert K.counters.get("mfma.smobj_wide", 0) == c0.get("mfma.smobj_wide", 0) + 1
    assert K.counters.get("mfma.smgrad_wide", 0) == c0.get("mfma.smgrad_wide", 0) + 1
