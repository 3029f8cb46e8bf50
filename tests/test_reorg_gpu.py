"""reorg.hip / sort.hip: right indexing, casts, transpose, lower/upper.tri, row gathers, CSR
windows and the device radix sort behind order() / quantiles, each against a plain PyTorch
reference of the same op (fp32 / fp64 exact: these kernels copy or convert cells)."""
import numpy as np
import pytest
import torch

from systemml_amd.ops.kernels import _rowpitch

pytestmark = pytest.mark.gpu

DT = [torch.bfloat16, torch.float32, torch.float64]


def test_fastdiv_host_model():
    """The multiply-high division copy_flat uses (n / d for n < 2^31), modelled on the host."""
    rng = np.random.default_rng(0)
    for d in [1, 2, 3, 5, 7, 11, 63, 64, 100, 1000, 4097]:
        s = 0
        while (1 << s) < d:
            s += 1
        m = ((1 << 32) * ((1 << s) - d)) // d + 1
        ns = np.concatenate([rng.integers(0, 2 ** 31 - 1, 2000), np.arange(0, 3 * d), [2 ** 31 - 1]])
        for n in ns.tolist():
            assert (((n * m) >> 32) + n) >> s == n // d, (n, d)


@pytest.mark.parametrize("tin", DT)
@pytest.mark.parametrize("tout", DT)
@pytest.mark.parametrize("shape,win", [((1000, 7), (slice(3, 900), slice(1, 6))),
                                       ((300, 517), (slice(10, 250), slice(5, 500))),
                                       ((64, 64), (slice(0, 64), slice(0, 64)))])
def test_copy2d_window_and_cast(tin, tout, shape, win):
    from systemml_amd.ops import kernels
    x = torch.randn(shape, device="cuda", dtype=torch.float64).to(tin)
    v = x[win]
    r = kernels.copy2d(v, tout)
    assert r is not None and r.is_contiguous() and r.dtype == tout
    torch.testing.assert_close(r, v.to(tout), rtol=0, atol=0)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("shape", [(1000, 3), (3, 1000), (257, 131), (4096, 1024), (1, 50), (50, 1)])
def test_transpose(dt, shape):
    from systemml_amd.ops import kernels
    x = torch.randn(shape, device="cuda", dtype=torch.float64).to(dt)
    r = kernels.transpose(x)
    assert torch.equal(r, x.t().contiguous())
    # a strided window (slice view) transposes without a copy first
    if shape[1] > 2:
        v = x[:, 1:]
        assert _rowpitch(v) == (shape[1] if shape[0] > 1 else shape[1] - 1)
        assert torch.equal(kernels.transpose(v), v.t().contiguous())


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("lower", [True, False])
@pytest.mark.parametrize("diag", [True, False])
@pytest.mark.parametrize("values", [True, False])
def test_tri(dt, lower, diag, values):
    from systemml_amd.ops import kernels
    x = torch.randn(77, 130, device="cuda", dtype=torch.float64).to(dt)
    k = (0 if diag else -1) if lower else (0 if diag else 1)
    src = x if values else torch.ones_like(x)
    ref = torch.tril(src, k) if lower else torch.triu(src, k)
    assert torch.equal(kernels.tri(x, lower, diag, values), ref)


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("D", [1, 5, 63, 64, 300])
@pytest.mark.parametrize("idt", [torch.int32, torch.int64])
def test_gather_rows(dt, D, idt):
    from systemml_amd.ops import kernels
    x = torch.randn(5000, D, device="cuda", dtype=torch.float64).to(dt)
    idx = torch.randint(0, 5000, (3001,), device="cuda", dtype=idt)
    assert torch.equal(kernels.gather_rows(x, idx), x[idx.long()])


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
def test_slice_csr(dt):
    from systemml_amd.ops import kernels
    g = torch.Generator().manual_seed(3)
    d = torch.rand(2000, 700, generator=g, dtype=torch.float64)
    d[d < 0.97] = 0
    x = d.to(dt).cuda().to_sparse_csr()
    for (r0, r1, c0, c1) in [(0, 2000, 0, 700), (5, 900, 10, 200), (1999, 2000, 699, 700), (100, 101, 0, 700)]:
        r = kernels.slice_csr(x, r0, r1, c0, c1)
        assert torch.equal(r, d.to(dt).cuda()[r0:r1, c0:c1])


@pytest.mark.parametrize("dt", DT)
@pytest.mark.parametrize("dec", [False, True])
def test_order_perm_stable(dt, dec):
    from systemml_amd.ops import kernels
    g = torch.Generator().manual_seed(5)
    m = torch.randint(0, 7, (20000, 3), generator=g).to(torch.float64)
    m[::7, 0] = -0.0
    x = m.to(dt).cuda()
    # one key: stable (ties keep the input order), as torch's stable sort
    p = kernels.order_perm(x, [2], dec).long()
    ref = torch.sort(x[:, 1].double(), descending=dec, stable=True).indices
    assert torch.equal(p, ref)
    # two keys: first column major
    p2 = kernels.order_perm(x, [1, 3], dec).long()
    perm = torch.arange(x.shape[0], device="cuda")
    for k in (2, 0):
        perm = perm[torch.sort(x[perm, k].double(), descending=dec, stable=True).indices]
    assert torch.equal(p2, perm)
    assert torch.equal(kernels.perm_index(p2.int(), torch.float64).reshape(-1), (perm + 1).double())


def test_sort_values_and_dml_paths():
    """order / quantile / median / lower.tri / t / slices through DML on the GPU backend,
    against the CPU backend, with the HIP kernels counted."""
    from systemml_amd.api import executor as EX
    from systemml_amd.conf import DMLConfig
    from systemml_amd.ops import kernels
    rng = np.random.default_rng(1)
    X = rng.standard_normal((3000, 40))
    X[:, 3] = np.round(X[:, 3])
    src = """
    A = order(target=X, by=4, decreasing=TRUE)
    I = order(target=X, by=4, index.return=TRUE)
    B = order(target=X, by=matrix("4 1", rows=2, cols=1))
    q = quantile(X[, 2], 0.3)
    md = median(X[, 5])
    L = lower.tri(target=X[1:2000, ], diag=TRUE, values=TRUE)
    U = upper.tri(target=X[1:2000, ], diag=FALSE, values=FALSE)
    T = t(X[, 3:20])
    W = X[100:2000, 5:33]
    """
    outs = ["A", "I", "B", "q", "md", "L", "U", "T", "W"]
    before = dict(kernels.counters)
    g, _ = EX.execute(EX.compile_script(src, {}, inputs={"X": X}, outputs=outs,
                                        config=DMLConfig(gpu=True, precision="double")), {"X": X})
    c, _ = EX.execute(EX.compile_script(src, {}, inputs={"X": X}, outputs=outs,
                                        config=DMLConfig(gpu=False)), {"X": X})
    for k in outs:
        a = g[k].cpu().numpy() if hasattr(g[k], "cpu") else g[k]
        b = c[k].cpu().numpy() if hasattr(c[k], "cpu") else c[k]
        np.testing.assert_allclose(np.asarray(a, dtype=float), np.asarray(b, dtype=float), rtol=0, atol=0, err_msg=k)
    grew = {k for k, v in kernels.counters.items() if v > before.get(k, 0)}
    assert {"order", "tri", "transpose"} <= grew, grew
