"""Sparse matrix-multiply family on the MI355X (ops/hip/spgemm.hip; reference
LibMatrixMult.java:1105 / :1397 / :1839, LibMatrixCuMatMult.java:173): every kernel against a
dense fp64 torch evaluation of the same product -- nnz-balanced SpMM (int32 column indices,
power-law skewed rows, empty rows, K from 1 to 70), dense x sparse, SpGEMM (canonical
output), sparse tsmm; and the operator dispatch (ops/sparse.mm / tsmm) through DML."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from systemml_amd.ops import kernels
    kernels.load(required=True)
    from systemml_amd.ops.backend import backend
    from systemml_amd.conf import DMLConfig
    backend.configure(DMLConfig(precision="single"))


def _csr(m, n, density, skew=False, seed=0, empty_rows=0):
    g = np.random.default_rng(seed)
    if skew:
        per = np.minimum(n, (g.pareto(1.2, m) * 3 + 1).astype(int))
        per[: max(1, m // 50)] = n // 2                       # a few very long rows
    else:
        per = g.binomial(n, density, m)
    if empty_rows:
        per[g.choice(m, empty_rows, replace=False)] = 0
    rows, cols = [], []
    for i, k in enumerate(per):
        c = g.choice(n, int(k), replace=False)
        rows += [i] * len(c)
        cols += list(c)
    vals = g.standard_normal(len(rows))
    d = torch.zeros((m, n), dtype=torch.float64)
    if rows:
        d[torch.tensor(rows), torch.tensor(cols)] = torch.tensor(vals)
    return d


@pytest.mark.parametrize("m,n,K,skew", [(1000, 700, 1, False), (3000, 500, 4, True), (513, 2000, 16, True),
                                        (257, 300, 70, False), (2000, 5000, 10, True)])
def test_spmm_balanced(m, n, K, skew):
    _need_gpu()
    from systemml_amd.ops import kernels
    d = _csr(m, n, 0.02, skew=skew, seed=m + K, empty_rows=m // 10)
    A = d.to("cuda", torch.float32).to_sparse_csr()
    B = torch.randn(n, K, dtype=torch.float64)
    C = kernels.spmm_bal(A, B.to("cuda", torch.float32))
    ref = d @ B
    torch.testing.assert_close(C.double().cpu(), ref, rtol=1e-4, atol=1e-4 * max(1.0, ref.abs().max().item()))
    C64 = kernels.spmm_bal(d.to("cuda").to_sparse_csr(), B.to("cuda"))
    torch.testing.assert_close(C64.cpu(), ref, rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("m,k,n", [(300, 400, 200), (1000, 700, 5000), (64, 3000, 32768)])
def test_spgemm_canonical(m, k, n):
    _need_gpu()
    from systemml_amd.ops import kernels
    a = _csr(m, k, 0.01, seed=1, empty_rows=m // 8)
    b = _csr(k, n, 0.005, skew=True, seed=2)
    C = kernels.spgemm(a.to("cuda", torch.float32).to_sparse_csr(), b.to("cuda", torch.float32).to_sparse_csr())
    assert C is not None and C.layout == torch.sparse_csr
    crow, col = C.crow_indices().cpu(), C.col_indices().cpu()
    for i in range(0, m, max(1, m // 50)):                    # sorted, duplicate-free rows
        r = col[crow[i]:crow[i + 1]]
        assert bool((r[1:] > r[:-1]).all())
    ref = a @ b
    torch.testing.assert_close(C.to_dense().double().cpu(), ref, rtol=1e-4, atol=1e-4)
    assert int(C.values().numel()) == int(((a != 0).double() @ (b != 0).double() != 0).sum())


@pytest.mark.parametrize("m,D,skew", [(5000, 300, False), (2000, 1500, True)])
def test_tsmm_sparse(m, D, skew):
    _need_gpu()
    from systemml_amd.ops import kernels
    x = _csr(m, D, 0.01, skew=skew, seed=5)
    C = kernels.tsmm_sparse(x.to("cuda", torch.float32).to_sparse_csr())
    ref = x.t() @ x
    torch.testing.assert_close(C.double().cpu(), ref, rtol=1e-4, atol=1e-3)
    C64 = kernels.tsmm_sparse(x.to("cuda").to_sparse_csr())
    torch.testing.assert_close(C64.cpu(), ref, rtol=1e-10, atol=1e-9)


def test_sparse_dispatch_through_dml():
    """Dense x sparse, sparse x sparse, t(S) %*% D, t(S) %*% S and S %*% D through the DML
    operators on the GPU backend: HIP kernels run (counters), results match the CPU backend."""
    _need_gpu()
    from systemml_amd.api import executor as EX
    from systemml_amd.conf import DMLConfig
    from systemml_amd.ops import kernels
    src = """
    a = sum(D %*% S)
    b = sum(S %*% T)
    c = sum(t(S) %*% t(D[1:8, ]))
    d = sum(t(S) %*% S)
    e = sum(S %*% E)
    """
    import scipy.sparse as sp
    rng = np.random.default_rng(7)
    ins = {"S": sp.random(3000, 2000, density=0.01, format="csr", random_state=3),
           "T": sp.random(2000, 1500, density=0.01, format="csr", random_state=4),
           "D": rng.standard_normal((40, 3000)), "E": rng.standard_normal((2000, 8))}
    before = dict(kernels.counters)
    out = {}
    for gpu in (True, False):
        cs = EX.compile_script(src, {}, inputs=ins, outputs=list("abcde"), config=DMLConfig(gpu=gpu, precision="double"))
        r, _ = EX.execute(cs, ins)
        out[gpu] = {k: float(r[k]) for k in "abcde"}
    grew = {k for k, v in kernels.counters.items() if v > before.get(k, 0)}
    assert {"spmm_bal", "tsmm_sparse"} <= grew, kernels.counters
    for k in "abcde":
        assert out[True][k] == pytest.approx(out[False][k], rel=1e-8), k


@pytest.mark.parametrize("prec", ["single", "double"])
def test_sparse_sparse_product_elementwise(prec):
    """S %*% T element by element against scipy: single precision runs the fp32 SpGEMM
    kernel; double precision must not (its LDS accumulator is fp32) and matches to fp64."""
    _need_gpu()
    from systemml_amd.api import executor as EX
    from systemml_amd.conf import DMLConfig
    from systemml_amd.ops import kernels
    import scipy.sparse as sp
    S = sp.random(3000, 2000, density=0.01, format="csr", random_state=3)
    T = sp.random(2000, 1500, density=0.01, format="csr", random_state=4)
    before = kernels.counters.get("spgemm", 0)
    r, _ = EX.execute(EX.compile_script("C = S %*% T", {}, inputs={"S": S, "T": T}, outputs=["C"],
                                        config=DMLConfig(gpu=True, precision=prec)), {"S": S, "T": T})
    C = r["C"]
    C = (C.to_dense() if C.layout != torch.strided else C).double().cpu().numpy()
    ref = (S @ T).toarray()
    if prec == "single":
        assert kernels.counters.get("spgemm", 0) > before
        np.testing.assert_allclose(C, ref, rtol=1e-5, atol=1e-6)
    else:
        assert kernels.counters.get("spgemm", 0) == before
        np.testing.assert_allclose(C, ref, rtol=1e-12, atol=1e-14)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [1, 10, 33, 64])
@pytest.mark.parametrize("form", ["mult", "multx", "div"])
@pytest.mark.parametrize("left", [False, True])
@pytest.mark.parametrize("blocked", [False, True])
@pytest.mark.parametrize("pad", [False, True])
def test_fused_wdivmm_matches_dense(K, form, left, blocked, pad, monkeypatch):
    """sddmm.hip wdivmm_kernel (one pass over W's pattern, the gathered factor row reused for
    the accumulation) against fp64 torch on the dense equivalent, right and left forms."""
    from systemml_amd.ops import quaternary as Q, kernels
    from systemml_amd.ops.backend import backend
    from systemml_amd.conf import DMLConfig
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    backend.configure(DMLConfig(gpu=True, precision="double"))
    g = torch.Generator().manual_seed(K)
    m, n = 3001, 2003
    mask = torch.rand(m, n, generator=g) < 0.01
    mask[7] = True                                   # a dense row: chunks split it
    Xd = torch.where(mask, torch.rand(m, n, generator=g, dtype=torch.float64) + 0.5, torch.zeros((), dtype=torch.float64))
    Wd = (Xd != 0).double() * (1.0 + torch.rand(m, n, generator=g, dtype=torch.float64))
    U = torch.rand(m, K, generator=g, dtype=torch.float64)
    V = torch.rand(n, K, generator=g, dtype=torch.float64)
    X = Xd.to_sparse_csr().cuda()
    W = torch.sparse_csr_tensor(X.crow_indices(), X.col_indices(), Wd[mask.nonzero(as_tuple=True)].cuda(), (m, n))
    uv = U @ V.t()
    q = {"mult": Wd * uv, "multx": Wd * (uv - Xd), "div": torch.where(mask, Wd / (uv + 0.5), torch.zeros((), dtype=torch.float64))}[form]
    ref = U.t() @ q if left else q @ V
    if blocked:
        # column-blocked passes (the gathered factor visited ~7 column blocks at a time)
        monkeypatch.setattr(kernels, "WD_BLOCK_MIN_NNZ", 0)
        monkeypatch.setattr(kernels, "WD_BLOCK_BYTES", K * 8 * 300)
    # pad: the gathered factor as a copy with power-of-two row pitch (K = 10 / 33: 16 / 64)
    monkeypatch.setattr(kernels, "WD_PAD", pad)
    monkeypatch.setattr(kernels, "WD_PAD_MIN_NNZ", 0)
    p0 = kernels.counters.get("wdivmm_padV", 0)
    c0 = kernels.counters.get("wdivmm", 0)
    b0 = kernels.counters.get("wdivmm_blocked", 0)
    got = Q.wdivmm(W, U.cuda(), V.cuda(), left, mult=form != "div", eps=0.5 if form == "div" else None,
                   X=X if form == "multx" else None)
    assert kernels.counters.get("wdivmm", 0) == c0 + 1
    assert kernels.counters.get("wdivmm_blocked", 0) == b0 + int(blocked)
    if pad and K == 10:
        assert kernels.counters.get("wdivmm_padV", 0) >= p0 + (0 if left else 1)
    torch.testing.assert_close(got.cpu(), ref, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("m,n,per", [(1000, 700, 9), (50, 100000, 40), (3000, 5, 3)])
def test_csr_transpose_counting_sort(m, n, per):
    """Transposed CSR pattern by counting sort (csrt.hip: column counts, atomic slot claims,
    per-segment bitonic sort by row) equals the key-sort plan: canonical t(A), and the value
    permutation gathers A's values into t(A)'s order."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from systemml_amd.ops import kernels
    kernels.load(required=True)
    g = torch.Generator().manual_seed(m + n)
    dense = (torch.rand(m, n, generator=g) < per / n).double() * torch.randn(m, n, generator=g, dtype=torch.float64)
    A = dense.to_sparse_csr().to("cuda")
    crow, col = A.crow_indices(), A.col_indices()
    t = kernels.csr_transpose_plan(crow, col, m, n)
    if (dense != 0).sum(0).max().item() > 1024:
        assert t is None                    # segments longer than the in-LDS sort: key-sort fallback
        return
    assert t is not None
    crowT, colT, perm = t
    ref = dense.t().contiguous().to_sparse_csr()
    assert torch.equal(crowT.cpu(), ref.crow_indices())
    assert torch.equal(colT.cpu(), ref.col_indices())
    vt = kernels.gather(A.values(), perm)
    assert torch.equal(vt.cpu(), ref.values())
    assert torch.equal(kernels.idx32_of(colT).cpu(), ref.col_indices().int())


@pytest.mark.parametrize("dt", [torch.float32, torch.float64, torch.bfloat16])
def test_dot_kernel(dt):
    """sum(a * b) (tak+*) on agg.hip: fp64 accumulation against fp64 torch."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from systemml_amd.ops import kernels
    kernels.load(required=True)
    g = torch.Generator().manual_seed(3)
    a = torch.randn(1234, 567, generator=g, dtype=torch.float64).to(dt)
    b = torch.randn(1234, 567, generator=g, dtype=torch.float64).to(dt)
    r = kernels.dot(a.cuda(), b.cuda())
    ref = (a.double() * b.double()).sum().item()
    assert r.dtype == torch.float64 and r.dim() == 0
    assert r.item() == pytest.approx(ref, rel=1e-10, abs=1e-8)
