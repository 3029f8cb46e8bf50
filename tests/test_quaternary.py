"""Weighted quaternary operators (wsloss / wsigmoid / wdivmm / wcemm / wumm): rewrite detection
and numerics of the fused sparse (sampled-product) and dense paths against numpy fp64
references of the unfused expressions (reference tests: test/integration/functions/quaternary/
Weighted*Test.java, which compare the rewritten against the unrewritten script)."""
import numpy as np
import pytest
import torch

from systemml_amd.api.executor import run, compile_script, explain
from systemml_amd.conf import DMLConfig
from systemml_amd.ops import quaternary as Q

CFG = DMLConfig(gpu=False)

GEN = """
X = rand(rows=300, cols=250, sparsity=%s, min=1, max=2, seed=1)
W = rand(rows=300, cols=250, sparsity=%s, min=0.5, max=1, seed=2)
U = rand(rows=300, cols=7, min=0.1, max=1, seed=3)
V = rand(rows=250, cols=7, min=0.1, max=1, seed=4)
"""

CASES = {
    "wsloss-post": ("r = sum(W * (X - U %*% t(V))^2)",
                    lambda X, W, U, V: np.sum(W * (X - U @ V.T) ** 2)),
    "wsloss-post_nz": ("r = sum((X != 0) * (X - U %*% t(V))^2)",
                       lambda X, W, U, V: np.sum((X != 0) * (X - U @ V.T) ** 2)),
    "wsloss-pre": ("r = sum((X - W * (U %*% t(V)))^2)",
                   lambda X, W, U, V: np.sum((X - W * (U @ V.T)) ** 2)),
    "wsloss-none": ("r = sum((X - U %*% t(V))^2)",
                    lambda X, W, U, V: np.sum((X - U @ V.T) ** 2)),
    "wsigmoid": ("r = W * sigmoid(U %*% t(V))",
                 lambda X, W, U, V: W / (1 + np.exp(-(U @ V.T)))),
    "wsigmoid-minus-log": ("r = W * log(sigmoid(-(U %*% t(V))))",
                           lambda X, W, U, V: W * np.log(1 / (1 + np.exp(U @ V.T)))),
    "wdivmm-right": ("r = (W / (U %*% t(V))) %*% V",
                     lambda X, W, U, V: (W / (U @ V.T)) @ V),
    "wdivmm-left-eps": ("r = t(U) %*% (W / (U %*% t(V) + 1e-6))",
                        lambda X, W, U, V: U.T @ (W / (U @ V.T + 1e-6))),
    "wdivmm-mult": ("r = (W * (U %*% t(V))) %*% V",
                    lambda X, W, U, V: (W * (U @ V.T)) @ V),
    "wcemm": ("r = sum(X * log(U %*% t(V)))",
              lambda X, W, U, V: np.sum(X * np.log(U @ V.T))),
    "wcemm-eps": ("r = sum(X * log(U %*% t(V) + 1e-15))",
                  lambda X, W, U, V: np.sum(X * np.log(U @ V.T + 1e-15))),
    "wumm": ("r = X * exp(U %*% t(V))",
             lambda X, W, U, V: X * np.exp(U @ V.T)),
    "wumm-div": ("r = X / (U %*% t(V))^2",
                 lambda X, W, U, V: X / (U @ V.T) ** 2),
}


def _np(v):
    if isinstance(v, torch.Tensor):
        if v.layout != torch.strided:
            v = v.to_dense()
        return v.double().numpy()
    return v


@pytest.mark.parametrize("sp", ["0.05", "1.0"])
@pytest.mark.parametrize("case", sorted(CASES))
def test_wquat_rewrite_and_numerics(case, sp):
    body, ref = CASES[case]
    src = GEN % (sp, sp) + body
    cs = compile_script(src, inputs={}, outputs=["r", "X", "W", "U", "V"], config=CFG)
    assert "wquat" in explain(cs.cp), explain(cs.cp)
    res = run(src, inputs={}, outputs=["r", "X", "W", "U", "V"], config=CFG, out=lambda s: None)
    X, W, U, V = (_np(res[k]) for k in "XWUV")
    expect = ref(X, W, U, V)
    np.testing.assert_allclose(_np(res["r"]), expect, rtol=1e-9, atol=1e-9)


def test_wquat_disabled_without_fusion():
    cfg = DMLConfig(gpu=False)
    cfg.fusion = False
    src = GEN % ("0.05", "0.05") + CASES["wsloss-post"][0]
    cs = compile_script(src, inputs={}, outputs=["r"], config=cfg)
    assert "wquat" not in explain(cs.cp)


def test_sparse_paths_match_dense_direct():
    g = torch.Generator().manual_seed(0)
    m, n, r = 120, 90, 5
    Wd = (torch.rand(m, n, generator=g) < 0.1).float() * torch.rand(m, n, generator=g)
    Xd = (torch.rand(m, n, generator=g) < 0.1).float() * (1 + torch.rand(m, n, generator=g))
    U = torch.rand(m, r, generator=g) + 0.1
    V = torch.rand(n, r, generator=g) + 0.1
    Ws, Xs = Wd.to_sparse_csr(), Xd.to_sparse_csr()
    uv = U @ V.T
    for kind in ("post", "pre", "none", "post_nz"):
        fused = Q.wsloss(kind, Xs if kind in ("none", "post_nz") else Xd, U, V, Ws)
        unfused = Q.wsloss(kind, Xd, U, V, Wd)
        assert fused == pytest.approx(unfused, rel=1e-4)
    np.testing.assert_allclose(Q.wsigmoid(Ws, U, V, True, False).to_dense(),
                               Wd * torch.sigmoid(-uv), rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(Q.wdivmm(Ws, U, V, True, False, 1e-6),
                               U.T @ (Wd / (uv + 1e-6)), rtol=1e-4)
    np.testing.assert_allclose(Q.wdivmm(Ws, U, V, False, True), (Wd * uv) @ V, rtol=1e-4)
    assert Q.wcemm(Xs, U, V) == pytest.approx(float((Xd * torch.log(uv)).sum()), rel=1e-5)
    np.testing.assert_allclose(Q.wumm(Xs, U, V, "exp").to_dense(), Xd * torch.exp(uv), rtol=1e-5)


def _near_converged(dtype=torch.float64, m=300, n=200, r=6, seed=0):
    """Large-magnitude sparse X that U V' reproduces up to a tiny residual: the regime in which
    sum(X^2) - 2 sum(X .* UV') + sum(UV'^2) cancels catastrophically."""
    g = torch.Generator().manual_seed(seed)
    U = (torch.rand(m, r, generator=g, dtype=torch.float64) + 0.5) * 100
    V = (torch.rand(n, r, generator=g, dtype=torch.float64) + 0.5) * 100
    mask = torch.rand(m, n, generator=g, dtype=torch.float64) < 0.05
    Xd = torch.where(mask, U @ V.T + 1e-3 * torch.randn(m, n, generator=g, dtype=torch.float64),
                     torch.zeros((), dtype=torch.float64))
    return Xd.to(dtype), U.to(dtype), V.to(dtype), mask


def test_wsloss_fp64_no_cancellation():
    """(advisor finding) the fused sparse paths compute in the engine precision (fp64) with
    the residual summed directly: near convergence on a large-magnitude X they agree with the
    fp64 unfused expression to ~1e-9 relative."""
    Xd, U, V, mask = _near_converged()
    Xs = Xd.to_sparse_csr()
    W = mask.double()
    Ws = W.to_sparse_csr()
    uv = U @ V.T
    exact = {
        "post_nz": float(((Xd - uv) ** 2 * mask).sum()),
        "post": float((W * (Xd - uv) ** 2).sum()),
        "none": float(((Xd - uv) ** 2).sum()),
        "pre": float(((Xd - W * uv) ** 2).sum()),
    }
    assert exact["post_nz"] < 1e-3 * float((Xd ** 2).sum()) * 1e-9      # residual is tiny
    got = {
        "post_nz": Q.wsloss("post_nz", Xs, U, V),
        "post": Q.wsloss("post", Xs, U, V, Ws),           # sparse X gathered at W's pattern
        "none": Q.wsloss("none", Xs, U, V),
        "pre": Q.wsloss("pre", Xd, U, V, Ws),
    }
    for k in exact:
        assert got[k] == pytest.approx(exact[k], rel=1e-9), (k, got[k], exact[k])
    # sparse X with a pattern different from W: looked up, not densified
    W2 = (torch.rand(Xd.shape, generator=torch.Generator().manual_seed(9), dtype=torch.float64) < 0.05).double()
    e2 = float((W2 * (Xd - uv) ** 2).sum())
    assert Q.wsloss("post", Xs, U, V, W2.to_sparse_csr()) == pytest.approx(e2, rel=1e-9)


def test_wquat_sparse_safe_semantics():
    """(advisor finding) zeros of X / W contribute 0 even where f(U V') overflows: dense and
    sparse representations give the same result (reference: the operators iterate over the
    non-zeros)."""
    g = torch.Generator().manual_seed(2)
    m, n, r = 40, 30, 3
    U = torch.rand(m, r, generator=g, dtype=torch.float64) * 400     # exp(U V') overflows to inf
    V = torch.rand(n, r, generator=g, dtype=torch.float64) * 400
    Xd = (torch.rand(m, n, generator=g, dtype=torch.float64) < 0.2).double() * 1e-300
    dense = Q.wumm(Xd, U, V, "exp")
    sparse = Q.wumm(Xd.to_sparse_csr(), U, V, "exp").to_dense()
    assert not torch.isnan(dense).any() and torch.equal(torch.isinf(dense), torch.isinf(sparse))
    assert bool((dense[Xd == 0] == 0).all())
    # log(sigmoid(-uv)) = -inf where uv is huge: zero weights stay 0
    ws = Q.wsigmoid(Xd, U, V, True, True)
    assert bool((ws[Xd == 0] == 0).all())


def test_wquat_rewrite_guards():
    """(advisor finding) like the reference: no rewrite when W is a broadcast vector (sizes
    differ) or when U %*% t(V) has another consumer."""
    src_vec = """
U = rand(rows=300, cols=4, seed=1)
V = rand(rows=250, cols=4, seed=2)
w = rand(rows=300, cols=1, seed=3)
r = w * exp(U %*% t(V))
"""
    cs = compile_script(src_vec, inputs={}, outputs=["r"], config=CFG)
    assert "wquat" not in explain(cs.cp)
    res = run(src_vec, inputs={}, outputs=["r", "U", "V"], config=CFG, out=lambda s: None)
    assert res["r"].shape == (300, 250)
    src_shared = GEN % ("0.05", "0.05") + """
UV = U %*% t(V)
r = sum(W * (X - UV)^2)
s = sum(UV)
"""
    cs = compile_script(src_shared, inputs={}, outputs=["r", "s"], config=CFG)
    assert "wquat" not in explain(cs.cp)


@pytest.mark.gpu
def test_sddmm_fp64_kernel_and_near_converged_wsloss_on_gpu():
    """fp64 SDDMM kernel (grouped-lane variant) against the host fp64 expression."""
    from systemml_amd.ops import kernels
    from systemml_amd.ops.backend import backend
    backend.configure(DMLConfig(gpu=True))          # kernels on (fp64 engine precision)
    dev = torch.device("cuda:0")
    Xd, U, V, mask = _near_converged(m=2000, n=1500, r=8)
    Xs = Xd.to_sparse_csr()
    exact = float(((Xd - U @ V.T) ** 2 * mask).sum())
    before = kernels.counters.get("sddmm", 0)
    got = Q.wsloss("post_nz", Xs.to(dev), U.to(dev), V.to(dev))
    assert kernels.counters.get("sddmm", 0) > before
    assert got == pytest.approx(exact, rel=1e-9)
    for r in (1, 5, 64, 100, 300):
        g = torch.Generator().manual_seed(r)
        S = (torch.rand(700, 500, generator=g) < 0.02).double().to_sparse_csr()
        Uh = torch.randn(700, r, generator=g, dtype=torch.float64)
        Vh = torch.randn(500, r, generator=g, dtype=torch.float64)
        crow, col = S.crow_indices(), S.col_indices()
        rows = torch.repeat_interleave(torch.arange(700), crow[1:] - crow[:-1])
        ref = (Uh[rows] * Vh[col]).sum(1)
        out = kernels.sddmm(crow.to(dev), col.to(dev), Uh.to(dev), Vh.to(dev), torch.float64)
        np.testing.assert_allclose(out.cpu().numpy(), ref.numpy(), rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
def test_wquat_sparse_on_gpu():
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(1)
    m, n, r = 4000, 3000, 16
    Wd = (torch.rand(m, n, generator=g) < 0.01).float()
    Xd = Wd * (1 + torch.rand(m, n, generator=g))
    U = torch.rand(m, r, generator=g)
    V = torch.rand(n, r, generator=g)
    ref = float((Wd * (Xd - U @ V.T) ** 2).sum())
    got = Q.wsloss("post_nz", Xd.to_sparse_csr().to(dev), U.to(dev), V.to(dev))
    assert got == pytest.approx(ref, rel=1e-4)
    ref2 = (Wd / (U @ V.T)) @ V
    got2 = Q.wdivmm(Wd.to_sparse_csr().to(dev), U.to(dev), V.to(dev), False)
    np.testing.assert_allclose(got2.cpu(), ref2, rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("r", [16, 7, 200])
def test_sddmm_hip_kernel_matches_fp32(r):
    from systemml_amd.ops import kernels
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(r)
    m, n = 5000, 3000
    S = ((torch.rand(m, n, generator=g) < 0.005).float()).to_sparse_csr()
    U = torch.randn(m, r, generator=g)
    V = torch.randn(n, r, generator=g)
    crow, col = S.crow_indices(), S.col_indices()
    rows = torch.repeat_interleave(torch.arange(m), crow[1:] - crow[:-1])
    ref = (U[rows] * V[col]).sum(1)
    got = kernels.sddmm(crow.to(dev), col.to(dev), U.to(dev), V.to(dev))
    assert got is not None
    torch.cuda.synchronize()
    np.testing.assert_allclose(got.cpu(), ref, rtol=1e-4, atol=1e-4)


def test_wdivmm_residual_forms_match_unfused():
    """W * (U %*% t(V) - X) in both product orientations (the ALS-CG gradients) runs as a
    sampled product at W's non-zeros and matches the unfused dense evaluation."""
    import torch
    from systemml_amd.api.executor import run, compile_script
    from systemml_amd.conf import DMLConfig
    g = torch.Generator().manual_seed(3)
    R, C, k = 300, 200, 10
    cols = torch.stack([torch.randperm(C, generator=g)[:k].sort().values for _ in range(R)])
    X = torch.sparse_csr_tensor(torch.arange(0, R * k + 1, k), cols.reshape(-1),
                                torch.randint(1, 6, (R * k,), generator=g).double(), (R, C))
    U, V = torch.rand(R, 4, generator=g).double(), torch.rand(C, 4, generator=g).double()
    for stmt in ("G = (W * (U %*% t(V) - X)) %*% V", "G = t(t(U) %*% (W * (U %*% t(V) - X)))"):
        src = "W = (X != 0)\n" + stmt
        ins = {"X": X, "U": U, "V": V}
        cs = compile_script(src, inputs=ins, outputs=["G"], config=DMLConfig(gpu=False))
        assert cs.cp.rewrite_stats.get("wquat-wdivmm") == 1, cs.cp.rewrite_stats
        a = run(src, inputs=ins, outputs=["G"], config=DMLConfig(gpu=False), out=lambda s: None)["G"]
        b = run(src, inputs=ins, outputs=["G"], config=DMLConfig(gpu=False, fusion=False), out=lambda s: None)["G"]
        np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=1e-12, atol=1e-10)


def test_sparse_inputs_with_duplicate_cells_are_canonicalised():
    """A CSR input that stores a cell twice means the sum (as its dense form); inputs are
    canonicalised so the operators at the non-zeros agree with the dense evaluation."""
    import torch
    from systemml_amd.api.executor import run
    from systemml_amd.conf import DMLConfig
    g = torch.Generator().manual_seed(4)
    R, C, k = 200, 150, 12
    cols = torch.randint(0, C, (R, k), generator=g).sort(1).values          # duplicates likely
    X = torch.sparse_csr_tensor(torch.arange(0, R * k + 1, k), cols.reshape(-1),
                                torch.randint(1, 6, (R * k,), generator=g).double(), (R, C))
    U, V = torch.rand(R, 3, generator=g).double(), torch.rand(C, 3, generator=g).double()
    src = "W = (X != 0)\nl = 0.5 * sum(W * (U %*% t(V) - X) ^ 2)\nG = (W * (U %*% t(V) - X)) %*% V"
    ins = {"X": X, "U": U, "V": V}
    a = run(src, inputs=ins, outputs=["l", "G"], config=DMLConfig(gpu=False), out=lambda s: None)
    b = run(src, inputs=ins, outputs=["l", "G"], config=DMLConfig(gpu=False, fusion=False), out=lambda s: None)
    assert float(a["l"]) == pytest.approx(float(b["l"]), rel=1e-12)
    np.testing.assert_allclose(a["G"].numpy(), b["G"].numpy(), rtol=1e-12, atol=1e-10)
