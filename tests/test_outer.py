"""Outer-product-template fusion (compiler/codegen.fuse_outer, ops/outer.py).

Reference tests: src/test/java/org/apache/sysml/test/integration/functions/codegen/
OuterProdTmplTest.java (sparse-safe cellwise DAGs over U %*% t(V) with cellwise, full
aggregate, left and right matrix-multiplication outputs must match the unfused plan and
appear as spoof outer-product operators).  CPU: plan shape, sparse-safety proof, exact parity
with fusion disabled.  GPU: sparse driver (SDDMM + generated cell kernel + CSR SpMM) and dense
driver (MFMA GEMM + cell kernel) against numpy fp64."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from systemml_amd.api import executor as EX
from systemml_amd.conf import DMLConfig

SCRIPT = """
a = sum(W * exp(U %*% t(V)) + W * 2)
b = (W * (U %*% t(V) - 1)^2) %*% V
c = t(W * abs(U %*% t(V) - X)) %*% U
d = (W != 0) * sqrt(abs(U %*% t(V)))
"""
OUTS = ["a", "b", "c", "d"]


def _inputs(m=60, n=45, r=4, density=0.1, seed=0):
    rng = np.random.default_rng(seed)
    W = sp.random(m, n, density=density, random_state=seed + 1, format="csr")
    return {"W": W, "U": rng.random((m, r)), "V": rng.random((n, r)), "X": rng.random((m, n))}


def _np(x):
    if isinstance(x, torch.Tensor):
        x = x.to_dense() if x.layout != torch.strided else x
        return x.double().cpu().numpy()
    return float(x.value()) if hasattr(x, "value") else float(x)


def _ref(ins):
    Wd = ins["W"].toarray()
    U, V, X = ins["U"], ins["V"], ins["X"]
    UV = U @ V.T
    return {"a": (Wd * np.exp(UV) + Wd * 2).sum(), "b": (Wd * (UV - 1) ** 2) @ V,
            "c": (Wd * np.abs(UV - X)).T @ U, "d": (Wd != 0) * np.sqrt(np.abs(UV))}


def test_outer_plans_and_parity_with_unfused():
    ins = _inputs()
    cs = EX.compile_script(SCRIPT, {}, inputs=ins, outputs=OUTS, config=DMLConfig(gpu=False))
    plan = EX.explain(cs.cp, "hops")
    for ot in ("|all", "|left", "|right", "|cell"):
        assert f"]{ot}" in plan and "outer[" in plan, (ot, plan)
    res, _ = EX.execute(cs, ins)
    cs0 = EX.compile_script(SCRIPT, {}, inputs=ins, outputs=OUTS, config=DMLConfig(gpu=False, fusion=False))
    assert "outer[" not in EX.explain(cs0.cp, "hops")
    ref, _ = EX.execute(cs0, ins)
    want = _ref(ins)
    for k in OUTS:
        np.testing.assert_allclose(_np(res[k]), _np(ref[k]), rtol=1e-13, atol=1e-13, err_msg=k)
        np.testing.assert_allclose(_np(res[k]), want[k], rtol=1e-12, atol=1e-12, err_msg=k)


def test_outer_requires_sparse_safe_driver():
    # W + f(UV') is not zero where W is: no outer operator (the product is materialised)
    src = "a = sum((W + 1) * exp(U %*% t(V)))\nb = (W - U %*% t(V)) %*% V"
    ins = _inputs()
    cs = EX.compile_script(src, {}, inputs=ins, outputs=["a", "b"], config=DMLConfig(gpu=False))
    assert "outer[" not in EX.explain(cs.cp, "hops")
    res, _ = EX.execute(cs, ins)
    Wd, U, V = ins["W"].toarray(), ins["U"], ins["V"]
    assert _np(res["a"]) == pytest.approx(((Wd + 1) * np.exp(U @ V.T)).sum(), rel=1e-12)
    np.testing.assert_allclose(_np(res["b"]), (Wd - U @ V.T) @ V, rtol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("density", [0.02, 1.0])
@pytest.mark.parametrize("precision", ["double", "single"])
def test_outer_kernels_on_gpu(density, precision):
    from systemml_amd.ops import outer
    ins = _inputs(m=3001, n=1203, r=16, density=density, seed=3)
    if density == 1.0:
        ins["W"] = ins["W"].toarray()                # dense driver: GEMM + cell kernel path
    before = dict(outer.stats)
    cfg = DMLConfig(gpu=True, precision=precision, gpu_min_cells=0)
    res, _ = EX.execute(EX.compile_script(SCRIPT, {}, inputs=ins, outputs=OUTS, config=cfg), ins)
    path = "sparse" if density < 1.0 else "dense"
    assert outer.stats[path] >= before[path] + 4, outer.stats
    want = _ref({**ins, "W": sp.csr_matrix(ins["W"])})
    tol = 1e-10 if precision == "double" else 2e-4
    for k in OUTS:
        g = _np(res[k])
        scale = max(1.0, float(np.abs(want[k]).max()))
        assert float(np.abs(g - want[k]).max()) / scale < tol, k
