"""Algebraic rewrites of round 5 (reference hops/rewrite/RewriteAlgebraicSimplificationDynamic.java
and RewriteAlgebraicSimplificationStatic.java): every rule fires on a small script (its -stats
counter) and the rewritten program computes what the unrewritten one does (DMLConfig(rewrites=
False)), on the CPU backend in fp64."""
import numpy as np
import pytest

from systemml_amd.api import executor as EX
from systemml_amd.conf import DMLConfig


def _run(src, ins, outs, rewrites=True):
    cfg = DMLConfig(gpu=False, rewrites=rewrites)
    cs = EX.compile_script(src, {}, inputs=ins, outputs=outs, config=cfg)
    out = []
    r, _ = EX.execute(cs, ins, out=out.append)
    return cs.cp.rewrite_stats or {}, {k: (v.double().numpy() if hasattr(v, "numpy") else v) for k, v in r.items()}, out


def _check(src, ins, outs, rule, fires=True):
    st, a, pa = _run(src, ins, outs)
    _, b, pb = _run(src, ins, outs, rewrites=False)
    assert (st.get(rule, 0) > 0) == fires, st
    for k in outs:
        np.testing.assert_allclose(np.asarray(a[k], dtype=float), np.asarray(b[k], dtype=float), rtol=1e-12,
                                   atol=1e-12, err_msg=k)
    assert pa == pb


RNG = np.random.default_rng(7)
A = RNG.random((6, 4))
B = RNG.random((6, 5))
C = RNG.random((1, 7))


def test_matrix_mult_diag():
    _check("v = rowSums(A)\nZ = diag(v) %*% B", {"A": A, "B": B}, ["Z"], "matrix-mult-diag")


def test_matrix_mult_diag_needs_a_vector():
    # diag(M) of a square M is its diagonal (a vector): diag(diag(M)) %*% B keeps its meaning
    M = RNG.random((6, 6))
    _check("Z = diag(diag(M)) %*% B", {"M": M, "B": B}, ["Z"], "matrix-mult-diag")
    _check("z = diag(M)\nZ = t(z) %*% B", {"M": M, "B": B}, ["Z"], "matrix-mult-diag", fires=False)


def test_diag_matrix_mult():
    _check("d = diag(A %*% t(B2))", {"A": A, "B2": RNG.random((6, 4))}, ["d"], "diag-matrix-mult")


def test_diag_binary_pushdown():
    _check("v = rowSums(A)\nW = diag(v) * 3", {"A": A}, ["W"], "diag-binary-pushdown")
    _check("v = rowSums(A)\nW = 2.5 * diag(v)", {"A": A}, ["W"], "diag-binary-pushdown")


def test_scalar_matrix_mult():
    _check("s = matrix(2, rows=1, cols=1)\nQ = s %*% C\nR = t(C) %*% s", {"C": C}, ["Q", "R"], "scalar-matrix-mult")
