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
    # a square M: diag(M) is its diagonal, and diag(diag(M)) %*% B is not rewritten (the
    # argument is not a column vector by construction)
    _check("Z = diag(diag(M)) %*% B", {"M": M, "B": B}, ["Z"], "matrix-mult-diag", fires=False)
    _check("Z = diag(rowSums(M)) %*% B", {"M": M, "B": B}, ["Z"], "matrix-mult-diag")


def test_diag_matrix_mult():
    _check("d = diag(A %*% t(A))", {"A": A}, ["d"], "diag-matrix-mult")
    _check("d = diag(t(A) %*% A)", {"A": A}, ["d"], "diag-matrix-mult")
    _check("d = diag(A %*% t(B2 * 2))", {"A": A, "B2": A}, ["d"], "diag-matrix-mult", fires=False)


def test_diag_binary_pushdown():
    _check("v = rowSums(A)\nW = diag(v) * 3", {"A": A}, ["W"], "diag-binary-pushdown")
    _check("v = rowSums(A)\nW = 2.5 * diag(v)", {"A": A}, ["W"], "diag-binary-pushdown")


def test_scalar_matrix_mult():
    _check("s = matrix(2, rows=1, cols=1)\nQ = s %*% C\nR = t(C) %*% s", {"C": C}, ["Q", "R"], "scalar-matrix-mult")


def test_scalar_matrix_mult_keeps_dimension_check():
    """A 1 x 1 times a matrix with more than one row is a dimension mismatch, not a scaling."""
    from systemml_amd.parser.errors import DMLRuntimeError
    with pytest.raises(Exception) as ei:
        _run("s = matrix(2, rows=1, cols=1)\nQ = s %*% A\nprint(sum(Q))", {"A": A}, ["Q"])
    assert "dim" in str(ei.value).lower() or isinstance(ei.value, DMLRuntimeError), ei.value


def test_square_matrix_mult():
    _check("v = t(colSums(A ^ 2))\nv[1, 1] = 2\nr = (A ^ 2) %*% (v ^ 2) + A %*% v\n", {"A": A}, ["r"],
           "square-matrix-mult")


def test_square_matrix_mult_over_intercept_column():
    """(cbind(A, 1) ^ 2) %*% v -> (A ^ 2) %*% v[1:D, ] + 1 ^ 2 * v[D + 1, 1] (MultiLogReg icpt=2)."""
    _check("X = cbind(A, matrix(1, rows=nrow(A), cols=1))\nv = t(colSums(X))\nv[1, 1] = 2\n"
           "r = (X ^ 2) %*% (v ^ 2) + 3\n", {"A": A}, ["r"], "square-matrix-mult-cbind")


V = np.floor(RNG.random((12, 1)) * 5) + 1
M2 = RNG.random((12, 3))


@pytest.mark.parametrize("src,outs,rule", [
    ("s = sum(A + A * 2)\nt = sum(A - B[, 1:4])\n", ["s", "t"], "pushdown-sum-additive"),
    ("R = (0 - A) %*% matrix(1, rows=4, cols=1)\n", ["R"], "reorder-minus-mm"),
    ("R = table(seq(1, nrow(A)), seq(nrow(A), 1, -1)) %*% A\n", ["R"], "reverse-operation"),
    ("R = 3 + A %*% t(A)\nQ = A %*% t(A) - 2\n", ["R", "Q"], "canonical-mm-scalar-add"),
    ("R = ifelse(TRUE, A, A * 2)\nQ = ifelse(FALSE, A, A * 2)\nS = ifelse(sum(A) > 1, A, A)\n",
     ["R", "Q", "S"], "ifelse-removal"),
    ("T = table(V, matrix(1, rows=nrow(V), cols=1), matrix(2, rows=nrow(V), cols=1))\n", ["T"],
     "ctable-const-inputs"),
    ("T = table(V, seq(1, nrow(V)), 5, nrow(V))\n", ["T"], "table-seq-expand"),
    ("G = aggregate(target=M2[, 1], groups=V, fn=\"count\")\n", ["G"], "grouped-aggregate-count"),
    ("O = outer(V, t(seq(1, 4)), \"==\")\n", ["O"], "outer-seq-expand"),
    ("s = sum(V ^ 2)\n", ["s"], "dot-product-sum"),
])
def test_remaining_algebraic_rules(src, outs, rule):
    _check(src, {"A": A, "B": B, "V": V, "M2": M2}, outs, rule)


def test_nnz():
    X = RNG.random((6, 5)) * (RNG.random((6, 5)) > 0.5)
    _check("n = sum(X != 0)\nprint(n)", {"X": X}, ["n"], "nnz")


def test_colwise_aggregates_of_vectors():
    src = """
    r = colSums(A)          # 1 x 4
    c = rowSums(A)          # 6 x 1
    a1 = colSums(r)
    a2 = rowMeans(c)
    a3 = colMaxs(c)
    a4 = rowMins(r)
    """
    _check(src, {"A": A}, ["a1", "a2", "a3", "a4"], "colwise-aggregate")


def test_unnecessary_cumulative():
    _check("r = colSums(A)\nZ = cumsum(r)\nW = cumprod(r)", {"A": A}, ["Z", "W"], "unnecessary-cumulative")


def test_datagen_reorg():
    _check("Z = t(matrix(3.5, rows=4, cols=2)) + B[1:2, 1:4]", {"B": B}, ["Z"], "datagen-reorg")


def test_transposed_append_and_fold():
    src = "Z = t(cbind(t(A), t(A2)))\nW = cbind(cbind(A, A2), A)"
    _check(src, {"A": A, "A2": RNG.random((6, 4))}, ["Z", "W"], "transposed-append")
    _check(src, {"A": A, "A2": RNG.random((6, 4))}, ["Z", "W"], "fold-append")


def test_minus_nz_and_log_nz():
    X = RNG.random((6, 5)) + 0.5
    X[X < 0.8] = 0
    _check("s = 0.25\nZ = X - s * (X != 0)", {"X": X}, ["Z"], "minus-nz")
    Xp = RNG.random((6, 5)) + 0.5
    _check("Z = (X != 0) * log(X)", {"X": Xp}, ["Z"], "log-nz")
    _check("W = log(X, 2) * (X != 0)", {"X": Xp}, ["W"], "log-nz")
    # zeros: log_nz is 0 where X is 0 (the reference's fused semantics, no 0 * -Inf)
    st, r, _ = _run("Z = (X != 0) * log(X)", {"X": X}, ["Z"])
    assert st.get("log-nz", 0) == 1
    np.testing.assert_allclose(r["Z"], np.where(X != 0, np.log(np.where(X != 0, X, 1)), 0), rtol=1e-12)


def test_sparse_minus_nz_keeps_csr():
    import scipy.sparse as sp
    import torch
    S = sp.random(200, 100, density=0.02, format="csr", random_state=1)
    st, r, _ = _run("Z = S - 0.5 * (S != 0)", {"S": S}, ["Z"])
    st2, r2, _ = _run("n = sum(S != 0)", {"S": S}, ["n"])
    assert st.get("minus-nz", 0) == 1 and st2.get("nnz", 0) == 1
    Z = r["Z"]
    assert r2["n"] == S.nnz
    ref = S.toarray() - 0.5 * (S.toarray() != 0)
    np.testing.assert_allclose(Z if isinstance(Z, np.ndarray) else np.asarray(Z), ref, rtol=1e-12)


def test_datagen_binary():
    src = "R = rand(rows=50, cols=40, min=0, max=1, seed=11) * 4\nS = rand(rows=50, cols=40, min=-1, max=1, seed=12) + 3"
    st, r, _ = _run(src, {}, ["R", "S"])
    assert st.get("datagen-binary", 0) == 2, st
    assert r["R"].min() >= 0 and r["R"].max() <= 4 and r["R"].max() > 3
    assert r["S"].min() >= 2 and r["S"].max() <= 4


def test_bushy_binary():
    X2 = RNG.random((6, 3))
    v = RNG.random((3, 1))
    _check("Z = A * (B3 * (X2 %*% rowSums(V)))", {"A": A, "B3": RNG.random((6, 4)), "X2": X2, "V": v}, ["Z"],
           "bushy-binary")


def test_sliced_matrix_mult():
    _check("P = A %*% t(B2)\nz = as.scalar(P[2, 3])\nP = A", {"A": A, "B2": RNG.random((6, 4))}, ["z"], "sliced-matrix-mult")


def test_constant_and_ordered_sort():
    src = """
    O1 = order(target=matrix(7, rows=5, cols=1))
    O2 = order(target=matrix(7, rows=5, cols=1), index.return=TRUE)
    O3 = order(target=seq(1, 6))
    O4 = order(target=seq(1, 6), decreasing=TRUE)
    O5 = order(target=seq(1, 6), decreasing=TRUE, index.return=TRUE)
    """
    _check(src, {}, ["O1", "O2", "O3", "O4", "O5"], "constant-sort")
    _check(src, {}, ["O1", "O2", "O3", "O4", "O5"], "ordered-sort")


def _stats_all(cs):
    st = dict(cs.cp.rewrite_stats or {})
    st.update(getattr(cs.cp, "licm_stats", {}) or {})
    return st


@pytest.mark.parametrize("src,outs", [
    ("s = 0\nfor (i in 2:5) { s = s + as.scalar(X[i, 2]) }", ["s"]),
    ("s = 1\nfor (i in 1:4) { s = s * as.scalar(X[2, i]) }", ["s"]),
    ("s = 10\nfor (i in 1:6) { s = min(s, as.scalar(X[i, 3])) }", ["s"]),
    ("Z = Y\nfor (i in 1:4) { Z[i, 2] = X[i, 1] * 2 + abs(Y[i, 3]) }", ["Z"]),
    ("Z = Y\nfor (i in 2:4) { Z[1, i] = sqrt(X[3, i]) - Z[1, i] }", ["Z"]),
    ("Z = Y\nc = 0.5\nfor (i in 1:6) { Z[i, 1] = as.scalar(X[i, 2]) * c }", ["Z"]),
    ("Z = Y\nfor (i in 1:6) { Z[i, 4] = 7 }", ["Z"]),
])
def test_for_loop_vectorization(src, outs):
    ins = {"X": RNG.random((6, 4)), "Y": RNG.random((6, 4))}
    cs = EX.compile_script(src + "\nprint(i)", {}, inputs=ins, outputs=outs, config=DMLConfig(gpu=False))
    assert _stats_all(cs).get("for-loop-vectorization", 0) == 1, _stats_all(cs)
    o1 = []
    r1, _ = EX.execute(cs, ins, out=o1.append)
    cs0 = EX.compile_script(src + "\nprint(i)", {}, inputs=ins, outputs=outs, config=DMLConfig(gpu=False, rewrites=False))
    o0 = []
    r0, _ = EX.execute(cs0, ins, out=o0.append)
    assert o1 == o0                    # the loop variable ends at its last value
    for k in outs:
        np.testing.assert_allclose(np.asarray(r1[k], dtype=float), np.asarray(r0[k], dtype=float), rtol=1e-12)


@pytest.mark.parametrize("src", [
    "s = 0\nfor (i in 2:5) { s = s + as.scalar(X[i, 2])\nprint(s) }",        # a second statement
    "Z = Y\nfor (i in 2:5) { Z[i, 2] = Z[i - 1, 2] + 1 }",                 # a recurrence
    "s = 0\nfor (i in 1:6) { s = s + as.scalar(X[i, 2]) * i }",            # the index in the value
])
def test_for_loop_vectorization_declines(src):
    ins = {"X": RNG.random((6, 4)), "Y": RNG.random((6, 4))}
    cs = EX.compile_script(src, {}, inputs=ins, outputs=[], config=DMLConfig(gpu=False))
    assert _stats_all(cs).get("for-loop-vectorization", 0) == 0


def test_for_loop_vectorization_descending_range():
    # 5:2 counts down in DML: the guarded original loop runs
    ins = {"X": RNG.random((6, 4))}
    out = []
    EX.run("s = 3\nn = 2\nfor (i in 5:n) { s = s + as.scalar(X[i, 2]) }\nprint(s)", inputs=ins,
           config=DMLConfig(gpu=False), out=out.append)
    assert float(out[0]) == pytest.approx(3 + ins["X"][1:5, 1].sum(), rel=1e-12)


def test_split_dag_after_data_dependent_operators():
    src = """
    R = removeEmpty(target=X, margin="rows")
    s = sum(R %*% t(R))
    T = table(y, z)
    u = sum(T * 2)
    G = table(seq(1, nrow(y)), y) %*% W
    print(s + u + sum(G))
    """
    X = RNG.random((8, 3))
    X[[1, 4, 6], :] = 0
    ins = {"X": X, "W": RNG.random((3, 2)), "y": np.array([[1.0], [2], [2], [3], [1], [2], [3], [3]]),
           "z": np.array([[2.0], [1], [1], [2], [2], [2], [1], [1]])}
    cs = EX.compile_script(src, {}, inputs=ins, outputs=["s", "u"], config=DMLConfig(gpu=False))
    # removeEmpty and the dimension-free table are cut; the one-hot table product stays a gather
    assert _stats_all(cs).get("split-dag", 0) == 2, _stats_all(cs)
    o1, o0 = [], []
    EX.execute(cs, ins, out=o1.append)
    EX.run(src, inputs=ins, config=DMLConfig(gpu=False, rewrites=False), out=o0.append)
    assert float(o1[0]) == pytest.approx(float(o0[0]), rel=1e-12)


def test_ipa_constant_binary_ops():
    src = """
    w = matrix(1, rows=nrow(X), cols=1)
    if (ncol(X) > 2) { print("wide") }
    Z = X * w
    s = sum(Z)
    """
    X = RNG.random((6, 4))
    cs = EX.compile_script(src, {}, inputs={"X": X}, outputs=["Z", "s"], config=DMLConfig(gpu=False))
    assert cs.cp.ipa_stats.get("constant-binary-ops", 0) == 1, cs.cp.ipa_stats
    r, _ = EX.execute(cs, {"X": X}, out=lambda s: None)
    np.testing.assert_allclose(r["Z"].numpy(), X)


@pytest.mark.parametrize("src,shape", [
    # outer-vector product: n x 1 times a ones row is n x k, never v * 1
    ("o = matrix(1, rows=1, cols=5)\nif (ncol(v) > 2) { print(\"x\") }\nZ = v * o\n", (6, 5)),
    # ones on the left, larger than the vector: n x k, not n x 1
    ("o = matrix(1, rows=nrow(v), cols=5)\nif (ncol(v) > 2) { print(\"x\") }\nZ = o * v\n", (6, 5)),
    # a column vector times a larger ones matrix on the right
    ("o = matrix(1, rows=nrow(v), cols=3)\nif (ncol(v) > 2) { print(\"x\") }\nZ = v * o\n", (6, 3)),
])
def test_ipa_constant_binary_ops_keeps_broadcast_shape(src, shape):
    v = RNG.random((6, 1))
    cs = EX.compile_script(src, {}, inputs={"v": v}, outputs=["Z"], config=DMLConfig(gpu=False))
    assert cs.cp.ipa_stats.get("constant-binary-ops", 0) == 0, cs.cp.ipa_stats
    r, _ = EX.execute(cs, {"v": v}, out=lambda s: None)
    z = r["Z"].numpy()
    assert z.shape == shape
    np.testing.assert_allclose(z, np.broadcast_to(v, shape))


def test_ipa_function_call_sizes():
    """FunctionCallSizeInfo: a function called from the main program with the same argument
    shapes at every site is planned with those shapes (its body's hops are sized)."""
    src = """
    f = function(matrix[double] A, matrix[double] B) return (matrix[double] C) {
      C = A %*% B %*% t(B)
      if (sum(C) > 1e9) { print("big") }
    }
    X = rand(rows=50, cols=20, seed=1)
    Y = rand(rows=20, cols=30, seed=2)
    C1 = f(X, Y)
    C2 = f(X, Y)
    """
    cfg = DMLConfig(gpu=False)          # the body has an if: not inlined
    cs = EX.compile_script(src, {}, outputs=["C1"], config=cfg)
    sized = getattr(cs.cp, "fcall_sized", set())
    assert {p for _, p in sized} >= {"A", "B"}, sized
    text = EX.explain(cs.cp, "hops")
    body = text.split("MAIN PROGRAM")[0]
    assert "M[50x30]" in body or "M[50x20]" in body, body
    r, _ = EX.execute(cs, {}, out=lambda s: None)
    assert tuple(r["C1"].shape) == (50, 20)


def _run_nofuse(src, ins, outs, rewrites=True):
    cfg = DMLConfig(gpu=False, rewrites=rewrites, fusion=False)
    cs = EX.compile_script(src, {}, inputs=ins, outputs=outs, config=cfg)
    r, _ = EX.execute(cs, ins)
    return cs.cp.rewrite_stats or {}, {k: v.double().numpy() for k, v in r.items()}


def test_fuse_axpy_without_operator_fusion():
    src = "s = 0.5\nZ = A + s * B2\nW = A - B2 * 2\nU = (3 * B2) + A"
    ins = {"A": A, "B2": RNG.random((6, 4))}
    st, a = _run_nofuse(src, ins, ["Z", "W", "U"])
    _, b = _run_nofuse(src, ins, ["Z", "W", "U"], rewrites=False)
    assert st.get("fuse-axpy", 0) == 3, st
    for k in ("Z", "W", "U"):
        np.testing.assert_allclose(a[k], b[k], rtol=1e-14)
    np.testing.assert_allclose(a["W"], A - 2 * ins["B2"], rtol=1e-14)


def test_fuse_axpy_keeps_broadcasting_semantics():
    src = "Z = A + 2 * r"                        # r: 1 x 4 row vector broadcast over A's rows
    ins = {"A": A, "r": RNG.random((1, 4))}
    st, a = _run_nofuse(src, ins, ["Z"])
    np.testing.assert_allclose(a["Z"], A + 2 * ins["r"], rtol=1e-14)


def test_order_chain_to_multi_key_order():
    M = np.array([[3, 1, 9], [1, 2, 8], [3, 0, 7], [1, 1, 6], [2, 2, 5], [3, 1, 4]], dtype=float)
    src = "O = order(target=order(target=M, by=2), by=1)\nP = order(target=order(target=M, by=3, decreasing=TRUE), " \
          "by=1, decreasing=TRUE)"
    _check(src, {"M": M}, ["O", "P"], "order-chain")
    st, a, _ = _run(src, {"M": M}, ["O"])
    # lexicographic on (column 1, column 2), stable
    np.testing.assert_array_equal(a["O"][:, :2], [[1, 1], [1, 2], [2, 2], [3, 0], [3, 1], [3, 1]])
