"""Row-template operator fusion (compiler/codegen.fuse_rows, ops/rowgen.py).

Reference tests: src/test/java/org/apache/sysml/test/integration/functions/codegen/
RowAggTmplTest.java (row-wise DAGs -- row aggregates, matrix-vector products, column
aggregates and t(X) %*% f(X %*% v) -- must match the unfused plan and appear as spoof row
operators) and the materialisation choices of PlanSelectionFuseCostBasedV2.  CPU: plan shape,
recomputation of shared matrix-vector products, exact parity with fusion disabled.  GPU: one
generated HIP kernel per program against an fp64 torch evaluation of the same operators."""
import numpy as np
import pytest
import torch

from systemml_amd.api import executor as EX
from systemml_amd.conf import DMLConfig

SCRIPT = """
A = X / rowSums(X)
B = exp(X - rowMaxs(X)); S = B / rowSums(B)
g = t(X) %*% (exp(X %*% v) - y)
c = colSums(X * (X %*% v))
m = max(X %*% v + rowSums(X^2))
r = rowSums(X * (X %*% v)) + y
cm = colMeans((X - rowMeans(X))^2)
"""
OUTS = ["A", "S", "g", "c", "m", "r", "cm"]


def _inputs(n=500, d=37, seed=0):
    rng = np.random.default_rng(seed)
    return {"X": rng.random((n, d)), "v": rng.random((d, 1)), "y": rng.random((n, 1))}


def _row_hops(cs):
    """Descriptions of the Row-template programs of the plan; a merged multi-output program
    (codegen.merge_row_programs) contributes its own and its source programs'."""
    from systemml_amd.compiler import hops as H
    from systemml_amd.compiler.blocks import BasicBlock
    out = []
    for b in cs.cp.blocks:
        if isinstance(b, BasicBlock):
            for h in H.walk(list(b.roots) + list(b.env_out.values())):
                if h.op == "row":
                    out.append(h.p["prog"].describe())
                    out.extend(p.describe() for p, _ in h.p["prog"].parts)
    return out


def test_row_plans_and_parity_with_unfused():
    ins = _inputs()
    cs = EX.compile_script(SCRIPT, {}, inputs=ins, outputs=OUTS, config=DMLConfig(gpu=False))
    fused = _row_hops(cs)
    text = "\n".join(fused)
    assert "row[rsum,/]" in text                             # X / rowSums(X)
    assert "row[rmax,-,exp,rsum,/]" in text                  # softmax, B recomputed in registers
    assert "row[dot,exp,-]|t(.)%*%" in text                  # t(X) %*% f(X %*% v)
    assert "|colsum" in text and "|max" in text and "|colmean" in text
    # X %*% v is shared by four statements; every region streams X anyway, so it is recomputed
    # in each of them and never materialised (no plain matrix product left in the plan)
    plan = EX.explain(cs.cp, "hops")
    assert " mm " not in plan.replace("(", " ").replace(")", " "), plan
    # all regions stream X: they are merged into multi-output programs (one pass over X)
    assert cs.cp.rewrite_stats.get("row-multi-output", 0) >= 1, cs.cp.rewrite_stats
    res, _ = EX.execute(cs, ins)
    cs0 = EX.compile_script(SCRIPT, {}, inputs=ins, outputs=OUTS, config=DMLConfig(gpu=False, fusion=False))
    assert not _row_hops(cs0)
    ref, _ = EX.execute(cs0, ins)
    for k in OUTS:
        a, b = res[k], ref[k]
        if isinstance(a, torch.Tensor):
            assert torch.allclose(a, b, rtol=1e-13, atol=1e-13), k
        else:
            assert float(a) == pytest.approx(float(b), rel=1e-13), k


def test_row_template_numpy_reference():
    ins = _inputs(n=123, d=9, seed=3)
    res, _ = EX.execute(EX.compile_script(SCRIPT, {}, inputs=ins, outputs=OUTS, config=DMLConfig(gpu=False)), ins)
    X, v, y = ins["X"], ins["v"], ins["y"]
    B = np.exp(X - X.max(1, keepdims=True))
    ref = {"A": X / X.sum(1, keepdims=True), "S": B / B.sum(1, keepdims=True),
           "g": X.T @ (np.exp(X @ v) - y), "c": (X * (X @ v)).sum(0, keepdims=True),
           "m": (X @ v + (X ** 2).sum(1, keepdims=True)).max(), "r": (X * (X @ v)).sum(1, keepdims=True) + y,
           "cm": ((X - X.mean(1, keepdims=True)) ** 2).mean(0, keepdims=True)}
    for k in OUTS:
        got = res[k]
        got = got.numpy() if isinstance(got, torch.Tensor) else float(got)
        np.testing.assert_allclose(got, ref[k], rtol=1e-12, atol=1e-12, err_msg=k)


def test_shared_value_with_outside_reader_is_not_recomputed_at_extra_cost():
    # Y is read by the second statement only through a materialised value: recomputing
    # exp(Y) inside the first region would add a full read of Y -> it stays materialised
    src = """
    E = exp(Y)
    a = colSums(X * (X %*% v) + E)
    b = sum(E * 2 + Z)
    """
    rng = np.random.default_rng(1)
    ins = {"X": rng.random((50, 6)), "Y": rng.random((50, 6)), "Z": rng.random((50, 6)), "v": rng.random((6, 1))}
    cs = EX.compile_script(src, {}, inputs=ins, outputs=["a", "b"], config=DMLConfig(gpu=False))
    res, _ = EX.execute(cs, ins)
    X, Y, Z, v = (ins[k] for k in "XYZv")
    np.testing.assert_allclose(res["a"].numpy(), (X * (X @ v) + np.exp(Y)).sum(0, keepdims=True), rtol=1e-12)
    assert float(res["b"]) == pytest.approx((np.exp(Y) * 2 + Z).sum(), rel=1e-12)


def test_row_fallback_errors_like_unfused():
    src = """
    X = rand(rows=5, cols=3, seed=1)
    v = rand(rows=4, cols=1, seed=2)
    print(sum(X / rowSums(X) + exp(X %*% v)))
    """
    with pytest.raises(Exception) as e:
        EX.run(src, config=DMLConfig(gpu=False))
    assert "3" in str(e.value) and "4" in str(e.value)


# ----------------------------------------------------------------------------- GPU kernels
def _ref(prog, args):
    """fp64 torch evaluation of a RowProgram (independent of ops/core)."""
    B = {"+": torch.add, "-": torch.sub, "*": torch.mul, "/": torch.div, "^": torch.pow,
         "min": torch.minimum, "max": torch.maximum, ">": lambda a, b: (a > b).double()}
    U = {"exp": torch.exp, "sq": lambda x: x * x, "abs": torch.abs, "log": torch.log, "sigmoid": torch.sigmoid,
         "sqrt": torch.sqrt, "tanh": torch.tanh}
    RA = {"sum": lambda t: t.sum(1, keepdim=True), "mean": lambda t: t.mean(1, keepdim=True),
          "sumsq": lambda t: (t * t).sum(1, keepdim=True), "max": lambda t: t.amax(1, keepdim=True),
          "min": lambda t: t.amin(1, keepdim=True)}
    vals = [a.double().cpu() if isinstance(a, torch.Tensor) else
            (torch.tensor(float(a.value()), dtype=torch.float64) if hasattr(a, "value") else
             torch.tensor(float(a), dtype=torch.float64)) for a in args]
    for kind, o, a, b in prog.ops:
        if kind == "b":
            vals.append(B[o](vals[a], vals[b]))
        elif kind == "u":
            vals.append(U[o](vals[a]))
        elif kind == "ragg":
            vals.append(RA[o](vals[a]))
        else:
            vals.append(vals[a] @ vals[b])
    r = vals[prog.out]
    ot = prog.otype
    if ot == "col":
        r = {"sum": r.sum(0, keepdim=True), "mean": r.mean(0, keepdim=True),
             "sumsq": (r * r).sum(0, keepdim=True)}[prog.oagg]
    elif ot == "tmv":
        r = r.t() @ vals[prog.extra]
    elif ot == "all":
        r = {"sum": r.sum(), "mean": r.mean(), "sumsq": (r * r).sum(), "max": r.max(), "min": r.min()}[prog.oagg]
    return r


def _gpu_check(prog, args, precision="single", tol=2e-5):
    from systemml_amd.ops import rowgen, kernels
    from systemml_amd.ops.backend import backend
    backend.configure(DMLConfig(gpu=True, precision=precision))
    dev = torch.device("cuda:0")
    dargs = [a.to(dev) if isinstance(a, torch.Tensor) else a for a in args]
    c0 = kernels.counters.get("row", 0)
    got = rowgen._kernel(prog, dargs)
    assert got is not None, "operands outside the kernel's scope"
    torch.cuda.synchronize()
    assert kernels.counters.get("row", 0) == c0 + 1
    ref = _ref(prog, args)
    g = torch.as_tensor(got.value() if hasattr(got, "value") else got, dtype=torch.float64).cpu()
    ref = ref.reshape(g.shape)
    scale = ref.abs().max().item() + 1e-30
    err = (g - ref).abs().max().item() / scale
    assert err < tol, err
    return got


def _mk(shape, dt, seed, lo=-1.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(shape, generator=g, dtype=torch.float64) * (hi - lo) + lo).to(dt)


SHAPES = [(1000, 5), (3001, 37), (257, 130), (2049, 1000), (17, 4100)]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dt", [torch.float32, torch.float64, torch.bfloat16])
def test_row_kernel_tmv_chain(shape, dt):
    from systemml_amd.ops.rowgen import RowProgram
    n, d = shape
    # t(X) %*% (exp(X %*% v) * w - y): w 1x1 device matrix, y N x 1
    prog = RowProgram(4, [("dot", None, 0, 1), ("u", "exp", 4, 0), ("b", "*", 5, 2), ("b", "-", 6, 3)],
                      0, "tmv", extra=7)
    X = _mk((n, d), dt, 1)
    v = _mk((d, 1), torch.float32, 2, -0.5 / d ** 0.5, 0.5 / d ** 0.5)
    _gpu_check(prog, [X, v, _mk((1, 1), torch.float32, 3), _mk((n, 1), torch.float32, 4)],
               "double" if dt == torch.float64 else "single", 1e-11 if dt == torch.float64 else 2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("otype", ["vec", "row", "col", "all"])
def test_row_kernel_softmax_and_outputs(shape, otype):
    from systemml_amd.ops.rowgen import RowProgram
    n, d = shape
    # P = exp(X - rowMaxs(X)) / rowSums(exp(X - rowMaxs(X))) * w + rowMeans(X); then per otype
    ops = [("ragg", "max", 0, 0), ("b", "-", 0, 2), ("u", "exp", 3, 0), ("ragg", "sum", 4, 0), ("b", "/", 4, 5),
           ("b", "*", 6, 1), ("ragg", "mean", 0, 0), ("b", "+", 7, 8)]
    out = 9
    if otype == "row":
        ops.append(("ragg", "sumsq", 9, 0))
        out = 10
    prog = RowProgram(2, ops, out, otype, oagg={"col": "mean", "all": "max"}.get(otype))
    _gpu_check(prog, [_mk((n, d), torch.float32, 5, -3, 3), _mk((1, d), torch.float32, 6)], tol=2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("agg", ["sum", "sumsq", "mean", "min", "max"])
def test_row_kernel_full_aggregates_and_device_scalars(agg):
    from systemml_amd.ops.rowgen import RowProgram
    from systemml_amd.runtime.scalars import DevScalar
    # agg((X - s)^2 / rowSums(abs(X)) + X %*% v) -- a per-row scalar plus a row vector
    prog = RowProgram(3, [("b", "-", 0, 1), ("u", "sq", 3, 0), ("u", "abs", 0, 0), ("ragg", "sum", 5, 0),
                          ("b", "/", 4, 6), ("dot", None, 0, 2), ("b", "+", 7, 8)], 9, "all", oagg=agg)
    X = _mk((4099, 63), torch.float32, 7)
    s = DevScalar(torch.tensor(0.25, dtype=torch.float64, device="cuda"))
    _gpu_check(prog, [X, s, _mk((63, 1), torch.float32, 8)], tol=2e-5)


@pytest.mark.gpu
def test_row_script_on_gpu_matches_cp():
    from systemml_amd.ops import rowgen
    ins = _inputs(n=3001, d=37, seed=4)
    ref, _ = EX.execute(EX.compile_script(SCRIPT, {}, inputs=ins, outputs=OUTS, config=DMLConfig(gpu=False)), ins)
    k0 = rowgen.stats["kernel"]
    cfg = DMLConfig(gpu=True, precision="double", gpu_min_cells=0)
    got, _ = EX.execute(EX.compile_script(SCRIPT, {}, inputs=ins, outputs=OUTS, config=cfg), ins)
    assert rowgen.stats["kernel"] >= k0 + 7
    for k in OUTS:
        a, b = got[k], ref[k]
        a = a.double().cpu() if isinstance(a, torch.Tensor) else torch.tensor(float(a.value() if hasattr(a, "value") else a))
        b = b.double().cpu() if isinstance(b, torch.Tensor) else torch.tensor(float(b))
        assert torch.allclose(a, b, rtol=1e-9, atol=1e-9), k


# ----------------------------------------------------------------------------- K-wide row vectors
def _ref_w(prog, args):
    """fp64 torch evaluation of a RowProgram with K-wide vectors and several outputs."""
    B = {"+": torch.add, "-": torch.sub, "*": torch.mul, "/": torch.div}
    U = {"exp": torch.exp, "log": torch.log, "sq": lambda x: x * x}
    RA = {"sum": lambda t: t.sum(1, keepdim=True), "max": lambda t: t.amax(1, keepdim=True),
          "mean": lambda t: t.mean(1, keepdim=True)}
    vals = [a.double().cpu() if isinstance(a, torch.Tensor) else torch.tensor(float(a), dtype=torch.float64)
            for a in args]
    for kind, o, a, b in prog.ops:
        if kind == "b":
            vals.append(B[o](vals[a], vals[b]))
        elif kind == "u":
            vals.append(U[o](vals[a]))
        elif kind == "ragg":
            vals.append(RA[o](vals[a]))
        elif kind == "cbindc":
            vals.append(torch.cat([vals[a], vals[b].reshape(1, 1).expand(vals[a].shape[0], 1)], 1))
        elif kind == "wcols":
            vals.append(vals[a][:, :b])
        else:
            vals.append(vals[a] @ vals[b])
    res = []
    for node, ot, oagg, extra in prog.outputs():
        r = vals[node]
        if ot == "tmv":
            r = r.t() @ vals[extra]
        elif ot == "col":
            r = r.sum(0, keepdim=True)
        elif ot == "all":
            r = r.sum() if oagg == "sum" else r.max()
        res.append(r)
    return res


def _softmax_objective_program():
    from systemml_amd.ops.rowgen import RowProgram
    # inputs: 0 X (N x D), 1 B (D x K side), 2 Y (N x K+1), 3 c (scalar 0), 4 Yk (N x K)
    ops = [("dot", None, 0, 1),          # 5  W = X %*% B
           ("cbindc", None, 5, 3),       # 6  LT = cbind(W, 0)
           ("ragg", "max", 6, 0),        # 7  rowMaxs(LT)
           ("b", "-", 6, 7),             # 8  LT - rowMaxs
           ("u", "exp", 8, 0),           # 9  E
           ("ragg", "sum", 9, 0),        # 10 rowSums(E)
           ("b", "/", 9, 10),            # 11 P
           ("b", "*", 2, 8),             # 12 Y * LT
           ("u", "log", 10, 0),          # 13 log(rowSums(E))
           ("wcols", None, 11, None),    # 14 P[, 1:K]  (k filled below)
           ("b", "-", 14, 4)]            # 15 P[, 1:K] - Yk
    return ops


@pytest.mark.gpu
@pytest.mark.parametrize("n,d,k", [(2049, 1000, 5), (3001, 37, 3), (257, 130, 10), (40000, 256, 2)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_row_kernel_side_matrix_multi_output(n, d, k, dt):
    """The MultiLogReg candidate pass as ONE generated program: X %*% B (D x K side matrix),
    cbind of the baseline column, row max / exp / row sum softmax, the objective's data terms
    and t(X) %*% (P[, 1:K] - Y[, 1:K]) -- five outputs from one pass over X."""
    from systemml_amd.ops import rowgen, kernels
    from systemml_amd.ops.rowgen import RowProgram
    from systemml_amd.ops.backend import backend
    ops = _softmax_objective_program()
    ops[9] = ("wcols", None, 11, k)
    prog = RowProgram(5, ops, 11, "vec", more=[(12, "all", "sum", None), (13, "all", "sum", None),
                                              (0, "tmv", None, 15), (10, "row", None, None)])
    X = _mk((n, d), dt, 1)
    Bm = _mk((d, k), torch.float32, 2, -2.0 / d ** 0.5, 2.0 / d ** 0.5)
    Y = torch.zeros(n, k + 1)
    Y[torch.arange(n), torch.randint(0, k + 1, (n,), generator=torch.Generator().manual_seed(3))] = 1.0
    args = [X, Bm, Y, 0.0, Y[:, :k].contiguous()]
    backend.configure(DMLConfig(gpu=True, precision="single"))
    dev = torch.device("cuda:0")
    dargs = [a.to(dev) if isinstance(a, torch.Tensor) else a for a in args]
    c0 = kernels.counters.get("row", 0)
    got = rowgen._kernel(prog, dargs)
    assert got is not None, "operands outside the kernel's scope"
    torch.cuda.synchronize()
    assert kernels.counters.get("row", 0) == c0 + 1 and len(got) == 5
    refs = _ref_w(prog, [X.double(), Bm, Y, 0.0, Y[:, :k]])
    for q, (g, r) in enumerate(zip(got, refs)):
        g = torch.as_tensor(g.value() if hasattr(g, "value") else g, dtype=torch.float64).cpu().reshape(r.shape)
        err = (g - r).abs().max().item() / (r.abs().max().item() + 1e-30)
        assert err < 2e-5, (q, err)


@pytest.mark.gpu
def test_multilogreg_pass_planned_by_row_template_on_gpu():
    """With the hand matcher off, the candidate pass of MultiLogReg is planned by the Row
    template (merged multi-output program) and runs as generated kernels on the GPU, matching
    the CPU plan."""
    import systemml_amd.compiler.rewrites as RW
    from systemml_amd.ops import rowgen
    src = """
    LT = cbind(X %*% B, matrix(0, rows=nrow(X), cols=1))
    LT = LT - rowMaxs(LT)
    E = exp(LT)
    P = E / rowSums(E)
    o1 = sum(Y * LT)
    o2 = sum(log(rowSums(E)))
    G = t(X) %*% (P[, 1:4] - Y[, 1:4])
    """
    rng = np.random.default_rng(0)
    ins = {"X": rng.standard_normal((20000, 300)) * 0.05, "B": rng.standard_normal((300, 4)),
           "Y": np.eye(5)[rng.integers(0, 5, 20000)]}
    outs = ["P", "o1", "o2", "G"]
    old = RW.SOFTMAX_MATCHER
    RW.SOFTMAX_MATCHER = False
    try:
        res = {}
        for gpu in (True, False):
            cfg = DMLConfig(gpu=gpu, precision="double", gpu_min_cells=0)
            cs = EX.compile_script(src, {}, inputs=ins, outputs=outs, config=cfg)
            assert cs.cp.rewrite_stats.get("row-multi-output", 0) >= 1, cs.cp.rewrite_stats
            k0 = rowgen.stats["kernel"]
            r, _ = EX.execute(cs, ins)
            if gpu:
                assert rowgen.stats["kernel"] > k0
            res[gpu] = {k: (v.double().cpu().numpy() if hasattr(v, "numpy") else np.array(float(v))) for k, v in r.items()}
    finally:
        RW.SOFTMAX_MATCHER = old
    for k in outs:
        np.testing.assert_allclose(res[True][k], res[False][k], rtol=1e-9, atol=1e-9, err_msg=k)




def test_softmax_layer_forward_backward_row_fused():
    """nn/layers/softmax.dml forward and backward each become ONE Row-template operator."""
    import os
    from systemml_amd.api.mlcontext import SCRIPTS_DIR
    src = 'source("nn/layers/softmax.dml") as softmax\nP = softmax::forward(S)\ndS = softmax::backward(dP, S)'
    rng = np.random.default_rng(4)
    ins = {"S": rng.standard_normal((300, 10)), "dP": rng.standard_normal((300, 10))}
    cs = EX.compile_script(src, {}, inputs=ins, outputs=["P", "dS"], config=DMLConfig(gpu=False),
                           filename=os.path.join(SCRIPTS_DIR, "sm.dml"))
    main = EX.explain(cs.cp, "runtime").split("MAIN PROGRAM")[1]
    ops = [ln.split()[0] for ln in main.splitlines()[1:] if ln.strip()]
    assert ops.count("spoofRA") + ops.count("fout") >= 2 and "rowSums" not in main, main
    res, _ = EX.execute(cs, ins)
    S, dP = ins["S"], ins["dP"]
    e = np.exp(S - S.max(1, keepdims=True))
    P = e / e.sum(1, keepdims=True)
    np.testing.assert_allclose(res["P"].numpy(), P, rtol=1e-12)
    np.testing.assert_allclose(res["dS"].numpy(), P * (dP - (dP * P).sum(1, keepdims=True)), rtol=1e-12)
