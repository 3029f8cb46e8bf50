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
    return [ln for ln in EX.explain(cs.cp, "hops").splitlines() if "row[" in ln]


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
