"""Cell-template operator fusion (compiler/codegen.py, ops/cell.py, ops/hip/cell.hip).

Reference tests: src/test/java/org/apache/sysml/test/integration/functions/codegen/
CellwiseTmplTest.java (fused cellwise DAGs with none / full / row / column aggregation must
match the unfused plan and must show up as spoof operators in the plan).  CPU: plan shape and
exact equality with fusion disabled.  GPU: one HIP kernel per fused DAG against an fp64 torch
evaluation of the same operators, every opcode, broadcast mode, input dtype and aggregate."""
import math

import numpy as np
import pytest
import torch

from systemml_amd.api import executor as EX
from systemml_amd.conf import DMLConfig

SCRIPT = """
Z = exp(X * 2 - y) / (1 + abs(X)) + w
s = sum((X - 0.5)^2 * y + sqrt(abs(X)))
r = rowSums(sigmoid(X) * X - w)
c = colMeans(log(abs(X) + 1) * y)
mx = max(tanh(X) - X %% 0.3)
mn = rowMins(floor(X * 3) + (X > 0.5))
q = sum(Z) + s + sum(r) + sum(c) + mx + sum(mn)
"""


def _run(cfg, n=57, m=13):
    rng = np.random.default_rng(n * m)
    ins = {"X": rng.uniform(-1, 2, (n, m)), "y": rng.uniform(0.5, 1.5, (n, 1)), "w": rng.uniform(0, 1, (1, m))}
    cs = EX.compile_script(SCRIPT, {}, inputs=ins, outputs=["q", "Z", "r", "c"], config=cfg)
    res, _ = EX.execute(cs, ins)
    return cs, res


def _fused_hops(cs):
    text = EX.explain(cs.cp, "hops")
    return [ln for ln in text.splitlines() if "cell[" in ln]


def test_cell_plans_and_parity_with_unfused():
    cs, res = _run(DMLConfig(gpu=False))
    fused = _fused_hops(cs)
    # Z (block output), full-sum, row / col aggregates, max, rowMins
    assert any("|sum-all" in ln for ln in fused), fused
    assert any("|sum-row" in ln for ln in fused), fused
    assert any("|mean-col" in ln for ln in fused), fused
    assert any("|max-all" in ln for ln in fused), fused
    assert any("|min-row" in ln for ln in fused), fused
    cs0, ref = _run(DMLConfig(gpu=False, fusion=False))
    assert not _fused_hops(cs0)
    for k in ("q", "Z", "r", "c"):
        a, b = res[k], ref[k]
        if isinstance(a, torch.Tensor):
            assert torch.equal(a, b), k
        else:
            assert a == b, k


def test_shared_intermediate_recomputed_when_cheaper():
    """Cost-based materialisation (reference PlanSelectionFuseCostBasedV2): T = exp(X) + 1 has
    two aggregate consumers; recomputing it inside both reads X once in ONE multi-aggregate
    pass instead of writing T and reading it twice."""
    src = """
    X = rand(rows=20, cols=4, seed=5)
    T = exp(X) + 1
    a = sum(T * 2 + X)
    b = sum(T / 3 - X)
    print(a + b)
    """
    cs = EX.compile_script(src, {}, config=DMLConfig(gpu=False))
    fused = _fused_hops(cs)
    assert len(fused) == 1 and "magg[" in fused[0] and "exp" in fused[0], fused
    assert cs.cp.rewrite_stats.get("cell-plan-inlined", 0) >= 1
    out, ref = [], []
    EX.run(src, config=DMLConfig(gpu=False), out=out.append)
    EX.run(src, config=DMLConfig(gpu=False, fusion=False), out=ref.append)
    assert abs(float(out[0]) - float(ref[0])) < 1e-12 * abs(float(ref[0]))


def test_shared_intermediate_materialised_for_a_matrix_product():
    """A shared intermediate that a non-cellwise consumer needs anyway is materialised once;
    its cellwise consumer reads it instead of recomputing exp."""
    src = """
    X = rand(rows=20, cols=4, seed=5)
    v = rand(rows=4, cols=1, seed=6)
    T = exp(X) + 1
    a = sum(T %*% v)
    b = sum(T * 2)
    print(a + b)
    """
    cs = EX.compile_script(src, {}, config=DMLConfig(gpu=False))
    fused = _fused_hops(cs)
    assert any("cell[exp,+]" in ln for ln in fused), fused
    assert cs.cp.rewrite_stats.get("cell-plan-inlined", 0) == 0


def test_sequential_fallback_errors_like_unfused():
    src = """
    X = rand(rows=5, cols=3, seed=1)
    Y = rand(rows=4, cols=3, seed=2)
    Z = exp(X) + Y * 2
    print(sum(Z))
    """
    with pytest.raises(Exception) as e1:
        EX.run(src, config=DMLConfig(gpu=False))
    assert "5x3" in str(e1.value) and "4x3" in str(e1.value)


# ----------------------------------------------------------------------------- GPU kernel
def _ref_eval(prog, args):
    """fp64 torch evaluation of a CellProgram (the test's independent reference)."""
    import systemml_amd.ops.core as C
    B = {"+": torch.add, "-": torch.sub, "*": torch.mul, "/": torch.div, "^": torch.pow,
         "%%": torch.remainder, "%/%": lambda a, b: torch.floor(a / b),
         "==": lambda a, b: (a == b).double(), "!=": lambda a, b: (a != b).double(),
         "<": lambda a, b: (a < b).double(), "<=": lambda a, b: (a <= b).double(),
         ">": lambda a, b: (a > b).double(), ">=": lambda a, b: (a >= b).double(),
         "&": lambda a, b: ((a != 0) & (b != 0)).double(), "|": lambda a, b: ((a != 0) | (b != 0)).double(),
         "xor": lambda a, b: ((a != 0) ^ (b != 0)).double(), "min": torch.minimum, "max": torch.maximum,
         "log": lambda a, b: torch.log(a) / torch.log(b)}
    U = dict(C.UN)
    U["sq"] = lambda x: x * x
    regs = []
    for a in args:
        if isinstance(a, torch.Tensor):
            regs.append(a.double().cpu())
        else:
            regs.append(torch.tensor(float(a), dtype=torch.float64))
    regs += [None] * (16 - len(regs))
    for kind, o, d, a, b in prog.ops:
        regs[d] = B[o](regs[a], regs[b]) if kind == "b" else U[o](regs[a])
    r = regs[prog.out]
    if prog.agg:
        o, dr = prog.agg
        dim = None if dr == "all" else (1 if dr == "row" else 0)
        f = {"sum": torch.sum, "sumsq": lambda t, **k: torch.sum(t * t, **k), "mean": torch.mean,
             "min": torch.amin, "max": torch.amax}[o]
        r = f(r) if dim is None else f(r, dim=dim, keepdim=True)
    return r


BIN_OPS = ["+", "-", "*", "/", "^", "%%", "%/%", "==", "!=", "<", "<=", ">", ">=", "&", "|", "xor", "min",
           "max", "log"]
UN_OPS = ["sq", "neg", "not", "abs", "exp", "log", "sqrt", "round", "floor", "ceil", "sign", "sin", "cos",
          "tan", "asin", "acos", "atan", "sinh", "cosh", "tanh", "sigmoid"]


def _mk(shape, dt, seed, lo=0.2, hi=1.7):
    g = torch.Generator().manual_seed(seed)
    t = torch.rand(shape, generator=g, dtype=torch.float64) * (hi - lo) + lo
    return t.to(dt)


def _check(prog, args, dt_out, tol, rtc=True):
    from systemml_amd.ops import cell, kernels
    from systemml_amd.ops.backend import backend
    cell.RTC = rtc
    n_rtc = cell.stats["rtc_launches"]
    backend.configure(DMLConfig(gpu=True, precision="single" if dt_out == torch.float32 else "double"))
    dev = torch.device("cuda:0")
    dargs = [a.to(dev) if isinstance(a, torch.Tensor) else a for a in args]
    c0 = kernels.counters.get("cell", 0)
    try:
        got = cell._kernel(prog, dargs)
    finally:
        cell.RTC = True
    assert got is not None
    torch.cuda.synchronize()
    assert kernels.counters.get("cell", 0) == c0 + 1
    assert cell.stats["rtc_launches"] == n_rtc + (1 if rtc else 0)     # generated kernel vs interpreter
    ref = _ref_eval(prog, [a.double() if isinstance(a, torch.Tensor) else a for a in args])
    g = torch.as_tensor(got.value() if hasattr(got, "value") else got, dtype=torch.float64).cpu()
    if isinstance(got, torch.Tensor):
        assert got.dtype == dt_out
    ref = ref.reshape(g.shape)
    fin = torch.isfinite(ref)
    assert torch.equal(torch.isnan(g), torch.isnan(ref))
    scale = ref[fin].abs().max().item() + 1e-30 if fin.any() else 1.0
    err = ((g[fin] - ref[fin]).abs().max().item() / scale) if fin.any() else 0.0
    assert err < tol, err


@pytest.mark.gpu
@pytest.mark.parametrize("dt,tol", [(torch.float64, 1e-12), (torch.float32, 2e-6)])
@pytest.mark.parametrize("op", BIN_OPS)
def test_cell_kernel_binary_ops(op, dt, tol):
    from systemml_amd.ops.cell import CellProgram
    # (X op Y) * 1.5 over a ragged 37 x 29 matrix
    prog = CellProgram([("b", op, 3, 0, 1), ("b", "*", 3, 3, 2)], 3, 3)
    X, Y = _mk((37, 29), dt, 1), _mk((37, 29), dt, 2)
    if op in ("==", "!=", "<=", ">="):
        Y[::3] = X[::3]
    _check(prog, [X, Y, 1.5], dt, tol)


@pytest.mark.gpu
@pytest.mark.parametrize("rtc", [True, False])
@pytest.mark.parametrize("dt,tol", [(torch.float64, 1e-12), (torch.float32, 4e-6)])
@pytest.mark.parametrize("op", UN_OPS)
def test_cell_kernel_unary_ops(op, dt, tol, rtc):
    from systemml_amd.ops.cell import CellProgram
    lo, hi = (-0.9, 0.9) if op in ("asin", "acos", "atanh") else (-2.5, 2.5)
    if op in ("log", "sqrt"):
        lo, hi = 0.05, 3.0
    prog = CellProgram([("u", op, 1, 0, 0), ("b", "+", 1, 1, 0)], 1, 1)
    X = _mk((41, 23), dt, 3, lo, hi)
    _check(prog, [X], dt, tol, rtc)


@pytest.mark.gpu
@pytest.mark.parametrize("agg", [None, ("sum", "all"), ("sumsq", "all"), ("mean", "all"), ("min", "all"),
                                 ("max", "all"), ("sum", "row"), ("mean", "row"), ("max", "row"),
                                 ("sum", "col"), ("min", "col"), ("mean", "col")])
@pytest.mark.parametrize("shape", [(1000, 5), (3001, 7), (257, 130), (9, 1000), (4099, 1),
                                   (300, 1024), (64, 2052)])   # wide: 4-column lanes, 2 / 1 row blocks
@pytest.mark.parametrize("rtc", [True, False])
def test_cell_kernel_broadcast_and_aggregates(shape, agg, rtc):
    from systemml_amd.ops.cell import CellProgram
    from systemml_amd.runtime.scalars import DevScalar
    n, m = shape
    # exp(X * w - y) / (1 + abs(X)) - s  with w a row vector, y a column vector, s a 1x1 matrix
    prog = CellProgram([("b", "*", 5, 0, 1), ("b", "-", 5, 5, 2), ("u", "exp", 5, 5, 0),
                        ("u", "abs", 6, 0, 0), ("b", "+", 6, 6, 4), ("b", "/", 5, 5, 6),
                        ("b", "-", 5, 5, 3)], 5, 5, agg)
    X = _mk((n, m), torch.float32, 5, -1, 1)
    w = _mk((1, m), torch.float32, 6)
    y = _mk((n, 1), torch.float32, 7)
    s = _mk((1, 1), torch.float32, 8)
    _check(prog, [X, w, y, s, 1.0], torch.float32, 3e-6 if agg is None or agg[0] in ("min", "max") else 1e-5, rtc)


@pytest.mark.gpu
def test_cell_kernel_bf16_inputs_views_and_device_scalars():
    from systemml_amd.ops.cell import CellProgram
    from systemml_amd.runtime.scalars import DevScalar
    from systemml_amd.ops.backend import backend
    backend.configure(DMLConfig(gpu=True, precision="single"))
    dev = torch.device("cuda:0")
    prog = CellProgram([("b", "*", 3, 0, 2), ("b", "+", 3, 3, 1), ("u", "sigmoid", 3, 3, 0)], 3, 3, ("sum", "row"))
    X = _mk((5003, 64), torch.float64, 9, -2, 2).to(torch.bfloat16)
    Y = _mk((5003, 65), torch.float32, 10)[:, 1:]       # strided view, not 16-B aligned
    ds = DevScalar(torch.tensor(0.75, dtype=torch.float64, device=dev))
    from systemml_amd.ops import cell
    got = cell._kernel(prog, [X.to(dev), Y.to(dev), ds])
    ref = torch.sigmoid(X.double() * 0.75 + Y.double()).sum(1, keepdim=True)
    err = (got.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, err


@pytest.mark.gpu
def test_fused_script_on_gpu_matches_cp():
    from systemml_amd.ops import kernels
    _, ref = _run(DMLConfig(gpu=False), n=3001, m=37)
    def fused():
        return kernels.counters.get("cell", 0) + kernels.counters.get("row", 0)
    c0, m0 = fused(), kernels.counters.get("magg", 0)
    _, got = _run(DMLConfig(gpu=True, precision="double", gpu_min_cells=0), n=3001, m=37)
    # Z, the row / column aggregates and rowMins as cell kernels (sum(rowMins(..)) as a row
    # kernel); sum(...) and max(...) over X as one multi-aggregate kernel
    assert fused() >= c0 + 4
    assert kernels.counters.get("magg", 0) >= m0 + 1
    for k in ("q", "Z", "r", "c"):
        a, b = got[k], ref[k]
        a = a.double().cpu() if isinstance(a, torch.Tensor) else torch.tensor(float(a))
        b = b.double().cpu() if isinstance(b, torch.Tensor) else torch.tensor(float(b))
        assert torch.allclose(a, b, rtol=1e-9, atol=1e-9), k


def test_multi_aggregate_template_parity():
    """Full aggregates over shared inputs become one magg operator (reference
    TemplateMultiAgg / MultiAggTmplTest) and match the unfused evaluation."""
    src = """
    a = sum(X * Y)
    b = sum(X ^ 2)
    c = sum(Y ^ 2 + 1)
    d = max(X - Y)
    e = min(abs(X) * 2)
    q = a + b + c + d + e
    """
    rng = np.random.default_rng(11)
    ins = {"X": rng.standard_normal((33, 7)), "Y": rng.standard_normal((33, 7))}
    outs = ["a", "b", "c", "d", "e"]
    cs = EX.compile_script(src, {}, inputs=ins, outputs=outs, config=DMLConfig(gpu=False))
    text = EX.explain(cs.cp, "hops")
    assert "magg[" in text, text
    res, _ = EX.execute(cs, ins)
    cs0 = EX.compile_script(src, {}, inputs=ins, outputs=outs, config=DMLConfig(gpu=False, fusion=False))
    ref, _ = EX.execute(cs0, ins)
    for k in outs:
        assert float(res[k]) == pytest.approx(float(ref[k]), rel=1e-12), k


@pytest.mark.gpu
def test_multi_aggregate_kernel_gpu():
    """One generated HIP kernel for the multi-aggregate (fp32 / fp64 / bf16 inputs, row and
    column broadcast operands) against an fp64 torch evaluation."""
    from systemml_amd.ops import cell as CELL
    src = """
    a = sum(X * Y)
    b = sum((X - v) ^ 2)
    c = max(X * w)
    d = min(Y + v)
    e = mean(X / 3)
    """
    rng = np.random.default_rng(12)
    for dt in (torch.float32, torch.float64, torch.bfloat16):
        X = torch.from_numpy(rng.standard_normal((1003, 37))).to("cuda", dt)
        Y = torch.from_numpy(rng.standard_normal((1003, 37))).to("cuda", dt)
        v = torch.from_numpy(rng.standard_normal((1003, 1))).to("cuda", torch.float32)
        w = torch.from_numpy(rng.standard_normal((1, 37))).to("cuda", torch.float32)
        ins = {"X": X, "Y": Y, "v": v, "w": w}
        before = CELL.stats.get("magg_kernel", 0)
        cs = EX.compile_script(src, {}, inputs=ins, outputs=list("abcde"), config=DMLConfig(gpu=True, precision="double"))
        res, _ = EX.execute(cs, ins)
        assert CELL.stats.get("magg_kernel", 0) > before
        Xd, Yd, vd, wd = (t.double() for t in (X, Y, v, w))
        ref = {"a": (Xd * Yd).sum(), "b": ((Xd - vd) ** 2).sum(), "c": (Xd * wd).max(), "d": (Yd + vd).min(),
               "e": (Xd / 3).mean()}
        for k, r in ref.items():
            got = res[k]
            got = float(got.value()) if hasattr(got, "value") else float(got)
            assert got == pytest.approx(float(r), rel=1e-6 if dt == torch.float32 else 1e-9, abs=1e-9), (k, dt)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows", [256, 1000])
def test_cell_kernel_channel_column_sums(dt, rows):
    """colSums((X - m per channel)^2) over an N x (C*HW) activation (the batch-norm variance
    pass): 4-column lanes with vector loads, per-channel operand, one or several row blocks."""
    from systemml_amd.ops.cell import CellProgram
    from systemml_amd.ops import cell
    from systemml_amd.ops.backend import backend
    backend.configure(DMLConfig(gpu=True, precision="single"))
    dev = torch.device("cuda:0")
    C, HW = 16, 196
    prog = CellProgram([("b", "bias+", 2, 0, 1), ("u", "sq", 2, 2, 0)], 2, 2, ("sum", "col"))
    X = _mk((rows, C * HW), torch.float64, 21, -2, 2).to(dt)
    m = _mk((C, 1), torch.float32, 22, -0.5, 0.5)
    got = cell._kernel(prog, [X.to(dev), m.to(dev)])
    torch.cuda.synchronize()
    ref = ((X.double().reshape(rows, C, HW) + m.double().reshape(1, C, 1)) ** 2).reshape(rows, -1).sum(0, keepdim=True)
    assert got.shape == (1, C * HW)
    err = (got.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, err


BIAS_SCRIPT = """
Xc = bias_add(X, -m)
norm = bias_multiply(Xc, istd)
out = max(bias_add(bias_multiply(norm, g), b), 0)
s = sum(out)
"""


def _bias_inputs(N=6, C=10, HW=9, seed=0):
    rng = np.random.default_rng(seed)
    return {"X": rng.standard_normal((N, C * HW)), "m": rng.standard_normal((C, 1)), "istd": rng.random((C, 1)),
            "g": rng.random((C, 1)), "b": rng.standard_normal((C, 1))}


def test_bias_ops_fuse_with_cellwise_chains():
    """bias_add / bias_multiply (per-channel broadcasts of batch-norm / scale layers) fuse into
    the Cell template with the surrounding cellwise work; results equal the unfused plan."""
    ins = _bias_inputs()
    cs = EX.compile_script(BIAS_SCRIPT, {}, inputs=ins, outputs=["norm", "out", "s"], config=DMLConfig(gpu=False))
    fused = _fused_hops(cs)
    assert any("cell[bias+,bias*]" in ln for ln in fused), fused
    assert any("cell[bias*,bias+,max]" in ln for ln in fused), fused
    res, _ = EX.execute(cs, ins)
    cs0 = EX.compile_script(BIAS_SCRIPT, {}, inputs=ins, outputs=["norm", "out", "s"],
                            config=DMLConfig(gpu=False, fusion=False))
    ref, _ = EX.execute(cs0, ins)
    for k in ("norm", "out"):
        assert torch.equal(res[k], ref[k]), k
    assert float(res["s"]) == float(ref["s"])


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(6, 10, 9), (32, 64, 3136), (3, 7, 1), (5, 3, 2), (7, 1, 1), (3, 5, 6),
                                   (2, 3, 8), (4, 6, 4), (3, 5, 12)])          # last three: one channel per 4-cell group
def test_bias_ops_cell_kernel_gpu(shape):
    from systemml_amd.ops import kernels
    N, C, HW = shape
    ins = _bias_inputs(N, C, HW, seed=N)
    c0 = kernels.counters.get("cell", 0)
    cfg = DMLConfig(gpu=True, precision="double", gpu_min_cells=0)
    got, _ = EX.execute(EX.compile_script(BIAS_SCRIPT, {}, inputs=ins, outputs=["norm", "out", "s"], config=cfg), ins)
    assert kernels.counters.get("cell", 0) >= c0 + 2
    X, m, istd, g, b = (torch.from_numpy(ins[k]) for k in ("X", "m", "istd", "g", "b"))
    ch = lambda v: v.reshape(1, C, 1)
    norm = ((X.reshape(N, C, HW) - ch(m)) * ch(istd))
    out = torch.clamp(norm * ch(g) + ch(b), min=0)
    assert torch.allclose(got["norm"].double().cpu(), norm.reshape(N, -1), rtol=1e-12, atol=1e-12)
    assert torch.allclose(got["out"].double().cpu(), out.reshape(N, -1), rtol=1e-12, atol=1e-12)


def test_conv2d_bias_add_rewrite():
    """bias_add(conv2d(..)) becomes one conv2d with a bias operand (reference DnnOp
    CONV2D_BIAS_ADD) when the convolution has no other consumer; results are unchanged."""
    src = """
o = conv2d(X, W, input_shape=[4,2,6,6], filter_shape=[3,2,3,3], stride=[1,1], padding=[1,1])
o = bias_add(o, b)
s = sum(o)
"""
    rng = np.random.default_rng(2)
    ins = {"X": rng.random((4, 72)), "W": rng.random((3, 18)) - 0.5, "b": rng.random((3, 1))}
    cs = EX.compile_script(src, {}, inputs=ins, outputs=["o", "s"], config=DMLConfig(gpu=False))
    assert cs.cp.rewrite_stats.get("conv2d-bias-add") == 1
    res, _ = EX.execute(cs, ins)
    cs0 = EX.compile_script(src, {}, inputs=ins, outputs=["o", "s"], config=DMLConfig(gpu=False, rewrites=False))
    ref, _ = EX.execute(cs0, ins)
    assert torch.allclose(res["o"], ref["o"], rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_column_multi_aggregate_with_channel_operands_on_gpu(dt):
    """Batch-norm statistics and parameter gradients: column sums over the same activations
    with per-channel (bias_add / bias_multiply) operands fuse into ONE column MAgg kernel
    (cell_rtc.inc sysml_cell_magg_col4) and match fp64 torch."""
    from systemml_amd.ops import cell as CELL, kernels
    from systemml_amd.ops.backend import backend
    src = """
    Xs = bias_add(X, -em)
    s1 = colSums(Xs)
    s2 = colSums(Xs ^ 2)
    db = colSums(dout)
    dg = colSums(dout * bias_multiply(bias_add(X, -m), istd))
    """
    C, HW, N = 16, 49, 64
    rng = np.random.default_rng(3)
    ins = {"X": rng.standard_normal((N, C * HW)), "dout": rng.standard_normal((N, C * HW)),
           "em": rng.standard_normal((C, 1)), "m": rng.standard_normal((C, 1)), "istd": rng.random((C, 1)) + 0.5}
    cfg = DMLConfig(gpu=True, precision="single", gpu_min_cells=0)
    cs = EX.compile_script(src, {}, inputs=ins, outputs=["s1", "s2", "db", "dg"], config=cfg)
    text = EX.explain(cs.cp, "hops")
    assert text.count("magg(") >= 1, text
    backend.configure(cfg)
    dins = {k: torch.tensor(v, dtype=torch.float32).to("cuda").to(dt if k in ("X", "dout") else torch.float32)
            for k, v in ins.items()}
    b0 = CELL.stats.get("magg_kernel", 0)
    res, _ = EX.execute(cs, dins)
    assert CELL.stats.get("magg_kernel", 0) > b0
    X = dins["X"].double().cpu().numpy()
    D = dins["dout"].double().cpu().numpy()
    ch = np.repeat(np.arange(C), HW)
    Xs = X - ins["em"][ch, 0].astype(np.float32)
    ref = {"s1": Xs.sum(0), "s2": (Xs ** 2).sum(0), "db": D.sum(0),
           "dg": (D * (X - ins["m"][ch, 0].astype(np.float32)) * ins["istd"][ch, 0].astype(np.float32)).sum(0)}
    for k, r in ref.items():
        g = res[k].double().cpu().numpy().ravel()
        np.testing.assert_allclose(g, r, rtol=2e-4, atol=2e-3, err_msg=k)
