"""Vector template (compiler/vecgen.py, ops/vprog.py) and if-conversion (compiler/ifconv.py).

CPU: plan shape (one vector program per solver-loop tail), parity of the run-time fallback
(the region's original operators) with the unfused plan, and parity of if-converted loops
(forced guard) with the original control flow.  GPU: the generated single-workgroup kernel
against an fp64 CPU evaluation of the same script for every operator class (cellwise,
select, sum / sumsq / min / max / mean / dot / dot3 aggregates, scalar algebra, int and
boolean scalar results), above the cell limit (fallback), and the solver scripts end to end
with their loop tails as vector programs."""
import numpy as np
import pytest
import torch

from systemml_amd.api import executor as EX
from systemml_amd.api.mlcontext import SCRIPTS_DIR
from systemml_amd.conf import DMLConfig

SCRIPT = """
A = A0 - 0.5
B = B0 + 0.1
k = 3
while (k > 0) {
  s = sum(A * B)
  t = sum(A ^ 2)
  m1 = max(A)
  m2 = min(B)
  mu = mean(B)
  C = A * s + B / t - min(A, B) * mu
  C2 = ifelse(s > 0, C, -C)
  d = sum(C2 * A * B)
  e = sqrt(abs(d)) + exp(-abs(m1)) + log(m2 + 1)
  D = C2 * e + (A > B) - (A <= 0.2) * m1
  f = sum(D)
  flag = (f > 0) | (e < 1)
  cnt = ifelse(flag, k, 0)
  A = D / (1 + abs(f))
  k = k - 1
}
"""
OUTS = ["C2", "D", "f", "flag", "e", "cnt", "A"]


def _inputs(r, c):
    rng = np.random.default_rng(r * 1000 + c)
    return {"A0": rng.uniform(0, 1, (r, c)), "B0": rng.uniform(0, 1, (r, c))}


def _run(cfg, r, c):
    ins = _inputs(r, c)
    cs = EX.compile_script(SCRIPT, {}, inputs=ins, outputs=OUTS, config=cfg)
    res, _ = EX.execute(cs, ins)
    return cs, {k: (v.double().cpu().numpy() if isinstance(v, torch.Tensor) else v) for k, v in res.items()}


def _check(a, b, tol):
    for k in OUTS:
        x, y = a[k], b[k]
        if isinstance(y, np.ndarray):
            np.testing.assert_allclose(x, y, rtol=tol, atol=tol, err_msg=k)
        else:
            assert type(x) is type(y), (k, x, y)
            assert x == pytest.approx(y, rel=tol, abs=tol), k


def test_plan_one_program_per_loop_tail():
    cs = EX.compile_script(SCRIPT, {}, inputs=_inputs(20, 5), outputs=OUTS, config=DMLConfig())
    assert cs.cp.rewrite_stats.get("vector-fused-ops", 0) >= 20, cs.cp.rewrite_stats
    text = EX.explain(cs.cp, "hops")
    assert sum("vprog[" in ln for ln in text.splitlines()) >= 1, text


def test_fallback_matches_unfused_cpu():
    _, a = _run(DMLConfig(), 20, 5)           # GPU plan (vector programs), run on the CPU fallback
    _, b = _run(DMLConfig(gpu=False, fusion=False), 20, 5)
    _check(a, b, 1e-12)


def test_linregcg_loop_tail_is_one_program():
    src = open(SCRIPTS_DIR + "/algorithms/LinearRegCG.dml").read()
    X = torch.rand(300, 12, dtype=torch.float64)
    y = X @ torch.linspace(-1, 1, 12, dtype=torch.float64).reshape(-1, 1)
    cs = EX.compile_script(src, dict(X="X", Y="y", B="B", icpt=0, reg=1e-6, tol=1e-12, maxi=40),
                           inputs={"X": X, "y": y}, outputs=["beta"], config=DMLConfig())
    from systemml_amd.compiler.blocks import WhileBlock
    loops = [b for b in cs.cp.blocks if isinstance(b, WhileBlock)]
    assert loops and len(loops[0].body) == 1
    ops = [i.opcode for i in loops[0].body[0].instrs]
    assert ops.count("spoofVec") == 1, ops
    r, _ = EX.execute(cs, {"X": X, "y": y}, out=lambda s: None)
    np.testing.assert_allclose(r["beta"].numpy(), np.linalg.lstsq(X.numpy(), y.numpy(), rcond=None)[0],
                               rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("icpt", [0, 2])
def test_if_conversion_forced_matches_control_flow(monkeypatch, icpt):
    """The CG step's trust-region branch becomes straight-line code with selects; with the
    guard forced on (SYSML_IFCONV=force) the CPU runs the converted blocks."""
    from systemml_amd.compiler import ifconv
    src = open(SCRIPTS_DIR + "/algorithms/MultiLogReg.dml").read()
    g = torch.Generator().manual_seed(3)
    X = torch.rand(800, 15, dtype=torch.float64, generator=g)
    y = (torch.argmax(X[:, :3] + 0.3 * torch.rand(800, 3, generator=g, dtype=torch.float64), 1) + 1)
    y = y.double().reshape(-1, 1)
    args = dict(X="X", Y="Y", B="B", icpt=icpt, reg=0.01, tol=1e-8, moi=6, mii=6)
    ins = {"X": X, "Y_vec": y}
    monkeypatch.setattr(ifconv, "MODE", "force")
    cs = EX.compile_script(src, args, inputs=ins, outputs=["B_out"], config=DMLConfig())
    assert cs.cp.licm_stats.get("if-converted", 0) >= 1, cs.cp.licm_stats
    out1 = []
    r1, _ = EX.execute(cs, ins, out=out1.append)
    monkeypatch.setattr(ifconv, "MODE", "0")
    cs0 = EX.compile_script(src, args, inputs=ins, outputs=["B_out"], config=DMLConfig(fusion=False))
    out0 = []
    r0, _ = EX.execute(cs0, ins, out=out0.append)
    np.testing.assert_allclose(r1["B_out"].numpy(), r0["B_out"].numpy(), rtol=1e-9, atol=1e-11)
    assert [ln.split("=")[0] for ln in out1] == [ln.split("=")[0] for ln in out0]


def test_if_conversion_keeps_undefined_variables_undefined(monkeypatch):
    from systemml_amd.compiler import ifconv
    monkeypatch.setattr(ifconv, "MODE", "force")
    src = """
    x = 1
    i = 0
    while (i < 2) {
      i = i + 1
      if (x > 5) { Z = matrix(1, 2, 2) }
      x = x + 1
    }
    print(exists(Z))
    """
    out = []
    EX.run(src, config=DMLConfig(), out=out.append)
    assert out == ["FALSE"]


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("rc", [(7, 3), (1000, 5), (200, 300), (300, 300)])
def test_vprog_kernel_matches_cpu(rc):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from systemml_amd.ops import kernels, vprog
    r, c = rc
    before = kernels.counters.get("vprog", 0)
    fb = vprog.stats["fallback"]
    cs, a = _run(DMLConfig(gpu=True, precision="double"), r, c)
    _, b = _run(DMLConfig(gpu=False, fusion=False), r, c)
    _check(a, b, 1e-9)
    if r * c <= vprog.VMAX:
        assert kernels.counters.get("vprog", 0) > before, kernels.counters
    else:
        # matrices above the single-workgroup limit: known at compile time here, so the Cell /
        # MAgg templates take the region (no vector program); a region sized only at run time
        # would take the guarded fallback instead
        assert kernels.counters.get("vprog", 0) == before or vprog.stats["fallback"] > fb


@pytest.mark.gpu
def test_vprog_kernel_single_precision():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _, a = _run(DMLConfig(gpu=True, precision="single"), 100, 10)
    _, b = _run(DMLConfig(gpu=False, fusion=False), 100, 10)
    for k in ("C2", "D", "A"):
        np.testing.assert_allclose(a[k], b[k], rtol=2e-4, atol=2e-4, err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("icpt", [0, 1, 2])
def test_solvers_with_vector_programs_on_gpu(icpt):
    """LinregCG and MultiLogReg on the GPU backend: loop tails as vector programs, the CG
    trust-region branch if-converted (guard true for D x K state), same answers as the CPU."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from systemml_amd.ops import kernels
    g = torch.Generator().manual_seed(11)
    X = torch.rand(4000, 30, dtype=torch.float64, generator=g)
    y = (torch.argmax(X[:, :3] + 0.3 * torch.rand(4000, 3, generator=g, dtype=torch.float64), 1) + 1)
    y = y.double().reshape(-1, 1)
    args = dict(X="X", Y="Y", B="B", icpt=icpt, reg=0.01, tol=1e-8, moi=8, mii=6)
    src = open(SCRIPTS_DIR + "/algorithms/MultiLogReg.dml").read()
    res = {}
    for gpu in (True, False):
        cfg = DMLConfig(gpu=gpu, precision="double")
        ins = {"X": X, "Y_vec": y}
        before = kernels.counters.get("vprog", 0)
        cs = EX.compile_script(src, args, inputs=ins, outputs=["B_out"], config=cfg)
        r, _ = EX.execute(cs, ins, out=lambda s: None)
        res[gpu] = r["B_out"].double().cpu().numpy()
        if gpu:
            assert kernels.counters.get("vprog", 0) - before >= 8, kernels.counters
            assert cs.cp.licm_stats.get("if-converted", 0) >= 1
    np.testing.assert_allclose(res[True], res[False], rtol=1e-6, atol=1e-8)


def test_if_conversion_branch_not_taken_may_fail(monkeypatch):
    """A branch valid only under its predicate (a shape mismatch otherwise): the converted
    block fails, the original control flow runs and takes the other branch."""
    from systemml_amd.compiler import ifconv
    monkeypatch.setattr(ifconv, "MODE", "force")
    src = """
    A = A0
    B = matrix(2, rows=as.integer(sum(A)) - 2, cols=2)
    i = 0
    C = A
    while (i < 2) {
      i = i + 1
      if (nrow(A) == nrow(B)) { C = A + B } else { C = A * 2 }
    }
    print(sum(C))
    """
    cs = EX.compile_script(src, {}, inputs={"A0": np.ones((3, 2))}, outputs=[], config=DMLConfig())
    assert cs.cp.licm_stats.get("if-converted", 0) >= 1, cs.cp.licm_stats
    out = []
    EX.execute(cs, {"A0": np.ones((3, 2))}, out=out.append)
    assert out == ["12.0"]
