"""Run-ahead while loops (runtime/program.py _exec_while_runahead).

CPU: which loops qualify (side-effect-free bodies only) and that the CPU backend never takes
the run-ahead path.  GPU: MultiLogReg and a vector-program loop give the same results with
and without run-ahead, every run-ahead loop ends by discarding exactly one speculative
iteration, the dead iteration's chain kernel returns at once (live flag), and an error
raised only by the dead iteration is not reported."""
import numpy as np
import pytest
import torch

from systemml_amd.api import executor as EX
from systemml_amd.api.mlcontext import SCRIPTS_DIR
from systemml_amd.compiler.blocks import WhileBlock
from systemml_amd.conf import DMLConfig
from systemml_amd.runtime import program as PR


def _loops(blocks, out=None):
    out = [] if out is None else out
    for b in blocks:
        if isinstance(b, WhileBlock):
            out.append(b)
            _loops(b.body, out)
        for attr in ("then_blocks", "else_blocks", "body"):
            if not isinstance(b, WhileBlock) and hasattr(b, attr) and isinstance(getattr(b, attr), list):
                _loops(getattr(b, attr), out)
    return out


def _qualifies(b):
    return (not getattr(b, "inplace_vars", None) and not b.pred.is_const and PR._pure_hops([b.pred.root])
            and PR._pure_blocks(b.body))


def test_pure_loops_qualify_and_side_effects_do_not():
    src = """
    A = A0
    s = 1
    while (s > 0.001) {
      A = A * 0.5
      s = sum(A ^ 2)
    }
    k = 0
    while (k < 3) {
      k = k + 1
      print("k " + k)
    }
    j = 0
    while (j < 2) {
      j = j + 1
      R = rand(rows=2, cols=2)
    }
    """
    cs = EX.compile_script(src, {}, inputs={"A0": np.ones((4, 4))}, outputs=["A"], config=DMLConfig())
    loops = _loops(cs.cp.blocks)
    assert len(loops) == 3
    # print(x) is buffered per iteration and printed once the iteration is live (the k loop,
    # SYSML_RUNAHEAD_PRINTS=1)
    assert [_qualifies(b) for b in loops] == [True, PR._RA_PRINTS, False]


def test_multilogreg_inner_cg_loop_qualifies():
    src = open(SCRIPTS_DIR + "/algorithms/MultiLogReg.dml").read()
    X = torch.rand(500, 16, dtype=torch.float64)
    y = torch.randint(1, 4, (500, 1)).double()
    cs = EX.compile_script(src, dict(X="X", Y="Y", B="B", icpt=0, reg=0.01, tol=1e-4, moi=3, mii=5),
                           inputs={"X": X, "Y_vec": y}, outputs=["B_out"], config=DMLConfig(precision="single"))
    loops = _loops(cs.cp.blocks)
    # outer Newton loop prints every iteration; the inner CG loop is pure
    assert [_qualifies(b) for b in loops] == [False, True]


def test_cpu_backend_never_runs_ahead():
    before = dict(PR.runahead_stats)
    src = "A = A0\ns = 1\nwhile (s > 0.01) {\n A = A * 0.5\n s = sum(A)\n}\nprint(s)"
    out = []
    EX.run(src, inputs={"A0": np.ones((3, 3))}, config=DMLConfig(gpu=False), out=out.append)
    assert PR.runahead_stats == before
    assert float(out[0]) < 0.01


# ----------------------------------------------------------------------------- GPU
def _mlr(X, y, icpt, runahead, monkeypatch):
    monkeypatch.setattr(PR, "RUNAHEAD", runahead)
    src = open(SCRIPTS_DIR + "/algorithms/MultiLogReg.dml").read()
    args = dict(X="X", Y="Y", B="B", icpt=icpt, reg=0.01, tol=1e-8, moi=6, mii=6)
    ins = {"X": X, "Y_vec": y}
    cs = EX.compile_script(src, args, inputs=ins, outputs=["B_out"], config=DMLConfig(gpu=True, precision="single"))
    out = []
    r, _ = EX.execute(cs, ins, out=out.append)
    return r["B_out"].double().cpu().numpy(), out


@pytest.mark.gpu
@pytest.mark.parametrize("icpt", [0, 2])
@pytest.mark.parametrize("depth", [1, 3])
def test_multilogreg_same_with_and_without_runahead(monkeypatch, icpt, depth):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setattr(PR, "RUNAHEAD_DEPTH", depth)
    g = torch.Generator().manual_seed(5)
    X = torch.rand(20000, 64, generator=g).to(torch.bfloat16).cuda()
    y = (torch.argmax(X[:, :4].float().cpu() + 0.3 * torch.rand(20000, 4, generator=g), 1) + 1).double()
    y = y.reshape(-1, 1).cuda().float()
    b0, out0 = _mlr(X, y, icpt, False, monkeypatch)
    st = dict(PR.runahead_stats)
    b1, out1 = _mlr(X, y, icpt, True, monkeypatch)
    loops = PR.runahead_stats["loops"] - st["loops"]
    dead = PR.runahead_stats["dead"] - st["dead"]
    assert loops >= 3, PR.runahead_stats
    # each loop is left by undoing the iterations queued past its end (1 .. depth of them)
    assert loops <= dead <= depth * loops, PR.runahead_stats
    if depth == 1:
        assert dead == loops, PR.runahead_stats
    # run-ahead iterations keep their small D x K bookkeeping in HBM (fp32 kernels) where the
    # op-by-op loop places it on the host: equal up to fp32 rounding through the solver
    np.testing.assert_allclose(b1, b0, rtol=1e-3, atol=1e-5)
    import re
    num = re.compile(r"[-+]?[0-9][0-9.eE+-]*")
    assert [num.sub("#", x) for x in out1] == [num.sub("#", x) for x in out0]   # same iterations / branches


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [1, 3])
def test_dead_iteration_errors_are_dropped(monkeypatch, depth):
    """The iteration queued past the end reads v[k + 1, 1] out of bounds; only a live
    iteration may raise."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setattr(PR, "RUNAHEAD_DEPTH", depth)
    src = """
    A = A0
    v = matrix(1, rows=3, cols=1)
    s = 100
    k = 0
    while (s > 0.5) {
      A = A * 0.1
      s = sum(A)
      k = k + 1
      x = as.scalar(v[k, 1])
    }
    print(k)
    """
    st = dict(PR.runahead_stats)
    out = []
    EX.run(src, inputs={"A0": np.full((200, 100), 0.005)}, config=DMLConfig(gpu=True, precision="double"),
           out=out.append)
    assert out == ["3"]
    assert PR.runahead_stats["loops"] - st["loops"] == 1, PR.runahead_stats


def test_runahead_depth_is_one_for_data_indexing_bodies():
    src = """
    s = 10
    y = Y0
    while (s > 1) {
      T = table(y, y, round(s) + 1, round(s) + 1)
      s = s / 2 + sum(T) / 1000
    }
    w = 10
    while (w > 1) {
      w = w / 2
    }
    """
    cs = EX.compile_script(src, {}, inputs={"Y0": np.ones((4, 1))}, outputs=[], config=DMLConfig())
    loops = _loops(cs.cp.blocks)
    assert [PR._runahead_depth(b) for b in loops] == [1, PR.RUNAHEAD_DEPTH]


# ----------------------------------------------------------------------------- graph replay (GPU)
def _graph_on(monkeypatch, on, depth=2):
    from systemml_amd.runtime import graphloop as GL
    monkeypatch.setattr(GL, "ENABLED", on)
    monkeypatch.setattr(GL, "DEPTH", depth)
    return GL


@pytest.mark.gpu
@pytest.mark.parametrize("icpt", [0, 2])
@pytest.mark.parametrize("gdepth", [1, 2])
def test_multilogreg_graph_replay_matches_op_by_op(monkeypatch, icpt, gdepth):
    """runtime/graphloop.py: the inner CG loop captured once and replayed for every later
    iteration and outer-loop entry gives the op-by-op run-ahead result."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = torch.Generator().manual_seed(7)
    X = torch.rand(20000, 64, generator=g).to(torch.bfloat16).cuda()
    y = (torch.argmax(X[:, :4].float().cpu() + 0.3 * torch.rand(20000, 4, generator=g), 1) + 1).double()
    y = y.reshape(-1, 1).cuda().float()
    _graph_on(monkeypatch, False)
    b0, out0 = _mlr(X, y, icpt, True, monkeypatch)
    GL = _graph_on(monkeypatch, True, gdepth)
    st = dict(GL.stats)
    b1, out1 = _mlr(X, y, icpt, True, monkeypatch)
    d = {k: GL.stats[k] - st[k] for k in st if k != "why"}
    if icpt == 0:
        # captured here or by an earlier compilation of the same script (the graph is reused)
        assert d["captures"] <= 1 and d["failed"] == 0 and d["replays"] > 0, d
        assert d["entries"] >= 3, d            # later outer iterations re-enter the captured loop
    np.testing.assert_allclose(b1, b0, rtol=1e-6, atol=1e-7)
    assert out1 == out0


@pytest.mark.gpu
@pytest.mark.parametrize("gdepth", [1, 3])
def test_graph_replay_counters_and_reentry(monkeypatch, gdepth):
    """Host counters become device state in the graph; every entry of the inner loop (new
    start matrix, reset counter) replays the one capture; dead replays change nothing."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    src = """
    for (j in 1:4) {
      A = A0 * j
      s = 100
      k = 0
      while (s > 0.5) {
        A = A * 0.9
        s = sum(A)
        k = k + 1
      }
      print(j + " " + k + " " + s)
    }
    """
    cfg = lambda: DMLConfig(gpu=True, precision="double")
    _graph_on(monkeypatch, False)
    ref = []
    EX.run(src, inputs={"A0": np.full((300, 200), 0.01)}, config=cfg(), out=ref.append)
    GL = _graph_on(monkeypatch, True, gdepth)
    st = dict(GL.stats)
    got = []
    EX.run(src, inputs={"A0": np.full((300, 200), 0.01)}, config=cfg(), out=got.append)
    d = {k: GL.stats[k] - st[k] for k in st if k != "why"}
    assert got == ref
    assert d["captures"] <= 1 and d["failed"] == 0 and d["entries"] == 4, d
    assert d["dead"] <= 4 * gdepth, d


@pytest.mark.gpu
def test_graph_capture_failure_falls_back(monkeypatch):
    """A body that needs the host (a device-scalar row index) cannot be captured: the loop
    continues op by op with the same result, and no capture is tried again."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    src = """
    A = A0
    v = seq(1, 50)
    s = 100
    k = 1
    while (s > 0.5) {
      A = A * 0.5
      s = sum(A) + as.scalar(v[k, 1]) * 0
      k = k + 1
    }
    print(k + " " + s)
    """
    _graph_on(monkeypatch, False)
    ref = []
    EX.run(src, inputs={"A0": np.full((200, 100), 0.01)}, config=DMLConfig(gpu=True, precision="double"),
           out=ref.append)
    GL = _graph_on(monkeypatch, True)
    st = dict(GL.stats)
    got = []
    EX.run(src, inputs={"A0": np.full((200, 100), 0.01)}, config=DMLConfig(gpu=True, precision="double"),
           out=got.append)
    assert got == ref
    assert GL.stats["captures"] == st["captures"]


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [1, 3])
def test_runahead_prints_only_live_iterations(monkeypatch, depth):
    """A loop that prints device scalars runs ahead: each iteration's lines are buffered
    (strings of unread device scalars stay deferred) and printed once the iteration is known
    to be live, in order; the speculative iterations past the end print nothing, and a
    string variable built in the loop leaves it resolved (LinearRegCG's per-iteration print
    and log appends)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from systemml_amd.runtime import scalars as S
    monkeypatch.setattr(PR, "RUNAHEAD_DEPTH", depth)
    monkeypatch.setattr(PR, "RA_PRINT_MIN_CELLS", 0)      # printing loops run ahead at any size
    monkeypatch.setattr(PR, "_RA_PRINTS", True)
    src = """
    A = A0
    s = 100
    log = "start"
    k = 0
    while (s > 0.5) {
      A = A * 0.5
      s = sum(A)
      k = k + 1
      print("it " + k + " s=" + s)
      log = append(log, "s " + s)
    }
    print("after " + k)
    print(log)
    """
    outs = {}
    for ra in (False, True):
        monkeypatch.setattr(PR, "RUNAHEAD", ra)
        st = dict(PR.runahead_stats)
        out = []
        r, _ = EX.execute(EX.compile_script(src, {}, inputs={"A0": np.full((200, 100), 0.01)}, outputs=["log"],
                                            config=DMLConfig(gpu=True, precision="double")),
                          {"A0": np.full((200, 100), 0.01)}, out=out.append)
        outs[ra] = out
        assert type(r["log"]) is str
        if ra:
            assert PR.runahead_stats["loops"] - st["loops"] == 1, PR.runahead_stats
    assert outs[True] == outs[False]
    assert outs[True][0].startswith("it 1 s=") and outs[True][-2] == "after 9"
    assert not any(type(x) is S.LazyStr for x in outs[True])
