"""Host (CP) fast paths of the solver-state operators: fused y +/- s * x cell programs as one
torch.add(alpha=), and the dense-host shortcuts of sum / sumsq / row- and column-sums / sum(a*b)
(ops/cell.py sequential, ops/core.py agg / tak).  They must agree with the general operator
paths (to the last ulp for the aggregates, within one rounding for the fused multiply-add)."""
import numpy as np
import pytest
import torch

from systemml_amd.api import executor as EX
from systemml_amd.conf import DMLConfig
from systemml_amd.ops import cell, core as C
from systemml_amd.ops.cell import CellProgram


@pytest.mark.parametrize("prog,args,ref", [
    (CellProgram([("b", "*", 2, 0, 1), ("b", "+", 2, 3, 2)], 4, 2), "s V 0 S", lambda V, S, a: S + a * V),
    (CellProgram([("b", "*", 0, 0, 1), ("b", "-", 0, 2, 0)], 3, 0), "V s S", lambda V, S, a: S - V * a),
    (CellProgram([("b", "*", 0, 0, 1), ("b", "+", 0, 0, 2)], 3, 0), "V s S", lambda V, S, a: V * a + S),
])
def test_axpy_programs(prog, args, ref):
    g = torch.Generator().manual_seed(3)
    V = torch.rand((40, 7), generator=g, dtype=torch.float64)
    S = torch.rand((40, 7), generator=g, dtype=torch.float64)
    a = 0.371
    m = {"s": a, "V": V, "S": S, "0": 0}
    got = cell.sequential(prog, [m[t] for t in args.split()])
    assert cell._axpy_form(prog) is not None
    torch.testing.assert_close(got, ref(V, S, a), rtol=0, atol=4e-16)


def test_axpy_form_rejects_other_shapes():
    # (x - s) * y is not an axpy
    assert cell._axpy_form(CellProgram([("b", "-", 2, 0, 1), ("b", "*", 2, 2, 3)], 4, 2)) is None
    # a broadcast row vector falls back to the operator-by-operator path
    prog = CellProgram([("b", "*", 2, 0, 1), ("b", "+", 2, 3, 2)], 4, 2)
    V = torch.rand((5, 3), dtype=torch.float64)
    r = torch.rand((1, 3), dtype=torch.float64)
    torch.testing.assert_close(cell.sequential(prog, [0.5, V, 0, r]), r + 0.5 * V)


def test_host_aggregate_fast_paths_match_general_paths():
    g = torch.Generator().manual_seed(5)
    x = torch.rand((33, 6), generator=g, dtype=torch.float64)
    y = torch.rand((33, 6), generator=g, dtype=torch.float64)
    assert C.agg("sum", "all", x) == float(torch.sum(x))
    assert C.agg("sumsq", "all", x) == float(torch.sum(x * x))
    assert torch.equal(C.agg("sum", "row", x), torch.sum(x, dim=1, keepdim=True))
    assert torch.equal(C.agg("sum", "col", x), torch.sum(x, dim=0, keepdim=True))
    assert C.tak(x, y) == float(torch.dot(x.reshape(-1), y.reshape(-1)))
    # empty matrices keep the general path's semantics
    assert C.agg("sum", "all", torch.zeros((0, 3), dtype=torch.float64)) == 0.0


def test_cg_solver_on_host_paths():
    """A CG solve whose state updates take the fused host paths converges to lstsq."""
    rng = np.random.default_rng(0)
    X = rng.standard_normal((200, 12))
    y = X @ rng.standard_normal((12, 1))
    src = open(__import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(
        __import__("os").path.abspath(__file__))), "systemml_amd", "scripts", "algorithms", "LinearRegCG.dml")).read()
    cs = EX.compile_script(src, dict(X="X", Y="y", B="B", maxi=50, tol=1e-12, reg=1e-12, fmt="csv"),
                           inputs={"X": X, "y": y}, outputs=["B_out"], config=DMLConfig(gpu=False))
    res, _ = EX.execute(cs, {"X": X, "y": y}, out=lambda s: None)
    np.testing.assert_allclose(res["B_out"].numpy(), np.linalg.lstsq(X, y, rcond=None)[0], rtol=1e-6, atol=1e-8)
