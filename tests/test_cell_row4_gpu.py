"""ops/hip/cell_rtc.inc sysml_cell_row4: generated row aggregates over 4-cell groups with vector
loads (bf16 / fp32 / fp64, full operands beside row vectors and scalars), against torch fp64."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32, torch.float64])
@pytest.mark.parametrize("cols", [64, 100, 1000, 4096])
@pytest.mark.parametrize("agg", ["sum", "sumsq", "max"])
def test_row_aggregate_vectorised(dt, cols, agg):
    from systemml_amd.conf import DMLConfig
    from systemml_amd.ops import cell as CELL
    from systemml_amd.ops.backend import backend
    backend.configure(DMLConfig(gpu=True, precision="double" if dt == torch.float64 else "single"))
    assert CELL.ROW4
    g = torch.Generator(device="cuda").manual_seed(cols)
    X = torch.randn(3001, cols, device="cuda", generator=g).to(dt)
    v = torch.randn(1, cols, device="cuda", generator=g, dtype=torch.float64).to(dt)
    # (x * 2 - v) ^ 2 then the row aggregate: a full operand, a row vector and a scalar
    prog = CELL.CellProgram([("b", "*", 3, 0, 2), ("b", "-", 4, 3, 1), ("u", "sq", 5, 4, 0)], 3, 5, (agg, "row"))
    before = CELL.stats["sequential"]
    r = CELL.evaluate(prog, [X, v, 2.0])
    assert CELL.stats["sequential"] == before
    E = (X.double() * 2 - v.double()) ** 2
    ref = {"sum": E.sum(1, keepdim=True), "sumsq": (E * E).sum(1, keepdim=True),
           "max": E.amax(1, keepdim=True)}[agg]
    tol = 2e-2 if dt == torch.bfloat16 else (1e-4 if dt == torch.float32 else 1e-10)
    torch.testing.assert_close(r.double(), ref, rtol=tol, atol=tol * float(ref.abs().max()))
