"""Intercept scripts on the GPU backend (icpt = 1 | 2: `X = cbind(X, ones)`): the constant-
column view (ops/augmented.ConstCol) gets a padded HBM copy with 16-B rows, and the fused
chain / softmax kernels run one pass over it per product.  Results against the CPU backend
on the same script; the threshold that keeps small views on the two-pass path is lowered so
the test matrices take the padded path."""
import numpy as np
import pytest
import torch

from systemml_amd.api import executor as EX
from systemml_amd.api.mlcontext import SCRIPTS_DIR
from systemml_amd.conf import DMLConfig

pytestmark = pytest.mark.gpu


def _data(n=4000, d=30, k=3, seed=11):
    g = torch.Generator().manual_seed(seed)
    X = torch.rand(n, d, dtype=torch.float64, generator=g)
    y = (torch.argmax(X[:, :k] + 0.3 * torch.rand(n, k, generator=g, dtype=torch.float64), 1) + 1)
    return X, y.double().reshape(-1, 1)


@pytest.mark.parametrize("icpt", [1, 2])
def test_multilogreg_intercept_on_padded_copy(icpt, monkeypatch):
    from systemml_amd.ops import augmented as AUG
    monkeypatch.setattr(AUG, "PAD_MIN_CELLS", 0)
    monkeypatch.setattr(AUG, "VIEW_MIN_CELLS", 0)
    X, y = _data()
    args = dict(X="X", Y="Y", B="B", icpt=icpt, reg=0.01, tol=1e-8, moi=8, mii=6)
    src = open(SCRIPTS_DIR + "/algorithms/MultiLogReg.dml").read()
    res = {}
    before = AUG.stats["padded"]
    for gpu in (True, False):
        cfg = DMLConfig(gpu=gpu, precision="single" if gpu else "double", gpu_min_cells=0)
        ins = {"X": X, "Y_vec": y}
        cs = EX.compile_script(src, args, inputs=ins, outputs=["B_out"], config=cfg)
        r, _ = EX.execute(cs, ins, out=lambda s: None)
        res[gpu] = r["B_out"].double().cpu().numpy()
    assert AUG.stats["padded"] > before
    np.testing.assert_allclose(res[True], res[False], rtol=2e-3, atol=1e-2)   # fp32 vs fp64 solves


def test_linreg_cg_intercept_on_padded_copy(monkeypatch):
    from systemml_amd.ops import augmented as AUG
    monkeypatch.setattr(AUG, "PAD_MIN_CELLS", 0)
    monkeypatch.setattr(AUG, "VIEW_MIN_CELLS", 0)
    g = torch.Generator().manual_seed(5)
    X = torch.rand(3000, 24, dtype=torch.float64, generator=g)
    y = X @ torch.rand(24, 1, dtype=torch.float64, generator=g) + 0.5
    src = open(SCRIPTS_DIR + "/algorithms/LinearRegCG.dml").read()
    args = dict(X="X", Y="y", B="B", icpt=1, reg=1e-6, tol=1e-10, maxi=40)
    res = {}
    before = AUG.stats["padded"]
    for gpu in (True, False):
        cfg = DMLConfig(gpu=gpu, precision="single" if gpu else "double", gpu_min_cells=0)
        ins = {"X": X, "y": y}
        cs = EX.compile_script(src, args, inputs=ins, outputs=["B_out"], config=cfg)
        r, _ = EX.execute(cs, ins, out=lambda s: None)
        res[gpu] = r["B_out"].double().cpu().numpy()
    assert AUG.stats["padded"] > before
    np.testing.assert_allclose(res[True], res[False], rtol=2e-3, atol=1e-2)   # fp32 vs fp64 solves


@pytest.mark.parametrize("agg", [None, ("sum", "col"), ("sum", "row"), ("sum", "all"), ("max", "col"),
                                 ("min", "row")])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_cell_program_over_const_column_operand(agg, dt):
    """ops/cell._split_cc: a Cell program (here (x - 0.5)^2 * 3, or (x - 0.5)^2 * t(v) with a row
    vector over all D + 1 columns) over cbind(X, c) runs its kernel over X and appends the
    constant column's value, against torch on the materialised matrix."""
    from systemml_amd.ops import augmented as AUG
    from systemml_amd.ops import cell as CELL
    from systemml_amd.ops.backend import backend
    backend.configure(DMLConfig(gpu=True, precision="single"))
    g = torch.Generator(device="cuda").manual_seed(3)
    X = torch.rand(4096, 64, device="cuda", generator=g).to(dt)
    cc = AUG.ConstCol(X, 1.0)
    prog = CELL.CellProgram([("b", "-", 3, 0, 1), ("u", "sq", 4, 3, 0), ("b", "*", 5, 4, 2)], 3, 5, agg)
    before = CELL.stats["sequential"]
    r = CELL.evaluate(prog, [cc, 0.5, 3.0])
    assert CELL.stats["sequential"] == before           # no operator-by-operator fallback
    M = torch.cat([X.double(), torch.ones(4096, 1, dtype=torch.float64, device="cuda")], 1)
    E = (M - 0.5) ** 2 * 3.0
    if agg is None:
        assert AUG.is_cc(r)
        got = r.materialize().double()
        ref = E
    else:
        o, d = agg
        f = {"sum": torch.sum, "max": torch.amax, "min": torch.amin}[o]
        ref = f(E) if d == "all" else f(E, dim=0 if d == "col" else 1, keepdim=True)
        got = r.double() if isinstance(r, torch.Tensor) else torch.tensor(float(r), dtype=torch.float64)
        got = got.to(ref.device)
    tol = 2e-2 if dt == torch.bfloat16 else 1e-4
    torch.testing.assert_close(got.reshape(ref.shape), ref, rtol=tol, atol=tol * max(1.0, float(ref.abs().max())))
