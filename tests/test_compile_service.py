"""Out-of-process compilation (api/compile_service.py): a plan compiled in the service
process from shape-only inputs, shipped without its closures and re-bound in the driver,
executes exactly like an in-process compilation; HOP ids are renumbered into the driver's
id space (dynamic recompilation in the driver must not collide with the worker's ids)."""
import numpy as np
import torch

from systemml_amd.api import compile_service as CSV
from systemml_amd.api import executor as EX
from systemml_amd.api.mlcontext import SCRIPTS_DIR
from systemml_amd.compiler import hops as H
from systemml_amd.conf import DMLConfig


def _data():
    rng = np.random.default_rng(0)
    X = torch.from_numpy(rng.random((1500, 12)) * 4 + 1)
    lab = torch.from_numpy(rng.integers(1, 6, (1500, 1)).astype(float))
    return X, lab


ARGS = dict(X="X", Y="Y", B="B", icpt=0, reg=0.01, tol=1e-4, moi=10, mii=5)


def test_dehydrate_hydrate_roundtrip():
    X, lab = _data()
    src = open(SCRIPTS_DIR + "/algorithms/MultiLogReg.dml").read()
    cfg = DMLConfig(gpu=False)
    meta = {"X": torch.empty(X.shape, device="meta"), "Y_vec": torch.empty(lab.shape, device="meta")}
    cs = EX.compile_script(src, ARGS, inputs=meta, outputs=["B_out"], config=cfg)
    blob = CSV.dehydrate(cs)
    before = next(H._ids)
    cs2 = CSV.hydrate(blob, {"X": X, "Y_vec": lab})
    ids = [ins.hop.id for lst in CSV._all_instr_lists(cs2.cp) for ins in lst]
    assert ids and min(ids) > before
    r2, _ = EX.execute(cs2, {"X": X, "Y_vec": lab}, out=lambda s: None)
    ref = EX.compile_script(src, ARGS, inputs={"X": X, "Y_vec": lab}, outputs=["B_out"], config=cfg)
    r1, _ = EX.execute(ref, {"X": X, "Y_vec": lab}, out=lambda s: None)
    np.testing.assert_array_equal(r2["B_out"].numpy(), r1["B_out"].numpy())


def test_service_process_compiles_in_order():
    X, lab = _data()
    src_m = open(SCRIPTS_DIR + "/algorithms/MultiLogReg.dml").read()
    src_l = open(SCRIPTS_DIR + "/algorithms/LinearRegCG.dml").read()
    y = X @ torch.linspace(-1, 1, X.shape[1], dtype=torch.float64).reshape(-1, 1)
    cfg = DMLConfig(gpu=False)
    svc = CSV.CompileService()
    try:
        p1 = svc.submit(src_l, dict(X="X", Y="y", B="B", icpt=0, reg=1e-6, tol=1e-12, maxi=50), {"X": X, "y": y},
                        ["beta"], cfg)
        p2 = svc.submit(src_m, ARGS, {"X": X, "Y_vec": lab}, ["B_out"], cfg)
        cs2, cs1 = p2.result(), p1.result()     # claimed out of order: each gets its own plan
    finally:
        svc.close()
    r1, _ = EX.execute(cs1, {"X": X, "y": y}, out=lambda s: None)
    np.testing.assert_allclose(r1["beta"].numpy(), np.linalg.lstsq(X.numpy(), y.numpy(), rcond=None)[0],
                               rtol=1e-6, atol=1e-8)
    r2, _ = EX.execute(cs2, {"X": X, "Y_vec": lab}, out=lambda s: None)
    assert np.isfinite(r2["B_out"].numpy()).all()
