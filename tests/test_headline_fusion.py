"""Fusion regression guard for the headline benchmark (bench.py: LinregCG + MultiLogReg on a
bf16 X in HBM).  The step must keep its fused plan -- a rewrite-order change that silently
drops back to unfused passes fails here:
  * compile time: MultiLogReg's accept-branch gradient is speculated into the candidate
    pass (compiler/speculate.py), the softmax objective template forms, the CG branch is
    if-converted and the loop tails become vector programs;
  * run time on the MI355X: one chain4m Hessian-vector pass per CG iteration, one smobj pass
    per outer iteration, vector programs for the solver tails, and no unfused X pass."""
import os

import numpy as np
import pytest
import torch

from systemml_amd.api import executor as EX
from systemml_amd.api.mlcontext import SCRIPTS_DIR
from systemml_amd.conf import DMLConfig

ROWS, COLS = 200_000, 1000
MLR_ARGS = dict(X="X", Y="Y", B="B", icpt=0, reg=0.01, tol=0.0001, moi=5, mii=5)
LR_ARGS = dict(X="X", Y="y", B="B", icpt=0, maxi=20, tol=0.0001, reg=0.01, fmt="csv")


def _src(name):
    with open(os.path.join(SCRIPTS_DIR, "algorithms", name)) as f:
        return f.read()


def test_headline_plan_shape_cpu_compile():
    X = torch.empty((ROWS, COLS), device="meta")
    Y = torch.empty((ROWS, 1), device="meta")
    cs = EX.compile_script(_src("MultiLogReg.dml"), MLR_ARGS, inputs={"X": X, "Y_vec": Y}, outputs=["B_out"],
                           config=DMLConfig(precision="single"))
    assert cs.cp.licm_stats.get("speculative-fused-products") == 1, cs.cp.licm_stats
    assert cs.cp.licm_stats.get("if-converted", 0) >= 1, cs.cp.licm_stats
    st = cs.cp.rewrite_stats
    assert st.get("softmax-objective", 0) >= 1 and st.get("mmchain-row", 0) >= 1, st
    assert st.get("vector-fused-ops", 0) >= 20, st
    cs = EX.compile_script(_src("LinearRegCG.dml"), LR_ARGS, inputs={"X": X, "y": Y}, outputs=["B_out"],
                           config=DMLConfig(precision="single"))
    assert cs.cp.rewrite_stats.get("vector-fused-ops", 0) >= 10, cs.cp.rewrite_stats


@pytest.mark.gpu
def test_headline_step_kernel_counts():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import bench
    from systemml_amd.ops import kernels
    from systemml_amd.ops.backend import backend
    cfg = DMLConfig(precision="single", dist_min_rows=100_000)
    backend.configure(cfg)
    X1, y1, X2, lab = bench.gen_data(None, ROWS, COLS, 5, torch.bfloat16)
    from systemml_amd.runtime import program as PR
    before = dict(kernels.counters)
    dead0 = PR.runahead_stats["dead"]
    out = []
    cs = EX.compile_script(_src("LinearRegCG.dml"), LR_ARGS, inputs={"X": X1, "y": y1}, outputs=["B_out"], config=cfg)
    EX.execute(cs, {"X": X1, "y": y1}, out=out.append)
    dead0 = PR.runahead_stats["dead"]        # LinearRegCG's loop runs ahead too (its prints buffered)
    cs = EX.compile_script(_src("MultiLogReg.dml"), MLR_ARGS, inputs={"X": X2, "Y_vec": lab}, outputs=["B_out"],
                           config=cfg)
    r, _ = EX.execute(cs, {"X": X2, "Y_vec": lab}, out=out.append)
    d = {k: v - before.get(k, 0) for k, v in kernels.counters.items() if v > before.get(k, 0)}
    outer = sum(1 for s in out if s.startswith("-- Outer Iteration"))
    cg = sum(int(s.split("Had ")[1].split(" CG")[0]) for s in out if s.startswith("-- Outer Iteration"))
    assert outer >= 2, out
    assert d.get("chain4m.smobj", 0) == outer, d                   # one fused candidate pass per outer iteration
    # one Hessian-vector pass per CG iteration, plus the launch of the run-ahead iteration queued
    # past each CG loop's end (its kernel reads the dead predicate and returns at once)
    dead = PR.runahead_stats["dead"] - dead0
    assert d.get("chain4.mmchain.XtPSXv", 0) == cg + dead, (d, cg, dead)
    assert d.get("vprog", 0) >= cg, d                              # solver tails as vector programs
    assert not any(k.startswith("mfma.xtg") for k in d if d[k] > 2), d   # no separate gradient pass
    assert np.isfinite(r["B_out"].float().cpu().numpy()).all()
