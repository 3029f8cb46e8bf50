"""ResNet-50 training-step plan guards (bench_resnet50.py, BASELINE config #5): the nn layer
functions are specialised on their literal arguments and inlined into one DAG per step, the
Cell template recomputes cheap shared intermediates there, and on the MI355X the step runs
on the GEMM / col2im convolution paths with bf16 activations and no operator falling back to
the unfused sequential evaluation.  A rewrite or dispatch change that loses any of this fails
here instead of silently slowing the benchmark down."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _compile(image=32, batch=4, config=None):
    import bench_resnet50 as B
    from systemml_amd.api import executor as EX
    from systemml_amd.api.mlcontext import SCRIPTS_DIR
    from systemml_amd.conf import DMLConfig
    src = B.build_script(B.resnet50_layers(image=image), (3, image, image), 2, batch)
    X = np.random.default_rng(0).standard_normal((batch * 2, 3 * image * image)).astype(np.float32)
    Y = np.eye(1000, dtype=np.float32)[np.arange(batch * 2) % 1000]
    cfg = config or DMLConfig(precision="single", gpu_min_cells=0, act_bf16_min_cells=1 << 22)
    cs = EX.compile_script(src, {"X": "X", "Y": "Y"}, inputs={"X": X, "Y": Y}, config=cfg,
                           filename=os.path.join(SCRIPTS_DIR, "resnet50_plan_test.dml"))
    return cs, X, Y


def test_layers_inlined_and_shared_intermediates_recomputed():
    from systemml_amd.api import executor as EX
    cs, _, _ = _compile()
    rt = EX.explain(cs.cp, "runtime")
    main = rt[rt.find("MAIN PROGRAM"):]
    ops = [ln.strip().split(" ")[0] for ln in main.splitlines() if ln.startswith("      ")]
    assert ops.count("fcall") <= 2, "nn layer calls left in the training loop"          # benchSync only
    assert ops.count("conv2d") == 53 and ops.count("conv2d_backward_filter") == 53
    assert "bias_add" not in ops and "bias_multiply" not in ops           # all inside generated kernels
    assert cs.cp.rewrite_stats.get("cell-plan-inlined", 0) >= 50, cs.cp.rewrite_stats


@pytest.mark.gpu
def test_resnet_step_on_gemm_paths_with_bf16_activations():
    import torch
    from systemml_amd.api import executor as EX
    from systemml_amd.ops import cell, kernels
    from systemml_amd.conf import DMLConfig
    from systemml_amd.runtime.udf import register_udf
    register_udf("sysml.bench.Sync", lambda ctx, A: (0.0,))       # bench_resnet50's step clock
    cfg = DMLConfig(precision="single", gpu_min_cells=0, act_bf16_min_cells=1 << 16)
    cs, X, Y = _compile(image=64, batch=16, config=cfg)
    c0 = dict(kernels.counters)
    seq0 = cell.stats["sequential"]
    out = []
    EX.execute(cs, {"X": X, "Y": Y}, out=out.append)
    torch.cuda.synchronize()
    d = {k: kernels.counters.get(k, 0) - c0.get(k, 0) for k in kernels.counters}
    assert d.get("conv1x1_gemm", 0) > 0 and d.get("conv_col2im", 0) > 0, d
    assert cell.stats["sequential"] == seq0                 # every fused program on a generated kernel
    losses = [float(s.split(" loss ")[1].split(" ")[0]) for s in out if s.startswith("STEP")]
    assert len(losses) == 2 and all(np.isfinite(losses)), out
