"""Horizontal Cell batches (compiler/codegen.batch_cells, ops/cell.evaluate_batch): independent
same-program updates of small operands -- an optimizer's per-parameter steps -- are one hop and,
on the MI355X, one generated kernel launch over all operand sets."""
import numpy as np
import pytest
import torch

SRC = """
lr = 0.1
mu = 0.9
v1 = mu * v1 - lr * g1
v2 = mu * v2 - lr * g2
v3 = mu * v3 - lr * g3
W1 = W1 + v1
W2 = W2 + v2
W3 = W3 + v3
"""


def _inputs():
    rng = np.random.default_rng(4)
    shapes = [(300, 300), (700, 200), (100000, 1)]     # above the Vector template's 64K cells
    ins = {}
    for i, s in enumerate(shapes, 1):
        ins[f"W{i}"] = rng.standard_normal(s)
        ins[f"v{i}"] = rng.standard_normal(s)
        ins[f"g{i}"] = rng.standard_normal(s)
    return ins


def _expected(ins):
    out = {}
    for i in (1, 2, 3):
        v = 0.9 * ins[f"v{i}"] - 0.1 * ins[f"g{i}"]
        out[f"v{i}"] = v
        out[f"W{i}"] = ins[f"W{i}"] + v
    return out


def test_batched_updates_plan_and_results_cpu():
    from systemml_amd.api import executor as EX
    from systemml_amd.conf import DMLConfig
    ins = _inputs()
    outs = [f"{n}{i}" for n in ("W", "v") for i in (1, 2, 3)]
    cfg = DMLConfig(gpu=True, force_cpu=True)
    cs = EX.compile_script(SRC, {}, inputs=ins, outputs=outs, config=cfg)
    assert cs.cp.rewrite_stats.get("cell-batched", 0) == 6, cs.cp.rewrite_stats
    res, _ = EX.execute(cs, ins)
    exp = _expected(ins)
    for k in outs:
        r = res[k]
        r = r.cpu().numpy() if isinstance(r, torch.Tensor) else np.asarray(r)
        np.testing.assert_allclose(r, exp[k], rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
def test_batched_updates_one_launch_gpu():
    from systemml_amd.api import executor as EX
    from systemml_amd.conf import DMLConfig
    from systemml_amd.ops import kernels
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ins = {k: torch.tensor(v, device="cuda", dtype=torch.float32) for k, v in _inputs().items()}
    outs = [f"{n}{i}" for n in ("W", "v") for i in (1, 2, 3)]
    cfg = DMLConfig(gpu=True, precision="single", gpu_min_cells=0)
    cs = EX.compile_script(SRC, {}, inputs=ins, outputs=outs, config=cfg)
    c0 = kernels.counters.get("hcell", 0)
    res, _ = EX.execute(cs, ins)
    assert kernels.counters.get("hcell", 0) == c0 + 2          # the v updates, then the W updates
    exp = _expected({k: v.double().cpu().numpy() for k, v in ins.items()})
    for k in outs:
        np.testing.assert_allclose(res[k].double().cpu().numpy(), exp[k], rtol=1e-5, atol=1e-5)
