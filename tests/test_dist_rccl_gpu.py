"""RCCL code paths of parallel/dist.py on one GPU (a one-rank process group): the device-scalar
all-reduce of full aggregates (DistContext.allreduce_dev -> DevScalar, no host round trip) and
the packed all-reduce of the fused softmax objective (gradient + both objective sums in one
collective).  Multi-rank RCCL runs are the driver's (8-GPU node); these pin the device-side
code that only an RCCL backend reaches."""
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def ctx():
    import torch.distributed as tdist
    from systemml_amd.parallel import dist as D
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    tdist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                             device_id=torch.device("cuda", 0))
    try:
        yield D.DistContext(0, 1, torch.device("cuda", 0))
    finally:
        tdist.destroy_process_group()


def test_full_aggregate_is_a_device_scalar(ctx):
    from systemml_amd.parallel import dist as D
    from systemml_amd.runtime.scalars import DevScalar
    X = torch.rand(1000, 37, dtype=torch.float64, device="cuda")
    dm = D.DistMatrix(X, 1000, 37, 0, ctx)
    for o, ref in (("sum", X.sum()), ("max", X.max()), ("sumsq", (X * X).sum())):
        r = D.agg(o, "all", dm)
        assert isinstance(r, DevScalar), type(r)
        assert r.value() == pytest.approx(float(ref), rel=1e-12)


def test_softmax_objective_one_packed_allreduce(ctx):
    from systemml_amd.ops import core as C, kernels
    from systemml_amd.parallel import dist as D
    kernels.load(required=True)
    n, d, k = 4096, 256, 4
    g = torch.Generator().manual_seed(3)
    X = (torch.rand(n, d, generator=g) * 0.1).to("cuda", torch.bfloat16)
    V = (torch.rand(d, k, generator=g) - 0.5).to("cuda")
    Y = torch.zeros(n, k + 1)
    Y[torch.arange(n), torch.randint(0, k + 1, (n,), generator=g)] = 1.0
    Y = Y.to("cuda")
    p0, g0, s10, s20 = C.smobj(X, V, Y, k)
    before = D.stats["allreduce"]
    p1, g1, s11, s21 = D.smobj(D.DistMatrix(X, n, d, 0, ctx), V, Y, k)
    assert D.stats["allreduce"] == before + 1
    torch.testing.assert_close(g1.double().cpu(), g0.double().cpu(), rtol=1e-6, atol=1e-6)
    assert s11 == pytest.approx(float(s10), rel=1e-6) and s21 == pytest.approx(float(s20), rel=1e-6)
    np.testing.assert_allclose(p1.local.double().cpu().numpy(), p0.double().cpu().numpy(), rtol=1e-6)


def test_headline_scripts_spmd_rccl_with_runahead(ctx, monkeypatch):
    """The headline's DIST plan end to end on a one-rank RCCL group: LinregCG + MultiLogReg on a
    row-partitioned bf16 X (as bench.py with SYSML_DIST_FORCE=1 / every rank of an N-GPU run)
    give the single-process results, with run-ahead CG loops under the NCCL context, device-
    scalar all-reduces and no fallback gather of a row-partitioned operand."""
    import os
    from systemml_amd.api import executor as EX
    from systemml_amd.api.mlcontext import SCRIPTS_DIR
    from systemml_amd.compiler import cost
    from systemml_amd.conf import DMLConfig
    from systemml_amd.parallel import dist as D
    from systemml_amd.runtime import program as PR
    from systemml_amd.runtime.scalars import DevScalar
    g = torch.Generator(device="cuda").manual_seed(11)
    n, d = 60000, 128
    X = (torch.rand(n, d, generator=g, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = torch.rand(d, 1, generator=g, device="cuda") - 0.5
    y = X.float() @ w + 0.01 * torch.randn(n, 1, generator=g, device="cuda")
    lab = (torch.argmax(X[:, :4].float() + 0.2 * torch.rand(n, 4, generator=g, device="cuda"), 1) + 1)
    lab = lab.float().reshape(-1, 1)
    srcs = {k: open(os.path.join(SCRIPTS_DIR, "algorithms", f)).read()
            for k, f in (("lr", "LinearRegCG.dml"), ("mlr", "MultiLogReg.dml"))}
    args = {"lr": dict(X="X", Y="y", B="B", icpt=0, maxi=20, tol=1e-9, reg=0.01, fmt="csv"),
            "mlr": dict(X="X", Y="Y", B="B", icpt=0, reg=0.01, tol=1e-9, moi=4, mii=5)}

    def run(spmd):
        out = {}
        for k in ("lr", "mlr"):
            ins = {"X": X, "y": y} if k == "lr" else {"X": X, "Y_vec": lab}
            if spmd:
                ins = {a: D.from_local(ctx, t, n) for a, t in ins.items()}
            cfg = DMLConfig(precision="single", dist_min_rows=10000)
            cs = EX.compile_script(srcs[k], args[k], inputs=ins, outputs=["B_out"], config=cfg)
            r, _ = EX.execute(cs, ins, out=lambda s: None, dist=ctx if spmd else None)
            b = r["B_out"]
            out[k] = (D.gather(b) if D._is_d(b) else b).double().cpu().numpy()
        return out

    ref = run(False)
    monkeypatch.setattr(cost, "_FORCE_DIST", True)
    monkeypatch.setattr(D, "_CTX", ctx)
    D.reset_stats()
    st = dict(PR.runahead_stats)
    calls = []
    orig = D.DistContext.allreduce_dev

    def spy(self, v, op="sum"):
        r = orig(self, v, op)
        calls.append(type(r))
        return r
    monkeypatch.setattr(D.DistContext, "allreduce_dev", spy)
    got = run(True)
    for k in ("lr", "mlr"):
        np.testing.assert_allclose(got[k], ref[k], rtol=2e-3, atol=2e-4, err_msg=k)
    assert D.stats["fallback_gathers"] == 0, D.fallback_sites
    assert D.stats["allreduce"] > 0
    assert calls and all(c is DevScalar for c in calls), calls[:5]
    assert PR.runahead_stats["loops"] > st["loops"], PR.runahead_stats
    assert PR.runahead_stats["dead"] > st["dead"], PR.runahead_stats


def test_headline_mlr_spmd_graph_replay_with_collectives(ctx, monkeypatch):
    """runtime/graphloop.py under the one-rank RCCL group: the inner CG iteration is captured
    in segments cut at its all-reduce, replayed with the all-reduce issued between them, and
    gives the op-by-op SPMD result; the collectives per replayed iteration are the op-by-op
    ones (same count with and without graphs, plus the ranks' one agreement on the capture)."""
    import os
    from systemml_amd.api import executor as EX
    from systemml_amd.api.mlcontext import SCRIPTS_DIR
    from systemml_amd.compiler import cost
    from systemml_amd.conf import DMLConfig
    from systemml_amd.parallel import dist as D
    from systemml_amd.runtime import graphloop as GL
    g = torch.Generator(device="cuda").manual_seed(13)
    n, d = 60000, 128
    X = (torch.rand(n, d, generator=g, device="cuda") * 2 - 1).to(torch.bfloat16)
    lab = (torch.argmax(X[:, :4].float() + 0.2 * torch.rand(n, 4, generator=g, device="cuda"), 1) + 1)
    lab = lab.float().reshape(-1, 1)
    src = open(os.path.join(SCRIPTS_DIR, "algorithms", "MultiLogReg.dml")).read()
    args = dict(X="X", Y="Y", B="B", icpt=0, reg=0.01, tol=1e-9, moi=4, mii=5)
    monkeypatch.setattr(cost, "_FORCE_DIST", True)
    monkeypatch.setattr(D, "_CTX", ctx)

    def run():
        ins = {a: D.from_local(ctx, t, n) for a, t in {"X": X, "Y_vec": lab}.items()}
        cs = EX.compile_script(src, args, inputs=ins, outputs=["B_out"],
                               config=DMLConfig(precision="single", dist_min_rows=10000))
        D.reset_stats()
        r, _ = EX.execute(cs, ins, out=lambda s: None, dist=ctx)
        b = r["B_out"]
        return (D.gather(b) if D._is_d(b) else b).double().cpu().numpy(), D.stats["allreduce"]

    monkeypatch.setattr(GL, "ENABLED", False)
    ref, n_ref = run()
    monkeypatch.setattr(GL, "ENABLED", True)
    monkeypatch.setattr(GL, "DIST", True)
    st = dict(GL.stats)
    got, n_got = run()
    dd = {k: GL.stats[k] - st[k] for k in st if k != "why"}
    assert dd["captures"] >= 1 and dd["failed"] == 0 and dd["replays"] > 0, (dd, GL.stats["why"])
    assert dd["segments"] >= 2, dd              # cut at the Hessian-vector product's all-reduce
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-7)
    assert n_got == n_ref + dd["captures"], (n_got, n_ref, dd)   # + one success agreement per capture
