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
