"""cbind / rbind and left indexing on ops/hip/reorg.hip against torch (bit-exact copies), for
bf16 / fp32 / fp64 cells, ragged widths, many operands, scalar and matrix windows and the
update-in-place form; and through DML on the GPU backend against the CPU backend."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _need():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from systemml_amd.ops import kernels
    kernels.load(required=True)
    return kernels


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32, torch.float64])
@pytest.mark.parametrize("rows", [False, True])
def test_cat_matches_torch(dt, rows):
    K = _need()
    g = torch.Generator().manual_seed(3)
    shapes = [(37, 5), (37, 1), (37, 130), (37, 3), (37, 64)] if not rows else [(5, 37), (1, 37), (130, 37), (3, 37)]
    mats = [torch.randn(s, generator=g).to("cuda", dt) for s in shapes]
    before = K.counters.get("rbind" if rows else "cbind", 0)
    got = K.cat(rows, mats)
    ref = torch.cat(mats, 0 if rows else 1)
    torch.cuda.synchronize()
    assert K.counters.get("rbind" if rows else "cbind", 0) == before + 1
    assert torch.equal(got, ref)


def test_cat_sixteen_operands_and_strided_inputs():
    K = _need()
    mats = [torch.full((9, k + 1), float(k), device="cuda") for k in range(16)]
    mats[3] = torch.randn(20, 9, device="cuda").t()[:, :4]          # a strided view
    assert torch.equal(K.cat(False, mats), torch.cat(mats, 1))
    assert K.cat(False, mats + [mats[0]]) is None                    # > 16: declined


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32, torch.float64])
def test_lix_matches_torch(dt):
    K = _need()
    X = torch.randn(300, 70, device="cuda").to(dt)
    Y = torch.randn(40, 7, device="cuda").to(dt)
    out = torch.empty_like(X)
    assert K.lix(X, Y, out, 10, 50, 3, 10)
    ref = X.clone()
    ref[10:50, 3:10] = Y
    assert torch.equal(out, ref)
    out2 = torch.empty_like(X)
    assert K.lix(X, 2.5, out2, 0, 300, 69, 70)
    ref2 = X.clone()
    ref2[:, 69] = 2.5
    assert torch.equal(out2, ref2)
    # in place: only the window is written
    Z = X.clone()
    assert K.lix(Z, Y, Z, 100, 140, 60, 67)
    ref3 = X.clone()
    ref3[100:140, 60:67] = Y
    assert torch.equal(Z, ref3)


def test_append_and_left_indexing_through_dml():
    _need()
    from systemml_amd.api import executor as EX
    from systemml_amd.conf import DMLConfig
    from systemml_amd.ops import kernels
    src = """
    A = cbind(X, Y, X)
    B = rbind(X, Y)
    C = X
    C[5:20, 2:3] = Y[1:16, 1:2]
    C[1, ] = matrix(7, rows=1, cols=ncol(C))
    for (i in 1:4) { C[i * 10, 1] = i }
    """
    rng = np.random.default_rng(2)
    ins = {"X": rng.random((200, 150)), "Y": rng.random((200, 150))}
    before = {k: kernels.counters.get(k, 0) for k in ("cbind", "rbind", "lix")}
    res = {}
    for gpu in (True, False):
        cfg = DMLConfig(gpu=gpu, precision="double", gpu_min_cells=0)
        r, _ = EX.execute(EX.compile_script(src, {}, inputs=ins, outputs=["A", "B", "C"], config=cfg), ins)
        res[gpu] = {k: v.double().cpu().numpy() for k, v in r.items()}
    for k in ("cbind", "rbind", "lix"):
        assert kernels.counters.get(k, 0) > before[k], (k, kernels.counters)
    for k in ("A", "B", "C"):
        np.testing.assert_array_equal(res[True][k], res[False][k])


def test_append_of_host_and_device_operands():
    """GLM's rbind(t(X) %*% w, matrix(sw, 1, 1)): a small host operand joins the device one."""
    _need()
    from systemml_amd.runtime.builtins import b_rbind, b_cbind
    d = torch.arange(12, dtype=torch.float32, device="cuda").reshape(4, 3)
    h = torch.full((1, 3), 5.0)
    r = b_rbind(None, d, h)
    assert r.is_cuda and torch.equal(r.cpu(), torch.cat([d.cpu(), h]))
    r2 = b_rbind(None, h, d)
    assert r2.is_cuda and torch.equal(r2.cpu(), torch.cat([h, d.cpu()]))
    c = b_cbind(None, torch.ones(4, 1), d)
    assert c.is_cuda and torch.equal(c.cpu(), torch.cat([torch.ones(4, 1), d.cpu()], 1))


@pytest.mark.parametrize("dt", [torch.float32, torch.float64, torch.bfloat16])
def test_left_index_device_scalar_without_host_read(dt, monkeypatch):
    """R[i, j] = s with s a device-resident scalar: the kernel reads s on the device; the
    DevScalar is never materialised on the host."""
    _need()
    from systemml_amd.ops import core as C
    from systemml_amd.ops.backend import backend
    monkeypatch.setattr(backend, "use_kernels", True)
    from systemml_amd.runtime.scalars import DevScalar
    X = torch.zeros(50, 7, dtype=dt, device="cuda")
    s = DevScalar(torch.tensor(3.25, dtype=torch.float64, device="cuda"))
    out = C.lix(X, s, 5, 5, 2, 3)
    assert s._v is None                                 # not read on the host
    ref = torch.zeros(50, 7, dtype=torch.float64)
    ref[4, 1:3] = 3.25
    assert torch.equal(out.double().cpu(), ref)
