"""bf16 activations (DMLConfig.act_bf16_min_cells): fused cellwise results, convolution outputs
(forward / backward data) and pooling results stored bf16 with fp32 arithmetic, against fp64
PyTorch references on the same bf16-rounded operands.  The mixed-precision training mode of
the ResNet-50 benchmark (BASELINE config "scripts/nn ResNet-50 training bf16")."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


class _ActBf16:
    def __init__(self, cells=1):
        self.cells = cells

    def __enter__(self):
        from systemml_amd.ops.backend import backend
        self.old = backend.act_bf16_min_cells
        backend.act_bf16_min_cells = self.cells

    def __exit__(self, *a):
        from systemml_amd.ops.backend import backend
        backend.act_bf16_min_cells = self.old


def _bf(x):
    return x.to(torch.bfloat16).double()


# GEMM depths < 1024 (no split-K: a split-K launch accumulates fp32 atomically and keeps an fp32
# output); the last shape runs the 128 x 128 tiles
@pytest.mark.parametrize("shape", [(2, 100, 9, 11, 96, 3, 1, 1), (4, 64, 14, 14, 96, 3, 1, 1),
                                   (2, 100, 15, 15, 56, 3, 2, 1), (8, 32, 8, 8, 64, 1, 1, 0),
                                   (64, 64, 28, 28, 256, 1, 1, 0), (4, 64, 14, 14, 128, 1, 2, 0),
                                   (3, 40, 13, 13, 24, 3, 2, 1),
                                   # even widths: the stride-2 paired col2im
                                   (2, 64, 16, 16, 32, 3, 2, 1), (2, 48, 14, 14, 40, 3, 2, 1),
                                   (2, 32, 12, 12, 16, 3, 2, 0), (2, 3, 32, 32, 16, 7, 2, 3),
                                   # N*F*H*W not a multiple of 4: the bias epilogue's fp32 path
                                   (1, 16, 7, 7, 3, 1, 1, 0), (1, 16, 7, 7, 3, 3, 1, 1)])
def test_conv_bf16_output(shape):
    from systemml_amd.ops import kernels as Kn
    N, C, H, Wd, F_, K, s, p = shape
    g = torch.Generator().manual_seed(sum(shape))
    X = _bf(torch.randn(N, C * H * Wd, generator=g, dtype=torch.float64))
    W = _bf(torch.randn(F_, C * K * K, generator=g, dtype=torch.float64))
    b = torch.randn(F_, 1, generator=g, dtype=torch.float64)
    ref = F.conv2d(X.reshape(N, C, H, Wd), W.reshape(F_, C, K, K), stride=s, padding=p)
    Ho, Wo = ref.shape[2], ref.shape[3]
    G = _bf(torch.randn(N, F_ * Ho * Wo, generator=g, dtype=torch.float64))
    ref_b = torch.relu(ref + b.reshape(1, -1, 1, 1)).reshape(N, -1)
    ref_dx = torch.nn.grad.conv2d_input((N, C, H, Wd), W.reshape(F_, C, K, K), G.reshape(N, F_, Ho, Wo),
                                        stride=s, padding=p).reshape(N, -1)
    dev = torch.device("cuda:0")
    with _ActBf16():
        got = Kn.conv2d(0, X.to(dev, torch.bfloat16), W.to(dev, torch.float32), None, N, C, H, Wd, F_, K, K, s, s,
                        p, p, bias=b.to(dev, torch.float32), relu=True)
        gx = Kn.conv2d(1, None, W.to(dev, torch.float32), G.to(dev, torch.bfloat16), N, C, H, Wd, F_, K, K, s, s,
                       p, p)
    torch.cuda.synchronize()
    assert got.dtype == torch.bfloat16 and gx.dtype == torch.bfloat16
    if K == 1 and s == 1 and Kn.CONV1X1_GEMM:
        assert Kn.counters.get("conv1x1_gemm", 0) >= 2
    if s > 1 and Kn.CONV1X1_GEMM:
        assert Kn.counters.get("conv_col2im", 0) >= 1          # backward data: GEMM + col2im
    if K > 1 and Ho * Wo <= Kn.IM2COL_MAX_HW and C > 8 and Kn.CONV1X1_GEMM:
        assert Kn.counters.get("conv_im2col", 0) >= 1          # forward: im2col + GEMM
    for name, a, r in (("fwd", got, ref_b), ("bwd_data", gx, ref_dx)):
        err = (a.double().cpu() - r).abs().max().item() / (r.abs().max().item() + 1e-30)
        assert err < 1e-2, (name, err)


def test_pool_bf16_storage():
    from systemml_amd.ops import kernels as Kn
    N, C, H, W = 4, 8, 13, 13
    g = torch.Generator().manual_seed(4)
    X = _bf(torch.randn(N, C * H * W, generator=g, dtype=torch.float64))
    x4 = X.reshape(N, C, H, W).requires_grad_(True)
    out = F.max_pool2d(x4, 3, stride=2, padding=1)
    D = _bf(torch.randn(out.shape, generator=g, dtype=torch.float64))
    out.backward(D)
    dev = torch.device("cuda:0")
    with _ActBf16():
        p = Kn.pool2d(False, False, X.to(dev, torch.bfloat16), None, N, C, H, W, 3, 3, 2, 2, 1, 1)
        dp = Kn.pool2d(True, False, X.to(dev, torch.bfloat16), D.reshape(N, -1).to(dev, torch.bfloat16),
                       N, C, H, W, 3, 3, 2, 2, 1, 1)
        a = Kn.pool2d(False, True, X.to(dev, torch.bfloat16), None, N, C, H, W, 3, 3, 2, 2, 1, 1)
    torch.cuda.synchronize()
    assert p.dtype == torch.bfloat16 and dp.dtype == torch.bfloat16
    assert torch.equal(p.double().cpu(), out.detach().reshape(N, -1))      # max of bf16 values: exact
    np.testing.assert_allclose(dp.double().cpu().numpy(), x4.grad.reshape(N, -1).numpy(), rtol=1e-2, atol=1e-2)
    ref_avg = F.avg_pool2d(X.reshape(N, C, H, W), 3, stride=2, padding=1, count_include_pad=True).reshape(N, -1)
    np.testing.assert_allclose(a.double().cpu().numpy(), ref_avg.numpy(), rtol=1e-2, atol=1e-2)


def test_fused_cell_bf16_result_end_to_end():
    """A fused cellwise DAG over a large operand writes its result as bf16 (fp32 math); the
    aggregate over it matches the fp64 host result within bf16 rounding."""
    from systemml_amd.api.executor import run
    from systemml_amd.conf import DMLConfig
    rng = np.random.default_rng(2)
    X = rng.standard_normal((64, 4096))
    src = "Y = max(X * 1.5 - 0.25, 0)\nZ = Y * Y + Y\ns = sum(Z)"
    cfg = DMLConfig(gpu=True, precision="single", gpu_min_cells=0, act_bf16_min_cells=1 << 16)
    res = run(src, inputs={"X": X}, outputs=["Y", "s"], config=cfg, out=lambda s: None)
    Y = np.maximum(X * 1.5 - 0.25, 0)
    assert res["Y"].dtype == torch.bfloat16
    np.testing.assert_allclose(res["Y"].double().cpu().numpy(), Y, rtol=1e-2, atol=1e-2)
    ref = float((Y * Y + Y).sum())
    assert abs(float(res["s"]) - ref) < 1e-2 * abs(ref)


def test_lenet_layers_train_with_bf16_activations():
    """conv / bias / pool / backward passes of the nn builtins with bf16 activations against
    the fp64 host run of the same script."""
    from systemml_amd.api.executor import run
    from systemml_amd.conf import DMLConfig
    src = """
o = conv2d(X, W, input_shape=[16,3,16,16], filter_shape=[32,3,3,3], stride=[1,1], padding=[1,1])
o = bias_add(o, b)
r = max(o, 0)
p = max_pool(r, input_shape=[16,32,16,16], pool_size=[2,2], stride=[2,2], padding=[0,0])
o2 = conv2d(p, W2, input_shape=[16,32,8,8], filter_shape=[16,32,3,3], stride=[1,1], padding=[1,1])
d2 = o2 * 0.5
dp = conv2d_backward_data(W2, d2, input_shape=[16,32,8,8], filter_shape=[16,32,3,3], stride=[1,1], padding=[1,1])
dw2 = conv2d_backward_filter(p, d2, input_shape=[16,32,8,8], filter_shape=[16,32,3,3], stride=[1,1], padding=[1,1])
dr = max_pool_backward(r, dp, input_shape=[16,32,16,16], pool_size=[2,2], stride=[2,2], padding=[0,0])
do = dr * (r > 0)
dw = conv2d_backward_filter(X, do, input_shape=[16,3,16,16], filter_shape=[32,3,3,3], stride=[1,1], padding=[1,1])
s1 = sum(dw)
s2 = sum(dw2)
s3 = sum(abs(p))
"""
    rng = np.random.default_rng(1)
    ins = {"X": rng.standard_normal((16, 768)), "W": rng.standard_normal((32, 27)) * 0.2,
           "b": rng.standard_normal((32, 1)) * 0.1, "W2": rng.standard_normal((16, 288)) * 0.1}
    outs = ["s1", "s2", "s3", "dw"]
    gpu = run(src, inputs=ins, outputs=outs, config=DMLConfig(gpu=True, precision="single", gpu_min_cells=0,
                                                              act_bf16_min_cells=1024), out=lambda s: None)
    cpu = run(src, inputs=ins, outputs=outs, config=DMLConfig(gpu=False), out=lambda s: None)
    for k in ("s2", "s3"):
        assert abs(float(gpu[k]) - float(cpu[k])) < 3e-2 * abs(float(cpu[k])), k
    dw_g, dw_c = gpu["dw"].double().cpu().numpy(), cpu["dw"].cpu().numpy()
    assert np.abs(dw_g - dw_c).max() < 3e-2 * np.abs(dw_c).max()


@pytest.mark.parametrize("mult,relu", [(False, False), (True, False), (False, True)])
def test_bias_op_bf16(mult, relu):
    from systemml_amd.ops import kernels as Kn
    N, C, P = 6, 8, 50
    g = torch.Generator().manual_seed(7)
    X = _bf(torch.randn(N, C * P, generator=g, dtype=torch.float64))
    b = torch.randn(C, 1, generator=g, dtype=torch.float64)
    ref = X.reshape(N, C, P) * b.reshape(1, C, 1) if mult else X.reshape(N, C, P) + b.reshape(1, C, 1)
    ref = (torch.relu(ref) if relu else ref).reshape(N, -1)
    with _ActBf16():
        got = Kn.bias_op(X.to("cuda", torch.bfloat16), b.to("cuda", torch.float32), mult=mult, relu=relu)
    torch.cuda.synchronize()
    assert got.dtype == torch.bfloat16
    np.testing.assert_allclose(got.double().cpu().numpy(), ref.numpy(), rtol=8e-3, atol=8e-3)
