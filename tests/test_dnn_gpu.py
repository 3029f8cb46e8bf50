"""Hand-written CDNA4 DNN kernels (ops/hip/dnn.hip) against fp64 PyTorch references of the
same operators: implicit-GEMM conv2d forward / backward-data / backward-filter (exact fp32 and
fp64 MFMA, bf16 MFMA for bf16 operands), max / avg pooling and their backward passes, bias
add / multiply and relu backward.  Reference tests: test/integration/functions/tensor/
{Conv2DTest, Conv2DBackwardTest, Conv2DBackwardDataTest, PoolTest, PoolBackwardTest}."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [  # N, C, H, W, F, K, stride, pad
    (3, 5, 11, 9, 7, 3, 1, 1),
    (2, 3, 16, 16, 16, 5, 2, 2),
    (4, 8, 7, 7, 6, 1, 1, 0),
    (2, 2, 9, 13, 3, 3, 2, 0),
    (1, 64, 14, 14, 96, 3, 1, 1),
    # both GEMM dimensions >= 128 on the bf16 path: 128 x 128 tiles, ragged edges
    (2, 130, 9, 11, 136, 3, 1, 1),
    (3, 160, 8, 8, 200, 1, 1, 0),
    (2, 129, 15, 15, 131, 3, 2, 1),
]


def _ref_conv(X, W, N, C, H, Wd, F_, K, s, p):
    x = X.double().cpu().reshape(N, C, H, Wd).requires_grad_(True)
    w = W.double().cpu().reshape(F_, C, K, K).requires_grad_(True)
    out = F.conv2d(x, w, stride=s, padding=p)
    g = torch.randn(out.shape, dtype=torch.float64, generator=torch.Generator().manual_seed(7))
    out.backward(g)
    return out.reshape(N, -1).detach(), g.reshape(N, -1), x.grad.reshape(N, -1), w.grad.reshape(F_, -1)


@pytest.mark.parametrize("dt,tol", [(torch.float64, 1e-12), (torch.float32, 2e-5), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("shape", SHAPES)
def test_conv2d_kernels(shape, dt, tol):
    from systemml_amd.ops import kernels as Kn
    N, C, H, Wd, F_, K, s, p = shape
    g = torch.Generator().manual_seed(sum(shape))
    X = torch.randn(N, C * H * Wd, generator=g, dtype=torch.float64)
    W = torch.randn(F_, C * K * K, generator=g, dtype=torch.float64)
    if dt == torch.bfloat16:       # reference on the bf16-rounded operands
        X, W = X.to(dt).double(), W.to(dt).double()
    out, G, dX, dW = _ref_conv(X, W, N, C, H, Wd, F_, K, s, p)
    if dt == torch.bfloat16:
        G = G.to(dt).double()
    dev = torch.device("cuda:0")
    Xd, Wdv, Gd = X.to(dev, dt), W.to(dev, dt), G.to(dev, dt)
    c0 = dict(Kn.counters)
    got = Kn.conv2d(0, Xd, Wdv, None, N, C, H, Wd, F_, K, K, s, s, p, p)
    gx = Kn.conv2d(1, None, Wdv, Gd, N, C, H, Wd, F_, K, K, s, s, p, p)
    gw = Kn.conv2d(2, Xd, None, Gd, N, C, H, Wd, F_, K, K, s, s, p, p)
    torch.cuda.synchronize()
    for name, a, b in (("fwd", got, out), ("bwd_data", gx, dX), ("bwd_filter", gw, dW)):
        a = a.double().cpu()
        scale = b.abs().max().item() + 1e-30
        err = (a - b).abs().max().item() / scale
        assert err < tol, (name, err)
    assert Kn.counters["conv2d"] > c0.get("conv2d", 0)
    assert Kn.counters["conv2d_bwd_filter"] > c0.get("conv2d_bwd_filter", 0)


def test_conv2d_bias_relu_epilogue():
    from systemml_amd.ops import kernels as Kn
    N, C, H, Wd, F_, K = 2, 3, 8, 8, 5, 3
    g = torch.Generator().manual_seed(1)
    X = torch.randn(N, C * H * Wd, generator=g)
    W = torch.randn(F_, C * K * K, generator=g)
    b = torch.randn(F_, 1, generator=g)
    ref = torch.relu(F.conv2d(X.reshape(N, C, H, Wd), W.reshape(F_, C, K, K), padding=1) + b.reshape(1, -1, 1, 1))
    dev = torch.device("cuda:0")
    got = Kn.conv2d(0, X.to(dev), W.to(dev), None, N, C, H, Wd, F_, K, K, 1, 1, 1, 1, bias=b.to(dev), relu=True)
    np.testing.assert_allclose(got.cpu().numpy(), ref.reshape(N, -1).numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
@pytest.mark.parametrize("cfg", [(2, 3, 8, 8, 2, 2, 0), (3, 4, 9, 7, 3, 2, 1), (1, 2, 6, 6, 3, 1, 1),
                                 (5, 9, 7, 7, 7, 1, 0), (2, 3, 11, 11, 11, 2, 0)])    # last two: global windows
def test_pooling_kernels(cfg, dt):
    from systemml_amd.ops import kernels as Kn
    N, C, H, W, k, s, p = cfg
    g = torch.Generator().manual_seed(k * 10 + s)
    X = torch.randn(N, C * H * W, generator=g, dtype=torch.float64)
    dev = torch.device("cuda:0")
    for avg in (False, True):
        x = X.reshape(N, C, H, W).clone().requires_grad_(True)
        if avg:
            o = F.avg_pool2d(x, k, s, p, count_include_pad=True)
        else:
            o = F.max_pool2d(F.pad(x, (p, p, p, p), value=-float("inf")), k, s)
        G = torch.randn(o.shape, generator=g, dtype=torch.float64)
        o.backward(G)
        got = Kn.pool2d(False, avg, X.to(dev, dt), None, N, C, H, W, k, k, s, s, p, p)
        gx = Kn.pool2d(True, avg, X.to(dev, dt), G.reshape(N, -1).to(dev, dt), N, C, H, W, k, k, s, s, p, p)
        tol = 1e-12 if dt == torch.float64 else 1e-5
        np.testing.assert_allclose(got.double().cpu().numpy(), o.detach().reshape(N, -1).numpy(), rtol=tol, atol=tol)
        np.testing.assert_allclose(gx.double().cpu().numpy(), x.grad.reshape(N, -1).numpy(), rtol=tol, atol=tol)


@pytest.mark.parametrize("P", [10, 12, 49, 3136])      # P % 4 == 0: the 4-wide vector kernel
@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
def test_bias_and_relu_backward_kernels(P, dt):
    from systemml_amd.ops import kernels as Kn
    g = torch.Generator().manual_seed(3 + P)
    X = torch.randn(6, 4 * P, generator=g, dtype=torch.float64)
    b = torch.randn(4, 1, generator=g, dtype=torch.float64)
    D = torch.randn(6, 4 * P, generator=g, dtype=torch.float64)
    dev = torch.device("cuda:0")
    xr = X.reshape(6, 4, P)
    Xd, bd = X.to(dev, dt), b.to(dev, dt)
    tol = 1e-15 if dt == torch.float64 else 1e-6
    np.testing.assert_allclose(Kn.bias_op(Xd, bd).double().cpu().numpy(),
                               (xr + b.reshape(1, 4, 1)).reshape(6, -1).numpy(), rtol=tol, atol=tol)
    np.testing.assert_allclose(Kn.bias_op(Xd, bd, mult=True).double().cpu().numpy(),
                               (xr * b.reshape(1, 4, 1)).reshape(6, -1).numpy(), rtol=tol, atol=tol)
    np.testing.assert_allclose(Kn.relu_backward(Xd, D.to(dev, dt)).double().cpu().numpy(), (D * (X > 0)).numpy(),
                               rtol=tol, atol=tol)


def test_lenet_builtins_use_hip_kernels_end_to_end():
    """The nn library's conv / pool layers on the GPU backend run the dnn.hip kernels and
    match the CPU backend."""
    from systemml_amd.api.executor import run
    from systemml_amd.conf import DMLConfig
    from systemml_amd.ops import kernels as Kn
    src = """
o = conv2d(X, W, input_shape=[8,1,12,12], filter_shape=[4,1,3,3], stride=[1,1], padding=[1,1])
o = bias_add(o, b)
p = max_pool(o, input_shape=[8,4,12,12], pool_size=[2,2], stride=[2,2], padding=[0,0])
dp = max_pool_backward(o, p, input_shape=[8,4,12,12], pool_size=[2,2], stride=[2,2], padding=[0,0])
dw = conv2d_backward_filter(X, dp, input_shape=[8,1,12,12], filter_shape=[4,1,3,3], stride=[1,1], padding=[1,1])
dx = conv2d_backward_data(W, dp, input_shape=[8,1,12,12], filter_shape=[4,1,3,3], stride=[1,1], padding=[1,1])
s = sum(p) + sum(dw) + sum(dx)
"""
    rng = np.random.default_rng(1)
    ins = {"X": rng.random((8, 144)), "W": rng.random((4, 9)) - 0.5, "b": rng.random((4, 1))}
    c0 = dict(Kn.counters)
    gpu = run(src, inputs=ins, outputs=["s", "dw", "dx"], config=DMLConfig(gpu=True, gpu_min_cells=0),
              out=lambda s: None)
    cpu = run(src, inputs=ins, outputs=["s", "dw", "dx"], config=DMLConfig(gpu=False), out=lambda s: None)
    assert abs(float(gpu["s"]) - float(cpu["s"])) < 1e-9 * abs(float(cpu["s"]))
    for k in ("conv2d", "conv2d_bwd_filter", "conv2d_bwd_data", "pool", "pool_bwd"):
        assert Kn.counters.get(k, 0) > c0.get(k, 0), k
    # bias_add(conv2d(..)) is fused into the convolution's epilogue (conv2d + bias rewrite)
    assert Kn.counters.get("bias_add", 0) == c0.get("bias_add", 0)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 130, 9, 11, 136, 3, 1, 1), (4, 256, 7, 7, 128, 1, 1, 0), (1, 64, 14, 14, 96, 3, 1, 1),
                                   # the 7 x 7 / 2 RGB stem and a C <= 8 layer with F not a multiple
                                   # of 8: backward data on the direct kernel
                                   (2, 3, 32, 32, 64, 7, 2, 3), (2, 5, 12, 12, 20, 3, 1, 1)])
def test_conv2d_fp32_operands_on_bf16_mfma(shape):
    """fp32 activations / filters computed on bf16 MFMA (the ResNet bench mode, dtype code 3):
    against an fp64 reference of the bf16-rounded operands."""
    from systemml_amd.ops import kernels as Kn
    N, C, H, Wd, F_, K, s, p = shape
    g = torch.Generator().manual_seed(7 + sum(shape))
    X = torch.randn(N, C * H * Wd, generator=g, dtype=torch.float64)
    W = torch.randn(F_, C * K * K, generator=g, dtype=torch.float64)
    Xr, Wr = X.to(torch.bfloat16).double(), W.to(torch.bfloat16).double()
    _, G, _, _ = _ref_conv(Xr, Wr, N, C, H, Wd, F_, K, s, p)
    Gr = G.to(torch.bfloat16).double()
    dev = torch.device("cuda:0")
    old = Kn.CONV_BF16_FP32
    Kn.CONV_BF16_FP32 = True
    try:
        Xd, Wdv, Gd = X.to(dev, torch.float32), W.to(dev, torch.float32), Gr.to(dev, torch.float32)
        got = Kn.conv2d(0, Xd, Wdv, None, N, C, H, Wd, F_, K, K, s, s, p, p)
        gx = Kn.conv2d(1, None, Wdv, Gd, N, C, H, Wd, F_, K, K, s, s, p, p)
        gw = Kn.conv2d(2, Xd, None, Gd, N, C, H, Wd, F_, K, K, s, s, p, p)
    finally:
        Kn.CONV_BF16_FP32 = old
    torch.cuda.synchronize()
    x = Xr.reshape(N, C, H, Wd).requires_grad_(True)
    w = Wr.reshape(F_, C, K, K).requires_grad_(True)
    o = torch.nn.functional.conv2d(x, w, stride=s, padding=p)
    o.backward(Gr.reshape(o.shape))
    for name, a, b in (("fwd", got, o.reshape(N, -1).detach()), ("bwd_data", gx, x.grad.reshape(N, -1)),
                       ("bwd_filter", gw, w.grad.reshape(F_, -1))):
        a = a.double().cpu()
        err = (a - b).abs().max().item() / (b.abs().max().item() + 1e-30)
        assert err < 2e-2, (name, err)


def test_compare_backends_harness_quick():
    """The nn/test/compare_backends harness (CPU fp64 vs GPU backend for every DNN builtin,
    reference scripts/nn/test/compare_backends/run_tests.sh) in its quick sweep."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import importlib.util
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "systemml_amd/scripts/nn/test/compare_backends/run_tests.py")
    spec = importlib.util.spec_from_file_location("cmp_backends", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.main(["--quick"]) == 0


@pytest.mark.parametrize("shape", [(3, 64, 7, 7, 64), (2, 32, 14, 14, 160), (2, 64, 56, 56, 64), (3, 128, 28, 28, 128),
                                   (5, 96, 5, 9, 64), (1, 32, 3, 100, 256)])
def test_conv3_direct_forward_and_backward_data(shape, monkeypatch):
    """3x3 stride-1 pad-1 layers on the direct convolution of conv3.hip (input patch staged once
    per 32 channels; pixel tiles spanning images at 7x7 / 5x9; 64-row filter tiles for <= 64
    outputs; ragged filter tiles): forward with bias + relu epilogue and backward data against
    fp64 torch on the bf16-rounded operands."""
    from systemml_amd.ops import kernels as Kn
    from systemml_amd.ops.backend import backend
    monkeypatch.setattr(backend, "act_bf16_min_cells", 1)
    N, C, H, Wd, F_ = shape
    g = torch.Generator().manual_seed(sum(shape))
    X = torch.randn(N, C * H * Wd, generator=g, dtype=torch.float64).to(torch.bfloat16).double()
    W = (torch.randn(F_, C * 9, generator=g, dtype=torch.float64) / (3 * C ** 0.5)).to(torch.bfloat16).double()
    b = torch.randn(F_, 1, generator=g, dtype=torch.float64)
    out, G, dX, _ = _ref_conv(X, W, N, C, H, Wd, F_, 3, 1, 1)
    G = G.to(torch.bfloat16).double()
    x = X.reshape(N, C, H, Wd)
    dX = torch.nn.grad.conv2d_input(x.shape, W.reshape(F_, C, 3, 3), G.reshape(N, F_, H, Wd), padding=1).reshape(N, -1)
    ref = torch.relu(out.reshape(N, F_, H * Wd) + b.reshape(1, F_, 1)).reshape(N, -1)
    dev = torch.device("cuda:0")
    c0 = Kn.counters.get("conv3_direct", 0)
    got = Kn.conv2d(0, X.to(dev, torch.bfloat16), W.float().to(dev), None, N, C, H, Wd, F_, 3, 3, 1, 1, 1, 1,
                    bias=b.float().to(dev), relu=True)
    gx = Kn.conv2d(1, None, W.float().to(dev), G.to(dev, torch.bfloat16), N, C, H, Wd, F_, 3, 3, 1, 1, 1, 1)
    torch.cuda.synchronize()
    assert Kn.counters.get("conv3_direct", 0) == c0 + 2
    assert got.dtype == torch.bfloat16 and gx.dtype == torch.bfloat16
    for name, a, r in (("fwd", got, ref), ("bwd_data", gx, dX)):
        a = a.double().cpu()
        err = (a - r).abs().max().item() / (r.abs().max().item() + 1e-30)
        assert err < 1e-2, (name, err)


@pytest.mark.parametrize("shape", [(2, 64, 56, 56, 256), (3, 256, 14, 14, 1024), (5, 512, 7, 7, 96), (2, 40, 9, 9, 24)])
def test_wgrad_1x1_batched_nt_gemm(shape):
    """1x1 stride-1 filter gradient on wgrad.hip (images as the split-K axis, slab reduction;
    16-B / 8-B / scalar pixel loads for H*W % 8, % 4, odd) against fp64 torch."""
    from systemml_amd.ops import kernels as Kn
    N, C, H, Wd, F_ = shape
    g = torch.Generator().manual_seed(sum(shape))
    X = torch.randn(N, C * H * Wd, generator=g, dtype=torch.float64).to(torch.bfloat16).double()
    G = torch.randn(N, F_ * H * Wd, generator=g, dtype=torch.float64).to(torch.bfloat16).double()
    ref = torch.einsum("nfp,ncp->fc", G.reshape(N, F_, -1), X.reshape(N, C, -1))
    dev = torch.device("cuda:0")
    c0 = Kn.counters.get("wgrad_1x1", 0)
    got = Kn.conv2d(2, X.to(dev, torch.bfloat16), None, G.to(dev, torch.bfloat16), N, C, H, Wd, F_, 1, 1, 1, 1, 0, 0)
    torch.cuda.synchronize()
    assert Kn.counters.get("wgrad_1x1", 0) == c0 + 1
    err = (got.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-4, err


@pytest.mark.parametrize("shape", [(2, 64, 56, 56, 64), (3, 128, 28, 28, 128), (4, 256, 14, 14, 96), (5, 64, 7, 7, 200),
                                   (2, 40, 9, 13, 24)])
def test_wgrad3_direct_filter_gradient(shape, monkeypatch):
    """3x3 stride-1 pad-1 filter gradient on wgrad.hip (rows padded to 8-pixel runs, input patch
    staged as three column-shifted copies, chunks split over blocks with a slab reduction)
    against fp64 torch on the bf16-rounded operands (the kernel is opt-in: SYSML_WGRAD3=1)."""
    from systemml_amd.ops import kernels as Kn
    monkeypatch.setattr(Kn, "WGRAD3", True)
    N, C, H, Wd, F_ = shape
    g = torch.Generator().manual_seed(sum(shape))
    X = torch.randn(N, C * H * Wd, generator=g, dtype=torch.float64).to(torch.bfloat16).double()
    G = torch.randn(N, F_ * H * Wd, generator=g, dtype=torch.float64).to(torch.bfloat16).double()
    ref = torch.nn.grad.conv2d_weight(X.reshape(N, C, H, Wd), (F_, C, 3, 3), G.reshape(N, F_, H, Wd),
                                      padding=1).reshape(F_, -1)
    dev = torch.device("cuda:0")
    c0 = Kn.counters.get("wgrad_3x3", 0)
    got = Kn.conv2d(2, X.to(dev, torch.bfloat16), None, G.to(dev, torch.bfloat16), N, C, H, Wd, F_, 3, 3, 1, 1, 1, 1)
    torch.cuda.synchronize()
    assert Kn.counters.get("wgrad_3x3", 0) == c0 + 1
    err = (got.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-4, err
