"""GPU numerics of the hand-written MFMA GEMM / tsmm kernels (ops/hip/gemm.hip) against an
fp64 torch reference: ragged (non tile-multiple) shapes, every operand orientation
(A %*% B, t(A) %*% B, A %*% t(B), t(A) %*% t(B)), K from 1 to 4096, split-K, and tsmm."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=[32, 64])
def G(request):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from systemml_amd.ops import gemm
    gemm.set_bk(request.param)
    yield gemm
    gemm.set_bk(0)


def _mk(shape, dt, trans, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    r, c = shape
    base = torch.rand((c, r) if trans else (r, c), generator=g, device="cuda", dtype=torch.float64) * 2 - 1
    base = base.to(dt)
    return base.t() if trans else base


def _check(C, P, Q, tol):
    ref = P.double() @ Q.double()
    bound = P.double().abs() @ Q.double().abs()
    err = (C.double() - ref).abs()
    worst = (err - tol * bound - 1e-30).max().item()
    assert worst <= 0, f"max err {err.max().item():.3e} (bound {tol:g} * |A||B|)"


SHAPES = [(1, 1, 1), (7, 9, 5), (100, 9, 130), (257, 64, 255), (300, 100, 513), (256, 256, 256),
          (512, 4096, 300), (64, 777, 1000), (1000, 33, 8)]
TOL = {torch.bfloat16: 2e-6, torch.float32: 2e-6, torch.float64: 1e-14}


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32, torch.float64])
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("M,K,N", SHAPES)
def test_gemm_layouts(G, dt, ta, tb, M, K, N):
    P = _mk((M, K), dt, ta, 1 + M + K)
    Q = _mk((K, N), dt, tb, 2 + N)
    C = G.matmul(P, Q)
    assert C.shape == (M, N)
    # bf16 products are exact in fp32; the error is fp32 accumulation (~K * 2^-24)
    _check(C, P, Q, TOL[dt] * max(1, K) ** 0.5 * 8)


def test_gemm_identity_asymmetric(G):
    # A = I with an asymmetric B catches a transposed C/D write
    for dt in (torch.bfloat16, torch.float32, torch.float64):
        n = 300
        I = torch.eye(n, dtype=dt, device="cuda")
        B = torch.arange(n * 280, device="cuda", dtype=torch.float64).reshape(n, 280).remainder(97).to(dt)
        assert torch.equal(G.matmul(I, B).double(), B.double())
        assert torch.equal(G.matmul(B.t(), I).double(), B.t().double())


def test_gemm_mixed_bf16_fp32(G):
    P = _mk((3000, 512), torch.bfloat16, False, 3)
    Q = _mk((512, 70), torch.float32, False, 4)
    C = G.matmul(P, Q)
    _check(C, P.float(), Q, 2e-5)
    C2 = G.matmul(Q.t(), P.t())
    _check(C2, Q.t(), P.t().float(), 2e-5)


def test_gemm_splitk_tall(G):
    # t(X) %*% Y with X 200000 x 96: few output tiles, long K -> split-K slabs
    X = _mk((200_000, 96), torch.bfloat16, False, 5)
    Y = _mk((200_000, 40), torch.bfloat16, False, 6)
    C = G.matmul(X.t(), Y)
    _check(C, X.t(), Y, 2e-6 * 450 * 8)
    for dt in (torch.float32, torch.float64):
        Xf, Yf = X.to(dt), Y.to(dt)
        _check(G.matmul(Xf.t(), Yf), Xf.t(), Yf, TOL[dt] * 450 * 8)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32, torch.float64])
@pytest.mark.parametrize("n,d", [(5000, 300), (100_000, 520), (37, 9)])
@pytest.mark.parametrize("left", [True, False])
def test_tsmm(G, dt, n, d, left):
    if not left and n > 10000:
        n = 3000
    X = _mk((n, d), dt, False, 7 + d)
    C = G.tsmm(X, left)
    P, Q = (X.t(), X) if left else (X, X.t())
    _check(C, P, Q, TOL[dt] * max(n if left else d, 1) ** 0.5 * 8)
    assert torch.equal(C, C.t())


def test_gemm_nonfinite_tail(G):
    # K-tail masking must not turn a non-finite value past K into NaN: allocate the operand
    # inside a bigger buffer with inf beyond column K
    buf = torch.full((64, 72), float("inf"), dtype=torch.bfloat16, device="cuda")
    P = buf[:, :65]
    P.copy_(_mk((64, 65), torch.bfloat16, False, 9))
    Q = _mk((65, 40), torch.bfloat16, False, 10)
    C = G.matmul(P, Q)
    assert torch.isfinite(C).all()
    _check(C, P, Q, 1e-4)


# ----------------------------------------------------------------------------- image-blocked DNN GEMM
@pytest.mark.gpu
@pytest.mark.parametrize("M,K,nimg,hw,bias,relu", [
    (64, 256, 8, 3136, True, True),      # 64-row tile, pixels a multiple of 8
    (256, 64, 16, 784, False, False),    # 256-row tile
    (512, 2048, 32, 49, True, False),    # 7 x 7 images (padded to 56), split-K
    (128, 1152, 12, 196, False, True),   # 14 x 14 (padded to 200), 64-row tile, split-K
    (1000, 72, 3, 100, True, True),      # ragged M, padded pixels
    (512, 1024, 16, 196, True, True),    # 256-row tile, K % 64 == 0, one K split
])
@pytest.mark.parametrize("pf", [1, 2])
def test_gemm_img_matches_fp32(M, K, nimg, hw, bias, relu, pf):
    """sysml_gemm_dnn: out[n] = relu(A . B[n] + bias) for all images in one launch, bf16 out,
    against an fp32 torch evaluation on the same bf16 operands."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from systemml_amd.ops import kernels as Kn
    Kn.load(required=True)
    g = torch.Generator(device="cuda").manual_seed(M + K + hw)
    A = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    B = torch.randn(nimg, K, hw, device="cuda", generator=g).to(torch.bfloat16)
    b = torch.randn(M, device="cuda", generator=g) if bias else None
    out = torch.empty(nimg, M, hw, dtype=torch.bfloat16, device="cuda")
    before = Kn.counters.get("gemm_dnn", 0)
    from systemml_amd.ops import gemm as G
    G.set_pf(pf)      # 2: the register-pipelined kernel on the image-blocked DNN path too
    try:
        Kn._gemm_img(A, B, out, M, K, nimg, hw, bias=b, relu=relu)
        torch.cuda.synchronize()
    finally:
        G.set_pf(1)
    ref = torch.matmul(A.float(), B.float())
    if bias:
        ref = ref + b.reshape(1, -1, 1)
    if relu:
        ref = torch.relu(ref)
    torch.cuda.synchronize()
    assert Kn.counters.get("gemm_dnn", 0) == before + 1
    err = (out.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-30)
    assert err < 1e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("M,K,trans,pad8", [(64, 27, False, True), (256, 2304, True, False), (147, 60, True, True),
                                           (8, 8, False, False)])
def test_weight_cast_one_pass(M, K, trans, pad8):
    """gemm.hip cast_weight: fp32 filter -> bf16 (RNE), optionally transposed and zero-padded to
    a multiple of 8 columns, in one pass; equals torch's cast of the same view."""
    from systemml_amd.ops import kernels as KK
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    KK.load(required=True)
    W = torch.randn(M, K, device="cuda")
    c0 = KK.counters.get("cast_weight", 0)
    out = KK._WeightCasts().get(W, W.device, torch.bfloat16, trans=trans, pad8=pad8)
    assert KK.counters.get("cast_weight", 0) == c0 + 1
    ref = (W.t() if trans else W).to(torch.bfloat16)
    C = ref.shape[1]
    assert out.shape[0] == ref.shape[0] and out.shape[1] == ((C + 7) // 8 * 8 if pad8 else C)
    assert torch.equal(out[:, :C], ref)
    assert not out[:, C:].any()


@pytest.mark.gpu
@pytest.mark.parametrize("M,K,nimg,hw", [(256, 2304, 16, 196), (512, 2048, 8, 49), (200, 576, 4, 784)])
def test_gemm_img_128_row_tiles(M, K, nimg, hw, monkeypatch):
    """The 128-row tile variant of the image-blocked GEMM (gemm_bf16_kernel<.., 64, 128>)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from systemml_amd.ops import kernels as Kn
    Kn.load(required=True)
    monkeypatch.setattr(Kn, "GEMM_DNN_T128", 1 << 20)
    g = torch.Generator(device="cuda").manual_seed(M + K)
    A = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    B = torch.randn(nimg, K, hw, device="cuda", generator=g).to(torch.bfloat16)
    b = torch.randn(M, device="cuda", generator=g)
    out = torch.empty(nimg, M, hw, dtype=torch.bfloat16, device="cuda")
    Kn._gemm_img(A, B, out, M, K, nimg, hw, bias=b, relu=True)
    ref = torch.relu(torch.matmul(A.float(), B.float()) + b.reshape(1, -1, 1))
    torch.cuda.synchronize()
    err = (out.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-30)
    assert err < 1e-2, err


@pytest.mark.parametrize("hw", [196, 49, 30, 8])
def test_pad_pixels_vector_paths(hw):
    """The image-blocked GEMM's pixel padding (gemm.hip pad_pixels: 8-B / 4-B / 2-B source runs,
    one 16-B store per 8 output pixels) against torch."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from systemml_amd.ops import kernels as K
    L = K.load(required=True)
    planes = 333
    hwp = (hw + 7) & ~7
    x = torch.randn(planes, hw, device="cuda").to(torch.bfloat16)
    y = torch.full((planes, hwp), 7.0, device="cuda", dtype=torch.bfloat16)
    assert L.sysml_pad_pixels(x.data_ptr(), y.data_ptr(), planes, hw, hwp, K._stream()) == 0
    ref = torch.zeros(planes, hwp, dtype=torch.bfloat16)
    ref[:, :hw] = x.cpu()
    assert torch.equal(y.cpu(), ref)
