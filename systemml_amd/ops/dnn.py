"""DNN builtins (reference: runtime/matrix/data/LibMatrixDNN*.java, LibMatrixCuDNN.java,
src/main/cpp/libmatrixdnn.cpp; DML signatures in parser/BuiltinFunctionExpression.java).

DML keeps images as 2-D matrices: input  N x (C*H*W)  (row-major C,H,W per row),
filter F x (C*Hf*Wf).  On the MI355X every operator runs a hand-written kernel directly on
the 2-D matrices: ops/hip/dnn.hip (implicit-GEMM convolutions on MFMA -- bf16 operands on
bf16 MFMA, fp32 / fp64 on exact MFMA --, im2col / col2im, pooling and its backward pass,
channel-wise bias add / multiply and relu backward) and the image-blocked MFMA GEMM of
ops/hip/gemm.hip for 1x1 stride-1 convolutions, im2col forward and col2im backward data
(ops/kernels.py:_gemm_img; bias and relu in its epilogue).  No library GEMM (hipBLASLt /
rocBLAS) is called on this path.  On the host the same operators run through ATen on NCHW
views.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..parser.errors import DMLRuntimeError


def _dims(input_shape=None, filter_shape=None, stride=None, padding=None, pool_size=None):
    if input_shape is None:
        raise DMLRuntimeError("DNN builtin requires input_shape=[N,C,H,W]")
    N, C, H, W = input_shape
    s = stride or [1, 1]
    p = padding or [0, 0]
    return N, C, H, W, s, p


def _out_hw(H, W, kh, kw, s, p):
    return (H + 2 * p[0] - kh) // s[0] + 1, (W + 2 * p[1] - kw) // s[1] + 1


def _hip(*ts):
    from .backend import backend
    return backend.use_kernels and all(t is not None and t.is_cuda and t.layout == torch.strided for t in ts)


def _check(x, N, C, H, W, what):
    if x.shape[1] != C * H * W:
        raise DMLRuntimeError(f"{what}: input has {x.shape[1]} columns, expected C*H*W = {C * H * W}")
    return x.shape[0]


def conv2d(x, w, input_shape=None, filter_shape=None, stride=None, padding=None, bias=None, relu=False, **kw):
    N, C, H, W, s, p = _dims(input_shape, filter_shape, stride, padding)
    Fo, C2, Hf, Wf = filter_shape
    if C2 != C:
        raise DMLRuntimeError("conv2d: channel mismatch between input and filter")
    if w.shape[0] != Fo or w.shape[1] != C * Hf * Wf:
        raise DMLRuntimeError(f"conv2d: filter is {tuple(w.shape)}, expected {Fo}x{C * Hf * Wf}")
    if bias is not None and tuple(bias.shape) not in ((Fo, 1), (Fo,)):
        # the fused conv2d + bias_add epilogue (compiler/rewrites.fuse_conv_bias) reads one bias
        # per filter; any other bias shape keeps the unfused bias_add semantics (and its checks)
        out = conv2d(x, w, input_shape, filter_shape, stride, padding)
        out = bias_op(out, bias, mult=False)
        return torch.relu(out) if relu else out
    if _hip(x, w):
        from . import kernels as K
        n = _check(x, N, C, H, W, "conv2d")
        r = K.conv2d(0, x, w, None, n, C, H, W, Fo, Hf, Wf, s[0], s[1], p[0], p[1], bias=bias, relu=relu)
        if r is not None:
            return r
    xi = x.reshape(-1, C, H, W)
    wi = w.reshape(Fo, C, Hf, Wf).to(xi.dtype)
    out = F.conv2d(xi, wi, stride=tuple(s), padding=tuple(p))
    if bias is not None:
        out = out + bias.reshape(1, -1, 1, 1).to(out.dtype)
    if relu:
        out = torch.relu(out)
    return out.reshape(out.shape[0], -1)


def conv2d_backward_filter(x, dout, input_shape=None, filter_shape=None, stride=None, padding=None, **kw):
    N, C, H, W, s, p = _dims(input_shape, filter_shape, stride, padding)
    Fo, _, Hf, Wf = filter_shape
    Ho, Wo = _out_hw(H, W, Hf, Wf, s, p)
    if _hip(x, dout):
        from . import kernels as K
        n = _check(x, N, C, H, W, "conv2d_backward_filter")
        r = K.conv2d(2, x, None, dout, n, C, H, W, Fo, Hf, Wf, s[0], s[1], p[0], p[1])
        if r is not None:
            return r
    xi = x.reshape(-1, C, H, W)
    do = dout.reshape(-1, Fo, Ho, Wo).to(xi.dtype)
    gw = torch.nn.grad.conv2d_weight(xi, (Fo, C, Hf, Wf), do, stride=tuple(s), padding=tuple(p))
    return gw.reshape(Fo, -1)


def conv2d_backward_data(w, dout, input_shape=None, filter_shape=None, stride=None, padding=None, **kw):
    N, C, H, W, s, p = _dims(input_shape, filter_shape, stride, padding)
    Fo, _, Hf, Wf = filter_shape
    Ho, Wo = _out_hw(H, W, Hf, Wf, s, p)
    if _hip(w, dout):
        from . import kernels as K
        if dout.shape[1] != Fo * Ho * Wo:
            raise DMLRuntimeError(f"conv2d_backward_data: dout has {dout.shape[1]} columns, expected {Fo * Ho * Wo}")
        r = K.conv2d(1, None, w, dout, dout.shape[0], C, H, W, Fo, Hf, Wf, s[0], s[1], p[0], p[1])
        if r is not None:
            return r
    do = dout.reshape(-1, Fo, Ho, Wo)
    wi = w.reshape(Fo, C, Hf, Wf).to(do.dtype)
    gx = torch.nn.grad.conv2d_input((do.shape[0], C, H, W), wi, do, stride=tuple(s), padding=tuple(p))
    return gx.reshape(gx.shape[0], -1)


def pool(x, kind="max", input_shape=None, pool_size=None, stride=None, padding=None, **kw):
    N, C, H, W, s, p = _dims(input_shape, None, stride, padding)
    kh, kw_ = pool_size
    if _hip(x):
        from . import kernels as K
        n = _check(x, N, C, H, W, kind + "_pool")
        r = K.pool2d(False, kind != "max", x, None, n, C, H, W, kh, kw_, s[0], s[1], p[0], p[1])
        if r is not None:
            return r
    xi = x.reshape(-1, C, H, W)
    if kind == "max":
        if p[0] or p[1]:
            xi = F.pad(xi, (p[1], p[1], p[0], p[0]), value=-float("inf"))
        out = F.max_pool2d(xi, (kh, kw_), stride=tuple(s))
    else:
        out = F.avg_pool2d(xi, (kh, kw_), stride=tuple(s), padding=tuple(p), count_include_pad=True)
    return out.reshape(out.shape[0], -1)


def pool_backward(x, dout, kind="max", input_shape=None, pool_size=None, stride=None, padding=None, **kw):
    N, C, H, W, s, p = _dims(input_shape, None, stride, padding)
    kh, kw_ = pool_size
    if _hip(x, dout):
        from . import kernels as K
        n = _check(x, N, C, H, W, kind + "_pool_backward")
        r = K.pool2d(True, kind != "max", x, dout, n, C, H, W, kh, kw_, s[0], s[1], p[0], p[1])
        if r is not None:
            return r
    xi = x.reshape(-1, C, H, W).detach().clone().requires_grad_(True)
    with torch.enable_grad():
        if kind == "max":
            xp = F.pad(xi, (p[1], p[1], p[0], p[0]), value=-float("inf")) if (p[0] or p[1]) else xi
            out = F.max_pool2d(xp, (kh, kw_), stride=tuple(s))
        else:
            out = F.avg_pool2d(xi, (kh, kw_), stride=tuple(s), padding=tuple(p), count_include_pad=True)
        g = torch.autograd.grad(out, xi, dout.reshape(out.shape).to(out.dtype))[0]
    return g.reshape(g.shape[0], -1)


def relu_backward(x, dout):
    if _hip(x, dout):
        from . import kernels as K
        return K.relu_backward(x, dout)
    return dout * (x > 0).to(dout.dtype)


def bias_op(x, b, mult=False):
    """bias_add / bias_multiply: b (C x 1) broadcast over the H*W cells of each channel."""
    b = b.reshape(-1)
    C_ = b.numel()
    if x.shape[1] % C_:
        raise DMLRuntimeError(f"bias_{'multiply' if mult else 'add'}: {x.shape[1]} columns not a multiple of {C_}")
    if _hip(x, b):
        from . import kernels as K
        r = K.bias_op(x, b, mult)
        if r is not None:
            return r
    xr = x.reshape(x.shape[0], C_, -1)
    br = b.reshape(1, C_, 1).to(x.dtype)
    return (xr * br if mult else xr + br).reshape(x.shape[0], -1)
