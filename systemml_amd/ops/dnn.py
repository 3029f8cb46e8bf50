"""DNN builtins (reference: runtime/matrix/data/LibMatrixDNN*.java, LibMatrixCuDNN.java,
src/main/cpp/libmatrixdnn.cpp; DML signatures in parser/BuiltinFunctionExpression.java).

DML keeps images as 2-D matrices: input  N x (C*H*W)  (row-major C,H,W per row),
filter F x (C*Hf*Wf).  These functions view them as NCHW tensors and run the
convolution / pooling on the backend device (MIOpen-backed PyTorch kernels on the
MI355X, oneDNN/ATen on the host), returning 2-D matrices again.
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


def conv2d(x, w, input_shape=None, filter_shape=None, stride=None, padding=None, **kw):
    N, C, H, W, s, p = _dims(input_shape, filter_shape, stride, padding)
    Fo, C2, Hf, Wf = filter_shape
    if C2 != C:
        raise DMLRuntimeError("conv2d: channel mismatch between input and filter")
    xi = x.reshape(-1, C, H, W)
    wi = w.reshape(Fo, C, Hf, Wf).to(xi.dtype)
    out = F.conv2d(xi, wi, stride=tuple(s), padding=tuple(p))
    return out.reshape(out.shape[0], -1)


def conv2d_backward_filter(x, dout, input_shape=None, filter_shape=None, stride=None, padding=None, **kw):
    N, C, H, W, s, p = _dims(input_shape, filter_shape, stride, padding)
    Fo, _, Hf, Wf = filter_shape
    Ho, Wo = _out_hw(H, W, Hf, Wf, s, p)
    xi = x.reshape(-1, C, H, W)
    do = dout.reshape(-1, Fo, Ho, Wo).to(xi.dtype)
    gw = torch.nn.grad.conv2d_weight(xi, (Fo, C, Hf, Wf), do, stride=tuple(s), padding=tuple(p))
    return gw.reshape(Fo, -1)


def conv2d_backward_data(w, dout, input_shape=None, filter_shape=None, stride=None, padding=None, **kw):
    N, C, H, W, s, p = _dims(input_shape, filter_shape, stride, padding)
    Fo, _, Hf, Wf = filter_shape
    Ho, Wo = _out_hw(H, W, Hf, Wf, s, p)
    do = dout.reshape(-1, Fo, Ho, Wo)
    wi = w.reshape(Fo, C, Hf, Wf).to(do.dtype)
    gx = torch.nn.grad.conv2d_input((do.shape[0], C, H, W), wi, do, stride=tuple(s), padding=tuple(p))
    return gx.reshape(gx.shape[0], -1)


def pool(x, kind="max", input_shape=None, pool_size=None, stride=None, padding=None, **kw):
    N, C, H, W, s, p = _dims(input_shape, None, stride, padding)
    kh, kw_ = pool_size
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
    return dout * (x > 0).to(dout.dtype)
