"""Host side of the hand-written MFMA GEMM / tsmm kernels (ops/hip/gemm.hip).

Reference: LibMatrixMult.java:86 (matrixMult, `ba+*`), :331 (matrixMultTransposeSelf, tsmm)
and the GPU path LibMatrixCUDA.java:477 (matmultTSMM) / LibMatrixCuMatMult (cuBLAS).

Every dense GPU `%*%` that is not tall-skinny (those go to the row-streaming kernels in
ops/kernels.py) runs here:

* operand orientation is read from torch strides, so `t(A) %*% B`, `A %*% t(B)` and tsmm
  never materialise a transpose: a K-contiguous operand is consumed as is, an M/N-contiguous
  one through the hardware transpose read (ds_read_b64_tr_b16) in the kernel;
* bf16 operands run on the bf16 matrix cores (fp32 accumulate, fp32 result); an fp32
  operand multiplied with a bf16-stored one is split into hi + lo bf16 planes stacked along
  the free dimension, so one pass over the big bf16 operand yields a ~2^-17-accurate product;
* fp32 / fp64 operand pairs run the exact-precision f32 / f64 MFMA kernel;
* split-K (fp32 slabs + a reduction pass) fills the chip when the output has few tiles
  (t(X) %*% Y, tsmm of a tall X).
"""
from __future__ import annotations

import ctypes

import torch

from ..parser.errors import DMLRuntimeError

_DCODE = {torch.bfloat16: 2, torch.float32: 4, torch.float64: 8}
_lib = None
counters = {}
SLAB_BUDGET = 2 << 30          # bytes of split-K partials we are willing to allocate
_CUS = {}


def _L():
    global _lib
    if _lib is None:
        from . import kernels
        L = kernels.load(required=True)
        L.sysml_gemm.restype = ctypes.c_int
        L.sysml_gemm.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                 ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_void_p]
        L.sysml_gemm_tile.restype = ctypes.c_int
        L.sysml_gemm_tile.argtypes = [ctypes.c_int]
        L.sysml_gemm_ktile.restype = ctypes.c_int
        L.sysml_gemm_ktile.argtypes = [ctypes.c_int]
        L.sysml_gemm_set_bk.restype = None
        L.sysml_gemm_set_bk.argtypes = [ctypes.c_int]
        L.sysml_gemm_set_pf.restype = None
        L.sysml_gemm_set_pf.argtypes = [ctypes.c_int]
        _lib = L
    return _lib


def set_bk(bk):
    """bf16 K-tile override for A/B runs: 32 (4 LDS stages, counted vmcnt), 64 (2 stages), 0 = auto."""
    _L().sysml_gemm_set_bk(int(bk))


def set_pf(on):
    """bf16 main-loop variant for A/B runs (gemm.hip): 0/False the 8-wave kernel everywhere,
    1/True the register-pipelined one (gemm_bf16_pf) for plain GEMMs (the default), 2 also for
    the image-blocked DNN GEMMs (opt-in: measured no faster on ResNet-50)."""
    _L().sysml_gemm_set_pf(int(on))


def _count(k):
    counters[k] = counters.get(k, 0) + 1


def _cus(dev):
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    if i not in _CUS:
        _CUS[i] = torch.cuda.get_device_properties(i).multi_processor_count
    return _CUS[i]


def _r8(n):
    return (n + 7) & ~7


def _lhs(P, bf16):
    """Logical M x K operand -> (tensor, ta, lda): ta=0 K-contiguous rows, ta=1 stored [K][lda]."""
    M, K = P.shape
    s0, s1 = P.stride()
    if s1 == 1 and s0 >= max(K, 1) and M > 0:
        t, ta, ld = P, 0, s0
    elif s0 == 1 and s1 >= max(M, 1):
        t, ta, ld = P, 1, s1
    else:
        t, ta, ld = P.contiguous(), 0, max(K, 1)
    if bf16 and not _aligned(t, ld, K if ta == 0 else M):
        if ta == 0:
            buf = torch.zeros((M, _r8(K)), dtype=t.dtype, device=t.device)
            buf[:, :K] = t
            t, ld = buf, _r8(K)
        else:
            buf = torch.zeros((K, _r8(M)), dtype=t.dtype, device=t.device)
            buf[:, :M] = t.t()
            t, ld = buf, _r8(M)
    return t, ta, ld


def _rhs(Q, bf16):
    """Logical K x N operand -> (tensor, tb, ldb): tb=0 stored [K][ldb], tb=1 stored [N][ldb]."""
    K, N = Q.shape
    s0, s1 = Q.stride()
    if s1 == 1 and s0 >= max(N, 1) and K > 0:
        t, tb, ld = Q, 0, s0
    elif s0 == 1 and s1 >= max(K, 1):
        t, tb, ld = Q, 1, s1
    else:
        t, tb, ld = Q.contiguous(), 0, max(N, 1)
    if bf16 and not _aligned(t, ld, N if tb == 0 else K):
        if tb == 0:
            buf = torch.zeros((K, _r8(N)), dtype=t.dtype, device=t.device)
            buf[:, :N] = t
            t, ld = buf, _r8(N)
        else:
            buf = torch.zeros((N, _r8(K)), dtype=t.dtype, device=t.device)
            buf[:, :K] = t.t()
            t, ld = buf, _r8(K)
    return t, tb, ld


def _aligned(t, ld, cdim):
    return ld % 8 == 0 and t.data_ptr() % 16 == 0 and ld >= _r8(cdim) and ld * 256 < (1 << 31)


def _ksplit(code, M, N, K, tri, dev):
    L = _L()
    tile, kt = L.sysml_gemm_tile(code), L.sysml_gemm_ktile(code)
    tm, tn = -(-M // tile), -(-N // tile)
    tiles = tm * (tm + 1) // 2 if tri else tm * tn
    conc = _cus(dev) * (1 if code == 2 else 2)      # resident blocks: 128 KiB LDS (bf16) / 2 per CU
    ktiles = -(-K // kt)
    if tiles >= conc * 3 // 4 or ktiles < 8:
        return 1
    ks = max(1, min(conc // tiles, ktiles // 4))
    esz = 8 if code == 8 else 4
    while ks > 1 and ks * M * N * esz > SLAB_BUDGET:
        ks //= 2
    return ks


def _launch(code, P, ta, lda, Q, tb, ldb, C, M, N, K, tri=0, beta=0):
    L = _L()
    ks = _ksplit(code, M, N, K, tri, C.device)
    slab = None
    if ks > 1:
        slab = torch.empty((ks, M, N), dtype=C.dtype, device=C.device)
    st = torch.cuda.current_stream(C.device).cuda_stream
    rc = L.sysml_gemm(code, P.data_ptr(), lda, ta, Q.data_ptr(), ldb, tb, C.data_ptr(), C.stride(0), M, N, K, ks,
                      slab.data_ptr() if slab is not None else None, tri, beta, st)
    if rc != 0:
        raise DMLRuntimeError(f"sysml_gemm failed (rc={rc}, dtype={code}, M={M}, N={N}, K={K}, ta={ta}, tb={tb})")
    _count(("gemm.bf16" if code == 2 else "gemm.f32" if code == 4 else "gemm.f64") + (".tsmm" if tri else ""))
    return C


def _planes(x):
    hi = x.to(torch.bfloat16)
    lo = (x - hi.to(x.dtype)).to(torch.bfloat16)
    return hi, lo


def matmul(P, Q, out_dtype=None):
    """C = P @ Q for logical (possibly transposed-view) CUDA tensors P (M x K), Q (K x N)."""
    M, K = P.shape
    K2, N = Q.shape
    if K != K2:
        raise DMLRuntimeError(f"Matrix multiplication dimension mismatch: {M}x{K} %*% {K2}x{N}")
    dev = P.device
    if Q.device != dev:
        Q = Q.to(dev)
    pb, qb = P.dtype == torch.bfloat16, Q.dtype == torch.bfloat16
    if M == 0 or N == 0:
        dt = out_dtype or (torch.float32 if pb or qb else torch.promote_types(P.dtype, Q.dtype))
        return torch.zeros((M, N), dtype=dt, device=dev)
    if K == 0:
        dt = out_dtype or (torch.float32 if pb or qb else torch.promote_types(P.dtype, Q.dtype))
        return torch.zeros((M, N), dtype=dt, device=dev)
    if pb or qb:
        from .backend import backend
        if backend.act_bf16_min_cells > 0 and pb != qb:
            # bf16-activation training (DNN layers): the fp32 operand (a weight) is used as ONE
            # bf16 plane, cached per tensor version (kernels._wcast), like the convolutions' filters
            # -- not the hi / lo two-plane split that keeps fp32 accuracy for the solvers
            from . import kernels
            def one_plane(t):
                if t.is_contiguous():
                    return kernels._wcast.get(t, dev, torch.bfloat16)
                if t.t().is_contiguous():              # t(W) of a stored weight: its cached transposed copy
                    return kernels._wcast.get(t.t(), dev, torch.bfloat16, trans=True)
                return t.to(torch.bfloat16)
            C = _bf16(P, one_plane(Q)) if pb else _bf16(one_plane(P), Q)
            return C if out_dtype is None else C.to(out_dtype)
        if pb and not qb:
            # one pass over the bf16 operand: stack Q's hi / lo planes along N
            hi, lo = _planes(Q)
            C2 = _bf16(P, torch.cat([hi, lo], dim=1))
            C = C2[:, :N] + C2[:, N:]
        elif qb and not pb:
            hi, lo = _planes(P)
            C2 = _bf16(torch.cat([hi, lo], dim=0), Q)
            C = C2[:M] + C2[M:]
        else:
            C = _bf16(P, Q)
        return C if out_dtype is None else C.to(out_dtype)
    dt = torch.promote_types(P.dtype, Q.dtype)
    if dt not in (torch.float32, torch.float64):
        dt = torch.float32
    P, Q = P.to(dt), Q.to(dt)
    code = _DCODE[dt]
    Pt, ta, lda = _lhs(P, False)
    Qt, tb, ldb = _rhs(Q, False)
    C = torch.empty((M, N), dtype=dt, device=dev)
    _launch(code, Pt, ta, lda, Qt, tb, ldb, C, M, N, K)
    return C if out_dtype is None else C.to(out_dtype)


def _bf16(P, Q):
    M, K = P.shape
    N = Q.shape[1]
    Pt, ta, lda = _lhs(P, True)
    Qt, tb, ldb = _rhs(Q, True)
    C = torch.empty((M, N), dtype=torch.float32, device=P.device)
    return _launch(2, Pt, ta, lda, Qt, tb, ldb, C, M, N, K)


def tsmm(X, left=True):
    """t(X) %*% X (left) or X %*% t(X): only the upper block triangle is computed."""
    P = X.t() if left else X
    Q = X if left else X.t()
    M, K = P.shape
    dev = X.device
    if X.dtype == torch.bfloat16:
        Pt, ta, lda = _lhs(P, True)
        Qt, tb, ldb = _rhs(Q, True)
        C = torch.empty((M, M), dtype=torch.float32, device=dev)
        return _launch(2, Pt, ta, lda, Qt, tb, ldb, C, M, M, K, tri=1)
    dt = X.dtype if X.dtype in (torch.float32, torch.float64) else torch.float32
    P, Q = P.to(dt), Q.to(dt)
    Pt, ta, lda = _lhs(P, False)
    Qt, tb, ldb = _rhs(Q, False)
    C = torch.empty((M, M), dtype=dt, device=dev)
    return _launch(_DCODE[dt], Pt, ta, lda, Qt, tb, ldb, C, M, M, K, tri=1)
