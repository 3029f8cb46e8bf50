"""Python bindings for the in-tree HIP kernel library (`ops/lib/libsysml_hip.so`,
built from `ops/hip/*.hip` by `__graft_entry__.build()` / `python -m systemml_amd.ops.build`).

The library is loaded with ctypes (no torch C++ ABI coupling); kernels are
launched on PyTorch's current HIP stream so they order correctly with the
surrounding torch ops and are capturable in HIP graphs.

On a GPU box the library is REQUIRED: `load(required=True)` raises if it is
missing or fails to load, so GPU runs never silently fall back to eager torch
for the hot operators.
"""
from __future__ import annotations

import ctypes
import os

import torch
from ..utils import hosttrace as _HT

from ..parser.errors import DMLRuntimeError
from .backend import backend
from . import sparse as SP

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SYSML_HIP_LIB") or os.path.join(_HERE, "lib", "libsysml_hip.so")   # env: A/B builds
_lib = None

# modes (must match ops/hip/rowstream.hip)
XV, XTG, XTXV, XTWXV, XTXVY, XTPSXV, ROWSSQ, COLSSQ, COLSUM, ROWSUM, XTSMG, XTSMGO = range(12)
_CHAIN = {"XtXv": XTXV, "XtwXv": XTWXV, "XtXvy": XTXVY, "XtPSXv": XTPSXV}
MIN_ROWS = 2048       # below this the launch + partial reduction is not worth it
MIN_D = 32            # a wave per row: narrower rows waste most lanes (torch handles those)
MAX_D = 1024

counters = {}


def _count(name):
    counters[name] = counters.get(name, 0) + 1


def load(required=False):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        if required:
            raise DMLRuntimeError(f"HIP kernel library not built: {LIB_PATH} (run __graft_entry__.build())")
        return None
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        if required:
            raise DMLRuntimeError(f"cannot load HIP kernel library {LIB_PATH}: {e}")
        return None
    L.sysml_rowstream.restype = ctypes.c_int
    L.sysml_rowstream.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                  ctypes.c_void_p]
    L.sysml_rowstream_smg.restype = ctypes.c_int
    L.sysml_rowstream_smg.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                      ctypes.c_void_p]
    L.sysml_conv2d.restype = ctypes.c_int
    L.sysml_conv2d.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 6 + [ctypes.c_int] * 13 + \
        [ctypes.c_void_p]
    L.sysml_pool2d.restype = ctypes.c_int
    L.sysml_pool2d.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3 + [ctypes.c_int] * 10 + [ctypes.c_void_p]
    L.sysml_pool2d_ws.restype = ctypes.c_int
    L.sysml_pool2d_ws.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 10 + [ctypes.c_void_p]
    L.sysml_bias_op.restype = ctypes.c_int
    L.sysml_bias_op.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    L.sysml_relu_backward.restype = ctypes.c_int
    L.sysml_relu_backward.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_int64, ctypes.c_void_p]
    L.sysml_spmm.restype = ctypes.c_int
    L.sysml_spmm.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                             ctypes.c_int, ctypes.c_void_p]
    L.sysml_spmm_bal.restype = ctypes.c_int
    L.sysml_spmm_bal.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_void_p,
                                                                                        ctypes.c_int64, ctypes.c_int64,
                                                                                        ctypes.c_int, ctypes.c_int64,
                                                                                        ctypes.c_void_p]
    L.sysml_spgemm_count.restype = ctypes.c_int
    L.sysml_spgemm_count.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_int,
                                                                                            ctypes.c_void_p,
                                                                                            ctypes.c_void_p]
    L.sysml_spgemm_fill.restype = ctypes.c_int
    L.sysml_spgemm_fill.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 6 + [ctypes.c_int64, ctypes.c_int] + \
        [ctypes.c_void_p] * 5
    L.sysml_tsmm_sparse.restype = ctypes.c_int
    L.sysml_tsmm_sparse.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    L.sysml_sddmm2.restype = ctypes.c_int
    L.sysml_sddmm2.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.sysml_sddmm.restype = ctypes.c_int
    L.sysml_sddmm.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.sysml_set_rows_per_iter.argtypes = [ctypes.c_int]
    L.sysml_set_rows_per_iter.restype = None
    L.sysml_mchain.restype = ctypes.c_int
    L.sysml_mchain.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                               ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    L.sysml_mchain_occupancy.restype = ctypes.c_int
    L.sysml_mchain_occupancy.argtypes = [ctypes.c_int, ctypes.c_int]
    L.sysml_chain4.restype = ctypes.c_int
    L.sysml_chain4.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.c_int64, ctypes.c_void_p]
    L.sysml_chain4_occupancy.restype = ctypes.c_int
    L.sysml_chain4_occupancy.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.sysml_chain4m.restype = ctypes.c_int
    L.sysml_chain4m.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p,
                                ctypes.c_int, ctypes.c_void_p]
    L.sysml_gemm_dnn.restype = ctypes.c_int
    L.sysml_gemm_dnn.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                 ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    L.sysml_conv3s1.restype = ctypes.c_int
    L.sysml_conv3s1.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 7 + [ctypes.c_void_p]
    L.sysml_conv3_weight.restype = ctypes.c_int
    L.sysml_conv3_weight.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_void_p]
    L.sysml_wgrad_splits.restype = ctypes.c_int
    L.sysml_wgrad_splits.argtypes = [ctypes.c_int] * 4
    L.sysml_wgrad3_splits.restype = ctypes.c_int
    L.sysml_wgrad3_splits.argtypes = [ctypes.c_int] * 5
    L.sysml_wgrad3.restype = ctypes.c_int
    L.sysml_wgrad3.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 5 + [ctypes.c_void_p]
    L.sysml_wgrad_nt.restype = ctypes.c_int
    L.sysml_wgrad_nt.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 4 + [ctypes.c_int64] * 2 + [ctypes.c_void_p]
    L.sysml_csrt_count.restype = ctypes.c_int
    L.sysml_csrt_count.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p]
    L.sysml_csrt_fill.restype = ctypes.c_int
    L.sysml_csrt_fill.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    L.sysml_gather.restype = ctypes.c_int
    L.sysml_gather.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                               ctypes.c_void_p]
    L.sysml_fold_rows.restype = ctypes.c_int
    L.sysml_fold_rows.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                  ctypes.c_int64, ctypes.c_void_p]
    L.sysml_dot.restype = ctypes.c_int
    L.sysml_dot.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.c_int64, ctypes.c_void_p]
    L.sysml_cast_weight.restype = ctypes.c_int
    L.sysml_cast_weight.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_void_p]
    L.sysml_lix2.restype = ctypes.c_int
    L.sysml_lix2.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int64] * 6 + \
        [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    L.sysml_wdivmm.restype = ctypes.c_int
    L.sysml_wdivmm.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 7 + \
        [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
    L.sysml_pad_pixels.restype = ctypes.c_int
    L.sysml_pad_pixels.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_void_p]
    L.sysml_agg.restype = ctypes.c_int
    L.sysml_agg.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    L.sysml_agg_scratch.restype = ctypes.c_int64
    L.sysml_agg_scratch.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int]
    L.sysml_cat.restype = ctypes.c_int
    L.sysml_cat.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
    L.sysml_lix.restype = ctypes.c_int
    L.sysml_lix.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                            ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                            ctypes.c_uint64, ctypes.c_void_p]
    L.sysml_set_live.restype = None
    L.sysml_set_live.argtypes = [ctypes.c_void_p]
    L.sysml_chain4m_occupancy.restype = ctypes.c_int
    L.sysml_chain4m_occupancy.argtypes = [ctypes.c_int, ctypes.c_int]
    L.sysml_mwide.restype = ctypes.c_int
    L.sysml_mwide.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                              ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    L.sysml_mwide_occupancy.restype = ctypes.c_int
    L.sysml_mwide_occupancy.argtypes = [ctypes.c_int, ctypes.c_int]
    L.sysml_cumagg_chunks.restype = ctypes.c_int64
    L.sysml_cumagg_chunks.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    L.sysml_cumagg.restype = ctypes.c_int
    L.sysml_cumagg.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
    I64, VP, CI = ctypes.c_int64, ctypes.c_void_p, ctypes.c_int
    L.sysml_copy2d.restype = CI
    L.sysml_copy2d.argtypes = [CI, CI, VP, I64, VP, I64, I64, I64, VP]
    L.sysml_transpose.restype = CI
    L.sysml_transpose.argtypes = [CI, VP, I64, VP, I64, I64, VP]
    L.sysml_tri.restype = CI
    L.sysml_tri.argtypes = [CI, VP, VP, I64, I64, CI, CI, CI, VP]
    L.sysml_gather_rows.restype = CI
    L.sysml_gather_rows.argtypes = [CI, CI, VP, I64, VP, VP, I64, I64, VP]
    L.sysml_slice_csr.restype = CI
    L.sysml_slice_csr.argtypes = [CI, CI, VP, VP, VP, VP, I64, I64, I64, I64, VP]
    L.sysml_sort_keys_prep.restype = CI
    L.sysml_sort_keys_prep.argtypes = [CI, VP, I64, I64, VP, VP, VP, I64, VP]
    L.sysml_sort_pairs_scratch.restype = I64
    L.sysml_sort_pairs_scratch.argtypes = [I64]
    L.sysml_sort_pairs.restype = CI
    L.sysml_sort_pairs.argtypes = [VP, VP, VP, VP, I64, CI, VP, I64, VP]
    L.sysml_csr_block_offsets.restype = CI
    L.sysml_csr_block_offsets.argtypes = [CI, VP, VP, I64, CI, I64, VP, VP]
    L.sysml_wdivmm_blocked.restype = CI
    L.sysml_wdivmm_blocked.argtypes = [CI, CI] + [VP] * 7 + [I64, CI, CI, ctypes.c_double, I64, VP, CI, I64, VP]
    L.sysml_live_and.restype = CI
    L.sysml_live_and.argtypes = [VP, VP, VP, VP]
    L.sysml_commit_live.restype = CI
    L.sysml_commit_live.argtypes = [CI, VP, VP, VP, VP, VP]
    L.sysml_perm_compose.restype = CI
    L.sysml_perm_compose.argtypes = [VP, VP, VP, VP, CI, I64, VP]
    _lib = L
    return L


# ----------------------------------------------------------------------------
# MFMA chain kernels (ops/hip/mfma_chain.hip): bf16 X, D % 8 == 0, D <= 1024, K <= 4.
# SYSML_MFMA=0 routes everything to the VALU row-streaming kernels (A/B switch).
# ----------------------------------------------------------------------------
MFMA = os.environ.get("SYSML_MFMA", "1") != "0"
MFMA_ALL = os.environ.get("SYSML_MFMA", "1") == "all"
_occ = {}


def _mfma_ok(X, kp, mode=None):
    """MFMA path eligibility.  By measurement (profiles/mfma_chain_experiments.md) the
    matrix-core kernel wins for X %*% v with 1-2 columns and for t(X) %*% G; for the fused
    chains the prefetching VALU row-stream kernel is faster, so they stay there unless
    SYSML_MFMA=all."""
    if not (MFMA and X.dtype == torch.bfloat16 and kp <= 4 and X.shape[1] % 8 == 0 and
            X.shape[1] <= 1024 and X.is_contiguous() and X.data_ptr() % 16 == 0):
        return False
    if mode is None or MFMA_ALL:
        return True
    return mode == XTG or (mode == XV and kp <= 2)


def _mgrid(L, mode, X):
    key = (mode, X.shape[1], X.device.index)
    if key not in _occ:
        occ = L.sysml_mchain_occupancy(mode, X.shape[1])
        cus = torch.cuda.get_device_properties(X.device).multi_processor_count
        _occ[key] = max(1, occ) * cus if occ > 0 else -1
    ntiles = (X.shape[0] + 15) // 16
    return min(_occ[key], ntiles)


def _v3t(V, kp, D, device):
    """V (D x K) -> [16][Dp] bf16: rows 4s+k hold rounding plane s (hi, lo, lo2) of V[:, k]."""
    Dp = 256 * ((D + 255) // 256)
    v = V.to(device=device, dtype=torch.float32)
    planes = []
    for _ in range(3):
        h = v.to(torch.bfloat16)
        planes.append(h)
        v = v - h.to(torch.float32)
    out = torch.zeros((16, Dp), dtype=torch.bfloat16, device=device)
    for s_, h in enumerate(planes):
        out[4 * s_:4 * s_ + V.shape[1], :D] = h.t()
    return out


def _mchain(mode, X, kp, V=None, S=None, sbc=0):
    L = load(required=True)
    N, D = X.shape
    grid = _mgrid(L, mode, X)
    if grid <= 0:
        return None
    V3 = _v3t(V, kp, D, X.device) if V is not None else None
    if S is not None:
        S = S.to(device=X.device, dtype=torch.float32).contiguous()
    if mode == XV:
        out = torch.empty((N, kp), dtype=torch.float32, device=X.device)
        ldo = kp
    else:
        out = torch.empty((grid, D * kp), dtype=torch.float32, device=X.device)
        ldo = 0
    rc = L.sysml_mchain(mode, ctypes.c_void_p(X.data_ptr()), N, D,
                        ctypes.c_void_p(V3.data_ptr() if V3 is not None else 0),
                        ctypes.c_void_p(S.data_ptr() if S is not None else 0), S.shape[1] if S is not None else 0,
                        sbc, kp, ctypes.c_void_p(out.data_ptr()), ldo, grid, _stream())
    if rc != 0:
        return None
    if mode == XV:
        return out
    return _psum(out).reshape(D, kp)


WIDE_MAX = 16


def _wide_ok(X, K):
    """Wide MFMA products (5..16 columns, e.g. the 10-class MultiLogReg): bf16 X only."""
    return (MFMA and X.dtype == torch.bfloat16 and 4 < K <= WIDE_MAX and X.shape[1] % 8 == 0 and
            X.shape[1] <= 1024 and X.is_contiguous() and X.data_ptr() % 16 == 0)


def _wide_planes(V, D, device):
    """V (D x K, K <= 16) -> [3][16][Dp] bf16: plane p (hi, lo, lo2 rounding residues) of
    V[:, k] in row k of plane p."""
    K = V.shape[1]
    Dp = 256 * ((D + 255) // 256)
    v = V.to(device=device, dtype=torch.float32)
    VW = torch.zeros((3, 16, Dp), dtype=torch.bfloat16, device=device)
    for pl in range(3):
        h = v.to(torch.bfloat16)
        VW[pl, :K, :D] = h.t()
        v = v - h.to(torch.float32)
    return VW


def _mwide(mode, X, V=None, G=None, sbc=0, U=None, obj=None):
    """Wide products and chains with up to 16 columns (ops/hip/mfma_chain.hip wide_kernel):
    each of the three bf16 planes of V / G is its own MFMA into a 16-column tile.
    mode XV: U = X %*% V; XTG: t(X) %*% G; chains (XTXV / XTWXV / XTXVY / XTPSXV, G = the
    row-side operand w / y / P): t(X) %*% g(X %*% V) in one pass over X.  Softmax modes (G = Y):
    XTSMG writes X %*% V into U, XTSMGO the K + 1 class probabilities, appending its
    (blocks * waves, 2) fp64 objective partials to the list `obj`."""
    L = load(required=True)
    N, D = X.shape
    key = ("wide", mode, D, X.device.index)
    if key not in _occ:
        occ = L.sysml_mwide_occupancy(mode, D)
        cus = torch.cuda.get_device_properties(X.device).multi_processor_count
        _occ[key] = max(1, occ) * cus if occ > 0 else -1
    grid = min(_occ[key], (N + 15) // 16)
    if grid <= 0:
        return None
    K = V.shape[1] if V is not None else G.shape[1]
    VW = _wide_planes(V, D, X.device) if V is not None else None
    S, lds = _rows_f32(G, G.shape[1], sbc, X.device) if G is not None else (None, 0)
    up = ctypes.c_void_p(U.data_ptr() if U is not None else 0)
    ldu = U.stride(0) if U is not None else 0
    ob = None
    if mode == XTSMGO:
        ob = torch.empty((grid * 16, 2), dtype=torch.float64, device=X.device)
        ob.zero_()
    op = ctypes.c_void_p(ob.data_ptr() if ob is not None else 0)
    vp = ctypes.c_void_p(VW.data_ptr() if VW is not None else 0)
    sp = ctypes.c_void_p(S.data_ptr() if S is not None else 0)
    if mode == XV:
        out = torch.empty((N, K), dtype=torch.float32, device=X.device)
        rc = L.sysml_mwide(mode, ctypes.c_void_p(X.data_ptr()), N, D, vp, sp, lds, K,
                           ctypes.c_void_p(out.data_ptr()), K, grid, _stream(), up, ldu, op)
        return out if rc == 0 else None
    part = torch.empty((grid, D * K), dtype=torch.float32, device=X.device)
    rc = L.sysml_mwide(mode, ctypes.c_void_p(X.data_ptr()), N, D, vp, sp, lds, K,
                       ctypes.c_void_p(part.data_ptr()), 0, grid, _stream(), up, ldu, op)
    if rc != 0:
        return None
    if obj is not None and ob is not None:
        obj.append(ob)
    return _psum(part).reshape(D, K)


def _xcode(x):
    if x.dtype == torch.bfloat16:
        return 0, torch.float32
    if x.dtype == torch.float32:
        return 1, torch.float32
    if x.dtype == torch.float64:
        return 2, torch.float64
    return None, None


def _kpad(k):
    for p in (1, 2, 4, 8):
        if k <= p:
            return p
    return None


def _grid(n):
    cus = 256
    g = min((n + 63) // 64, cus * 4)
    return max(g, 1)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _dense(x):
    """x itself when contiguous, else a dense copy of the (row-major, any pitch) view on
    reorg.hip's copy2d -- no ATen copy kernel on HBM data."""
    if x.is_contiguous():
        return x
    if x.is_cuda and x.dim() == 2:
        r = copy2d(x)
        if r is not None:
            return r
    return x.contiguous()


def _pad_cols(m, kp, dt, device=None):
    m = m.to(dtype=dt) if device is None else m.to(device=device, dtype=dt)
    if m.shape[1] == kp and m.is_contiguous():
        return m
    out = torch.zeros((m.shape[0], kp), dtype=dt, device=m.device)
    out[:, :m.shape[1]] = m
    return out


def _launch(mode, X, V=None, S=None, sbc=0, K=1, out=None, ldo=1, grid=None):
    L = load(required=True)
    code, adt = _xcode(X)
    N, D = X.shape
    grid = grid or _grid(N)
    rpb = (N + grid - 1) // grid
    grid = (N + rpb - 1) // rpb
    rc = L.sysml_rowstream(mode, code, ctypes.c_void_p(X.data_ptr()), N, D,
                           ctypes.c_void_p(V.data_ptr() if V is not None else 0), V.shape[1] if V is not None else 0,
                           ctypes.c_void_p(S.data_ptr() if S is not None else 0), S.shape[1] if S is not None else 0,
                           sbc, ctypes.c_void_p(out.data_ptr()), ldo, K, grid, rpb, _stream())
    return rc, grid


def _ok_x(X):
    return (X.is_cuda and X.dim() == 2 and X.is_contiguous() and X.shape[0] >= MIN_ROWS
            and MIN_D <= X.shape[1] <= MAX_D and _xcode(X)[0] is not None)


def _result(t):
    # fp64 results (fp64 X) are kept exact; fp32 accumulations follow the backend dtype
    return t if (t.dtype == backend.dtype or t.dtype == torch.float64) else t.to(backend.dtype)


def xv(X, V):
    """U = X %*% V for tall X (N x D, D <= 1024) and skinny V (D x K, K <= 8; bf16 X: K <= 16)."""
    K = V.shape[1]
    if _wide_ok(X, K):
        U = _mwide(XV, X, V=V)
        if U is not None:
            _count("mfma.xv_wide")
            return _result(U)
    if K > 8:
        return None
    kp = _kpad(K)
    code, adt = _xcode(X)
    if X.dtype == torch.bfloat16 and K > 4:
        # 8 accumulator columns x 16 values per lane spill in the row-stream kernel (22 ms
        # vs 2 x 3.8 ms measured): run two 4-column passes instead
        a = xv(X, V[:, :4])
        b = xv(X, V[:, 4:])
        return None if a is None or b is None else torch.cat([a, b], dim=1)
    if _mfma_ok(X, kp, XV):
        U = _mchain(XV, X, kp, V=V)
        if U is not None:
            _count("mfma.xv")
            return _result(U if kp == K else _dense(U[:, :K]))
    Vp = _pad_cols(V, kp, adt, X.device).contiguous()
    U = torch.empty((X.shape[0], kp), dtype=adt, device=X.device)
    rc, _ = _launch(XV, X, V=Vp, K=kp, out=U, ldo=kp)
    if rc != 0:
        return None
    _count("rowstream.xv")
    return _result(U if kp == K else _dense(U[:, :K]))


def xtg(X, G):
    """R = t(X) %*% G for tall X and skinny G (N x K, K <= 8; bf16 X: K <= 16)."""
    K = G.shape[1]
    if _wide_ok(X, K):
        R = _mwide(XTG, X, G=G)
        if R is not None:
            _count("mfma.xtg_wide")
            return _result(R)
    if K > 8:
        return None
    kp = _kpad(K)
    code, adt = _xcode(X)
    Gp = _pad_cols(G, kp, adt, X.device).contiguous()
    if _mfma_ok(X, kp, XTG):
        R = _mchain(XTG, X, kp, S=Gp)
        if R is not None:
            _count("mfma.xtg")
            return _result(R if kp == K else _dense(R[:, :K]))
    grid = _grid(X.shape[0])
    part = torch.empty((grid, X.shape[1] * kp), dtype=adt, device=X.device)
    rc, g = _launch(XTG, X, S=Gp, K=kp, out=part, grid=grid)
    if rc != 0:
        return None
    _count("rowstream.xtg")
    R = _psum(part[:g]).reshape(X.shape[1], kp)
    return _result(R if kp == K else _dense(R[:, :K]))


# ----------------------------------------------------------------------------
# Row-group chain kernels (ops/hip/chain4.hip): batched transposing reductions over 4 rows.
# SYSML_CHAIN4=0 routes the chains back to the per-row rowstream kernels (A/B switch).
# ----------------------------------------------------------------------------
CHAIN4 = os.environ.get("SYSML_CHAIN4", "1") != "0"
_c4occ = {}


def _c4_ok(X, mode, kp):
    # K = 1 chains (LinregCG's XtXv) stay on the per-row kernel: one dot product per row has
    # nothing to batch and rowstream streams it 4-7 % faster (profiles/chain4_kbench_r2.txt)
    if not (CHAIN4 and X.dtype in (torch.bfloat16, torch.float32) and kp in ((1, 2, 4) if mode == XTSMG else (2, 4))):
        return False
    if X.shape[1] % 8 or X.data_ptr() % 16 or not X.is_contiguous():
        return False
    # the K = 4, D > 512 bf16 XtXv instantiation spills (hipcc register allocation): rowstream
    return not (mode == XTXV and kp == 4 and X.dtype == torch.bfloat16 and X.shape[1] > 512)


def _c4m(X, kp):
    """The matrix-core variant (chain4m_kernel: both products on 4x4x4 bf16 MFMAs) serves
    bf16 X with K = 4; SYSML_C4M=0 keeps the VALU kernel (A/B switch)."""
    return C4M and kp == 4 and X.dtype == torch.bfloat16


C4M = os.environ.get("SYSML_C4M", "1") != "0"
# kernel schedule variant (A/B tuning): 1 = row-side value and G planes read with the first
# batch of row / transposed reads (one lgkmcnt wait less per phase; profiles/chain4m_kbench_r3.txt)
C4M_VARIANT = int(os.environ.get("SYSML_C4M_VARIANT", "1"))


def _c4_grid(L, mode, X, kp):
    code = 0 if X.dtype == torch.bfloat16 else 1
    m = _c4m(X, kp)
    key = (mode, code, kp, X.shape[1] > 512, X.device.index, m)
    if key not in _c4occ:
        occ = L.sysml_chain4m_occupancy(mode, X.shape[1]) if m else L.sysml_chain4_occupancy(mode, code, kp, X.shape[1])
        cus = torch.cuda.get_device_properties(X.device).multi_processor_count
        _c4occ[key] = max(1, occ) * cus
    return _c4occ[key]


def _rows_f32(S, kp, sbc, device):
    """Row-side operand for chain4 as (fp32 tensor, leading dimension) without a copy when it is
    already an fp32 row-major view (e.g. P[, 1:K] of a wider P): the kernel reads S[r*lds + k]."""
    if S.device != device:
        S = S.to(device)
    if S.dtype != torch.float32:
        S = S.float()
    if S.stride(1) == 1 and S.stride(0) >= S.shape[1] and S.data_ptr() % 4 == 0:
        return S, S.stride(0)
    S = _dense(S)
    return S, S.shape[1]


def _chain4(mode, X, kp, V, S, lds, sbc, U=None, ldu=0, obj=None):
    """Launch chain4; returns the D x kp fp32 result (sum of the per-block partials).  `obj`
    (XTSMGO): a list that receives the (grid * 4, 2) fp64 objective partials."""
    L = load(required=True)
    N, D = X.shape
    code = 0 if X.dtype == torch.bfloat16 else 1
    grid = min(_c4_grid(L, mode, X, kp), (N + 63) // 64)
    rpb = (N + grid - 1) // grid
    grid = (N + rpb - 1) // rpb
    part = torch.empty((grid, D * kp), dtype=torch.float32, device=X.device)
    if S is None:
        S, lds = V, 0      # the kernel streams a row-side operand in every mode: any valid memory
    _HT.mark("chain-launch")
    if _c4m(X, kp):
        ob = None
        if obj is not None:
            ob = torch.empty((grid * 4, 2), dtype=torch.float64, device=X.device)
            obj.append(ob)
        rc = L.sysml_chain4m(mode, ctypes.c_void_p(X.data_ptr()), N, D, ctypes.c_void_p(V.data_ptr()), kp,
                             ctypes.c_void_p(S.data_ptr()), lds, sbc, ctypes.c_void_p(part.data_ptr()),
                             ctypes.c_void_p(U.data_ptr() if U is not None else 0), ldu, grid, rpb, _stream(),
                             C4M_VARIANT, ctypes.c_void_p(ob.data_ptr() if ob is not None else 0))
        if rc == 0:
            _count("chain4m")
    else:
        rc = L.sysml_chain4(mode, code, ctypes.c_void_p(X.data_ptr()), N, D, ctypes.c_void_p(V.data_ptr()), kp,
                            ctypes.c_void_p(S.data_ptr()), lds, sbc, ctypes.c_void_p(part.data_ptr()),
                            ctypes.c_void_p(U.data_ptr() if U is not None else 0), ldu, kp, grid, rpb, _stream())
    if rc != 0:
        return None
    return _psum(part).reshape(D, kp)


def _psum(part):
    """Sum over the leading (workgroup) dimension of a kernel's partial results, on agg.hip's
    16-byte-load column reduction (fp64 accumulation; torch's strided reduction over a
    grid x D*K fp32 block was ~90 us per call at D = 1001): returns the flattened sums."""
    g = part.shape[0]
    p2 = part.reshape(g, -1)
    if part.is_cuda and p2.dtype == torch.float32 and p2.shape[1] % 4 == 0 and p2.shape[1] >= 64 and g > 1 \
            and p2.is_contiguous():
        r = agg("sum", "col", p2)
        if r is not None:
            return r.reshape(-1)
    return part.sum(0).reshape(-1)


def mmchain(ctype, X, V, W=None):
    mode = _CHAIN[ctype]
    K = V.shape[1]
    kp = _kpad(K)
    code, adt = _xcode(X)
    sbc = 0
    if W is not None:
        if W.shape[0] != X.shape[0]:
            return None
        if mode == XTWXV and W.shape[1] == 1:
            sbc = 1
        elif W.shape[1] != K:
            return None

    def padded_S():
        # the row-side operand as a contiguous, kp-wide copy (only the paths that need one
        # build it: it is an N x kp pass over HBM per call)
        if W is None:
            return None
        if sbc:
            return W.to(device=X.device, dtype=adt).contiguous()
        return _pad_cols(W, kp, adt, X.device).contiguous()

    if _wide_ok(X, K):
        R = _mwide(mode, X, V=V, G=W, sbc=sbc)
        if R is not None:
            _count("mfma.mmchain_wide." + ctype)
            return _result(R)
    if kp is None:
        return None
    if _c4_ok(X, mode, kp):
        Vf = _pad_cols(V, kp, torch.float32, X.device).contiguous()
        # W as is (strided views included) when the kernel reads no column past it: sbc broadcast
        # or W already kp wide; otherwise the zero-padded copy
        src = W if (W is not None and (sbc or W.shape[1] == kp)) else padded_S()
        Sf, lds = _rows_f32(src, kp, sbc, X.device) if src is not None else (None, 0)
        R = _chain4(mode, X, kp, Vf, Sf, lds, sbc)
        if R is not None:
            _count("chain4.mmchain." + ctype)
            return _result(R if kp == K else _dense(R[:, :K]))
    S = padded_S()
    if _mfma_ok(X, kp, mode):
        R = _mchain(mode, X, kp, V=V, S=S, sbc=sbc)
        if R is not None:
            _count("mfma.mmchain." + ctype)
            return _result(R if kp == K else _dense(R[:, :K]))
    grid = _grid(X.shape[0])
    part = torch.empty((grid, X.shape[1] * kp), dtype=adt, device=X.device)
    Vp = _pad_cols(V, kp, adt, X.device).contiguous()
    rc, g = _launch(mode, X, V=Vp, S=S, sbc=sbc, K=kp, out=part, grid=grid)
    if rc != 0:
        return None
    _count("rowstream.mmchain." + ctype)
    R = _psum(part[:g]).reshape(X.shape[1], kp)
    return _result(R if kp == K else _dense(R[:, :K]))


def smobj(X, V, Y, defer=False):
    """Multinomial-logreg candidate evaluation in one pass over X (chain4m mode XTSMGO):
    with L = cbind(X %*% V, 0) and E = exp(L - rowMaxs(L)), returns (P, G, s1, s2):
    P = E / rowSums(E) (N x (K+1)), G = t(X) %*% (P[, 1:K] - Y[, 1:K]),
    s1 = sum(Y * (L - rowMaxs(L))), s2 = sum(log(rowSums(E))).  V is D x K (K <= 4), Y is
    N x (K+1).  None when the matrix-core kernel does not apply (bf16 X only)."""
    if not _ok_x(X) or X.dtype != torch.bfloat16:
        return None
    K = V.shape[1]
    if Y.shape != (X.shape[0], K + 1) or V.shape[0] != X.shape[1]:
        return None
    if K > 4:
        if not (_wide_ok(X, K) and K < WIDE_MAX):
            return None
        N = X.shape[0]
        P = torch.empty((N, K + 1), dtype=torch.float32, device=X.device)
        ob = []
        G = _mwide(XTSMGO, X, V=V, G=Y, sbc=1, U=P, obj=ob)
        if G is None:
            return None
        _count("mfma.smobj_wide")
        if defer:
            s = ob[0].sum(0)
            return _result(P), _result(G), s[0], s[1]
        s = ob[0].sum(0).tolist()
        return _result(P), _result(G), s[0], s[1]
    kp = 4                  # the matrix-core kernel's class layout; classes past K are masked
    if not (_c4_ok(X, XTSMG, kp) and _c4m(X, kp)):
        return None
    N = X.shape[0]
    Vf = _pad_cols(V, kp, torch.float32, X.device).contiguous()
    Yc, ldy = _rows_f32(Y, K + 1, 1, X.device)
    Ppad = torch.empty((N + 1, K + 1), dtype=torch.float32, device=X.device)   # row N: kernel's pad row
    ob = []
    G = _chain4(XTSMGO, X, kp, Vf, Yc, ldy, K, U=Ppad, ldu=K + 1, obj=ob)
    if G is None:
        return None
    _count("chain4m.smobj")
    if defer:                           # the caller reduces the sums further (one all-reduce)
        s = ob[0].sum(0)
        return _result(Ppad[:N]), _result(G if kp == K else _dense(G[:, :K])), s[0], s[1]
    s = ob[0].sum(0).tolist()            # one device sync for both objective terms
    return _result(Ppad[:N]), _result(G if kp == K else _dense(G[:, :K])), s[0], s[1]


def smgrad(X, V, Y):
    """(U, G) with U = X %*% V and G = t(X) %*% (softmax([U, 0])[, 1:K] - Y) in one pass over X
    (mode XTSMG: the multinomial-logreg objective / gradient at a candidate point).  V is
    D x K with K <= 4, Y is N x K.  Returns None when the kernel does not apply."""
    if not _ok_x(X) or X.dtype not in (torch.bfloat16, torch.float32):
        return None
    K = V.shape[1]
    if Y.shape != (X.shape[0], K) or V.shape[0] != X.shape[1]:
        return None
    if K > 4:
        if not (_wide_ok(X, K) and K < WIDE_MAX):
            return None
        U = torch.empty((X.shape[0], K), dtype=torch.float32, device=X.device)
        G = _mwide(XTSMG, X, V=V, G=Y, sbc=1, U=U)
        if G is None:
            return None
        _count("mfma.smgrad_wide")
        return _result(U), _result(G)
    kp = _kpad(K)
    N, D = X.shape
    if _c4_ok(X, XTSMG, kp):
        Vf = _pad_cols(V, kp, torch.float32, X.device).contiguous()
        Yc, ldy = _rows_f32(Y, K, 1, X.device)
        Upad = torch.empty((N + 1, K), dtype=torch.float32, device=X.device)   # row N: kernel's pad row
        G = _chain4(XTSMG, X, kp, Vf, Yc, ldy, K, U=Upad, ldu=K)
        if G is not None:
            _count("chain4.smgrad")
            return _result(Upad[:N]), _result(G if kp == K else _dense(G[:, :K]))
    kp = max(kp, 2)
    L = load(required=True)
    code, adt = _xcode(X)
    Vp = _pad_cols(V, kp, torch.float32, X.device).contiguous()
    Yc = Y.to(device=X.device, dtype=torch.float32).contiguous()
    Upad = torch.empty((N + 1, K), dtype=torch.float32, device=X.device)   # row N: kernel's pad row
    U = Upad[:N]
    grid = _grid(N)
    rpb = (N + grid - 1) // grid
    grid = (N + rpb - 1) // rpb
    part = torch.empty((grid, D * kp), dtype=torch.float32, device=X.device)
    rc = L.sysml_rowstream_smg(code, ctypes.c_void_p(X.data_ptr()), N, D, ctypes.c_void_p(Vp.data_ptr()), kp,
                               ctypes.c_void_p(Yc.data_ptr()), K, K, ctypes.c_void_p(Upad.data_ptr()), K,
                               ctypes.c_void_p(part.data_ptr()), kp, grid, rpb, _stream())
    if rc != 0:
        return None
    _count("rowstream.smgrad")
    G = _psum(part).reshape(D, kp)
    return _result(U), _result(G if kp == K else _dense(G[:, :K]))


# ----------------------------------------------------------------------------
# dispatch helpers used by ops/core.py
# ----------------------------------------------------------------------------
def try_mm(a, b, transA):
    """Dense GPU `%*%`: tall-skinny shapes on the row-streaming / MFMA-chain kernels, every
    other shape on the MFMA GEMM (ops/gemm.py -> ops/hip/gemm.hip)."""
    if not isinstance(b, torch.Tensor) or SP.is_sparse(b):
        return None
    if not b.is_cuda:
        b = b.to(a.device)
    if _ok_x(a):
        K = b.shape[1]
        if K <= 8 or (K <= WIDE_MAX and a.dtype == torch.bfloat16):
            if transA and b.shape[0] == a.shape[0]:
                r = xtg(a, b)
                if r is not None:
                    return r
            if not transA and b.shape[0] == a.shape[1]:
                r = xv(a, b)
                if r is not None:
                    return r
    from . import gemm
    return _result(gemm.matmul(a.t() if transA else a, b))


def try_mmchain(ctype, X, v, w):
    if not _ok_x(X) or not isinstance(v, torch.Tensor) or v.shape[0] != X.shape[1]:
        return None
    if v.shape[1] > (WIDE_MAX if _wide_ok(X, v.shape[1]) else 8):
        return None
    if w is not None and not isinstance(w, torch.Tensor):
        return None
    return mmchain(ctype, X, v, w)


def try_tsmm(x, left):
    """t(X) %*% X / X %*% t(X) on the MFMA GEMM, upper block triangle only (ops/hip/gemm.hip)."""
    from . import gemm
    return _result(gemm.tsmm(x, left))


def sumsq(x, d):
    if _ok_x(x):
        code, adt = _xcode(x)
        if d == "row":
            U = torch.empty((x.shape[0], 1), dtype=adt, device=x.device)
            rc, _ = _launch(ROWSSQ, x, K=1, out=U, ldo=1)
            if rc == 0:
                _count("rowstream.rowsumsq")
                return _result(U)
        elif d in ("col", "all"):
            grid = _grid(x.shape[0])
            part = torch.empty((grid, x.shape[1]), dtype=adt, device=x.device)
            rc, g = _launch(COLSSQ, x, K=1, out=part, grid=grid)
            if rc == 0:
                _count("rowstream.colsumsq")
                c = part[:g].sum(0).reshape(1, -1)
                if d == "all":
                    from .core import _lazy_out
                    return _lazy_out(c.sum())
                return _result(c)
    # generic: chunked to bound temporaries
    from .core import cvt
    if d == "all":
        tot = 0.0
        for s in range(0, x.shape[0], 1 << 16):
            c = cvt(x[s:s + (1 << 16)])
            tot += float(torch.sum(c * c).item())
        return tot
    xx = cvt(x)
    return torch.sum(xx * xx, dim=1 if d == "row" else 0, keepdim=True)


def wdivmm(crow, col, wv, xv, U, V, mode, eps=0.0, dtype=None):
    """Fused weighted divide / multiply product (ops/hip/sddmm.hip wdivmm_kernel):
    out[i, :] = sum_p q_p V[col_p, :] over row i's non-zeros with q = w * <U[i], V[j]> (mode 0),
    w * (<U[i], V[j]> - x) (1) or w / (<U[i], V[j]> + eps) (2); wv None: w = 1.  Returns m x K,
    or None when unsupported (K > 64)."""
    import torch
    L = load(required=True)
    m, K = U.shape
    if K < 1 or K > 64 or V.shape[1] != K or col.numel() == 0:
        return None
    if dtype is None:
        dtype = torch.float64 if torch.float64 in (U.dtype, V.dtype) else torch.float32
    U = U.to(dtype).contiguous()
    V = V.to(dtype).contiguous()
    crow = crow.to(torch.int64).contiguous()
    idx32 = col.dtype == torch.int32
    col = col.contiguous() if idx32 else col.to(torch.int64).contiguous()
    wv = wv.to(dtype).contiguous() if wv is not None else None
    xv = xv.to(dtype).contiguous() if xv is not None else None
    out = torch.zeros((m, K), dtype=dtype, device=U.device)
    nnz = int(col.numel())
    Vg, ldv = _wd_padded(V, nnz)
    blk = _wd_blocks(crow, col, idx32, V.shape[0], K * V.element_size(), nnz, m)
    if blk is not None:
        rbp, nb = blk
        rc = L.sysml_wdivmm_blocked(0 if dtype == torch.float32 else 1, int(idx32), crow.data_ptr(), col.data_ptr(),
                                    wv.data_ptr() if wv is not None else None,
                                    xv.data_ptr() if xv is not None else None, U.data_ptr(), Vg.data_ptr(),
                                    out.data_ptr(), m, K, int(mode), float(eps), nnz, rbp.data_ptr(), nb, ldv,
                                    _stream())
        if rc == 0:
            _count("wdivmm_blocked")
    else:
        rc = L.sysml_wdivmm(0 if dtype == torch.float32 else 1, int(idx32), crow.data_ptr(), col.data_ptr(),
                            wv.data_ptr() if wv is not None else None, xv.data_ptr() if xv is not None else None,
                            U.data_ptr(), Vg.data_ptr(), out.data_ptr(), m, K, int(mode), float(eps), nnz, ldv,
                            _stream())
    if rc == -1:
        return None
    if rc != 0:
        raise RuntimeError(f"sysml_wdivmm failed: {rc}")
    _count("wdivmm")
    return out


# Row padding of wdivmm's gathered factor (opt-in, SYSML_WD_PAD=1): a K-wide row whose byte
# length is not a power of two (rank 10 fp32: 40 B) straddles two 64-B segments for most column
# indices; a copy with the row pitch rounded up to a power of two keeps every gathered row in one
# segment.  Made once per factor version (the CG iterations of one ALS half-step reuse it).
# Off: ALS-CG 10M x 10M / 1e9 non-zeros measured 1.498 s padded vs 1.469 s (profiles/
# als_pad_r6.txt) -- the gathers are latency-bound, not segment-bound.
WD_PAD = os.environ.get("SYSML_WD_PAD", "0") == "1"
WD_PAD_MIN_NNZ = 1 << 22
_WD_PADDED = {}


def _wd_padded(V, nnz):
    import torch
    n, K = V.shape
    ld = 1
    while ld < K:
        ld *= 2
    if not WD_PAD or ld == K or nnz < WD_PAD_MIN_NNZ or ld * V.element_size() > 256:
        return V, K
    key = (V.data_ptr(), V._version, n, K, V.dtype)
    e = _WD_PADDED.get(key)
    if e is not None and e[0]() is V:
        return e[1], ld
    Vp = torch.zeros((n, ld), dtype=V.dtype, device=V.device)
    Vp[:, :K].copy_(V)
    import weakref
    for k in [k for k, v in _WD_PADDED.items() if v[0]() is None]:
        _WD_PADDED.pop(k, None)
    if len(_WD_PADDED) >= 2:
        _WD_PADDED.pop(next(iter(_WD_PADDED)))
    _WD_PADDED[key] = (weakref.ref(V), Vp)
    _count("wdivmm_padV")
    return Vp, ld


# Column blocking of wdivmm's V gathers (opt-in, SYSML_WD_BLOCK_MB=<block MB>): a gathered factor
# matrix larger than this many bytes is visited in column blocks of at most this size, so each
# block would stay resident in the 256 MB MALL.  Off by default: measured SLOWER on ALS-CG 10M x 10M
# / 1e9 non-zeros (1.49 s unblocked vs 1.69 / 1.86 / 2.46 s with 160 / 96 / 48 MB blocks,
# profiles/als_block_sweep_r6.txt) -- every pass re-walks all rows' pointers, and the unblocked
# gathers already hit the MALL for the most part.
WD_BLOCK_BYTES = int(float(os.environ.get("SYSML_WD_BLOCK_MB", "0")) * (1 << 20))
WD_BLOCK_MIN_NNZ = 1 << 26
_WD_PLANS = {}


def _wd_blocks(crow, col, idx32, n, row_bytes, nnz, m):
    """(row block offsets m x (nb + 1) int64, nb) for a column-blocked wdivmm, cached per pattern;
    None when V fits a block or the pattern is small."""
    if WD_BLOCK_BYTES <= 0 or nnz < WD_BLOCK_MIN_NNZ or n * row_bytes <= WD_BLOCK_BYTES:
        return None
    nb = -(-n * row_bytes // WD_BLOCK_BYTES)
    cb = -(-n // nb)
    key = (crow.data_ptr(), col.data_ptr(), nnz, m, n, nb, col._version)
    e = _WD_PLANS.get(key)
    if e is None:
        L = load(required=True)
        rbp = torch.empty((m, nb + 1), dtype=torch.int64, device=crow.device)
        rc = L.sysml_csr_block_offsets(int(idx32), crow.data_ptr(), col.data_ptr(), m, nb, cb, rbp.data_ptr(),
                                       _stream())
        if rc != 0:
            raise RuntimeError(f"sysml_csr_block_offsets failed: {rc}")
        if len(_WD_PLANS) >= 4:
            _WD_PLANS.pop(next(iter(_WD_PLANS)))
        e = _WD_PLANS[key] = (crow, col, rbp, nb)      # holds the pattern: its addresses stay unique
    return e[2], e[3]


def sddmm(crow, col, U, V, dtype=None):
    """<U[i_k], V[j_k]> at the non-zeros of a CSR pattern (ops/hip/sddmm.hip), computed and
    returned in `dtype` (fp32 or fp64; default: fp64 if either factor is fp64, else fp32 --
    bf16 factors are widened); None when the shape is unsupported."""
    import torch
    L = load(required=True)
    m, r = U.shape
    if dtype is None:
        dtype = torch.float64 if torch.float64 in (U.dtype, V.dtype) else torch.float32
    if col.numel() == 0 or r > (1024 if dtype == torch.float32 else 512):
        return None
    U = U.to(dtype).contiguous()
    V = V.to(dtype).contiguous()
    crow = crow.to(torch.int64).contiguous()
    idx32 = col.dtype == torch.int32
    col = col.contiguous() if idx32 else col.to(torch.int64).contiguous()
    out = torch.empty(col.numel(), dtype=dtype, device=U.device)
    st = torch.cuda.current_stream(U.device).cuda_stream
    rc = L.sysml_sddmm2(0 if dtype == torch.float32 else 1, int(idx32), crow.data_ptr(), col.data_ptr(), U.data_ptr(),
                        V.data_ptr(), m, r, out.data_ptr(), st)
    if rc == -1:
        return None
    if rc != 0:
        raise RuntimeError(f"sysml_sddmm failed: {rc}")
    _count("sddmm")
    return out


# ----------------------------------------------------------------------------
# DNN (ops/hip/dnn.hip)
# ----------------------------------------------------------------------------
CONV_BF16_FP32 = False     # fp32 convolutions on bf16 MFMA (fp32 accumulate) instead of exact fp32 MFMA
# 1x1 stride-1 convolutions of bf16 activations as image-blocked gemm.hip GEMMs (_gemm_img;
# SYSML_CONV1X1_GEMM=0: the implicit-GEMM kernel of dnn.hip)
CONV1X1_GEMM = os.environ.get("SYSML_CONV1X1_GEMM", "1") != "0"
CONV3_DIRECT = os.environ.get("SYSML_CONV3_DIRECT", "1") != "0"   # 3x3 stride-1 layers on conv3.hip
# 3x3 stride-1 filter gradient on wgrad.hip's patch kernel: off by default -- not faster than the
# implicit GEMM overall (tools/bench_conv_rn50.py, profiles/conv_rn50_b256_r5_wgrad3.txt: 122-239 TF;
# the 56x56 shapes, one output row per chunk, restage 3 input rows per 2 K steps)
WGRAD3 = os.environ.get("SYSML_WGRAD3", "0") == "1"
CONV_SLAB = os.environ.get("SYSML_CONV_SLAB", "1") != "0"   # backward-filter split-K into a slab, not atomics
IM2COL_MAX_HW = int(os.environ.get("SYSML_IM2COL_MAX_HW", "196"))   # forward k x k convolutions via im2col + GEMM up to this Ho*Wo
COL2IM_MAX_HW = int(os.environ.get("SYSML_COL2IM_MAX_HW", "196"))   # stride-1 backward data via GEMM + col2im up to this H*W (measured: faster at 14 x 14 and 7 x 7, slower at 28 x 28 and 56 x 56)
CONV_SPLIT_BLOCKS = int(os.environ.get("SYSML_CONV_SPLIT_BLOCKS", "2048"))   # split K until ~this many blocks
CONV_SPLIT_MINK = int(os.environ.get("SYSML_CONV_SPLIT_MINK", "1536"))       # ... each reducing >= this many products (sweep: profiles/conv_split_sweep_r4.txt)


class _WeightCasts:
    """bf16 copies of fp32 filters, keyed by tensor identity and version and dropped with the
    tensor: a training step reads each filter twice (forward, backward data) but casts it once."""

    def __init__(self):
        self._d = {}

    def get(self, t, dev, dt, trans=False, pad8=False, taps=0):
        """t (2-D) cast to dt on dev; trans: its transpose, contiguous (the K-major filter
        operand of a backward-data GEMM); pad8: rows zero-padded to a multiple of 8 columns (a
        16-B aligned row pitch for the GEMM's LDS-DMA staging; the padding is never read as data).
        taps: the tap-major operand of the direct 3x3 convolution (conv3.hip) of an F x C*9
        filter -- 1: forward, F x 9 x C; 2: backward data, flipped and transposed, C x 9 x F."""
        import weakref
        k = (id(t), trans, pad8, taps)
        e = self._d.get(k)
        if e is not None and e[0]() is t and e[1] == t._version and e[2].device == dev and e[2].dtype == dt:
            return e[2]
        L = _lib
        if taps:
            F, CK = t.shape
            C = CK // 9
            src = t if (t.dtype == torch.float32 and t.is_contiguous() and t.device == dev) else \
                t.to(device=dev, dtype=torch.float32).contiguous()
            c = torch.empty(((F, 9 * C) if taps == 1 else (C, 9 * F)), dtype=torch.bfloat16, device=dev)
            rc = L.sysml_conv3_weight(src.data_ptr(), c.data_ptr(), F, C, int(taps == 2), _stream())
            if rc != 0:
                raise RuntimeError(f"sysml_conv3_weight failed: {rc}")
            counters["cast_weight"] = counters.get("cast_weight", 0) + 1
            pad8 = False
        elif dt == torch.bfloat16 and t.dtype == torch.float32 and t.is_cuda and t.device == dev and t.dim() == 2 \
                and t.is_contiguous() and L is not None:
            # one pass: cast, transpose and pad (gemm.hip cast_weight)
            M, K = t.shape
            C = M if trans else K
            cp = (C + 7) & ~7 if pad8 else C
            c = torch.empty(((K if trans else M), cp), dtype=dt, device=dev)
            rc = L.sysml_cast_weight(t.data_ptr(), c.data_ptr(), M, K, int(trans), cp, _stream())
            if rc != 0:
                raise RuntimeError(f"sysml_cast_weight failed: {rc}")
            counters["cast_weight"] = counters.get("cast_weight", 0) + 1
            pad8 = False
        else:
            c = t.to(device=dev, dtype=dt)
            c = (c.t() if trans else c).contiguous()
        if pad8 and c.shape[1] % 8:
            p = torch.zeros((c.shape[0], (c.shape[1] + 7) & ~7), dtype=c.dtype, device=c.device)
            p[:, :c.shape[1]] = c
            c = p
        dd = self._d
        ref = weakref.ref(t, lambda _r, k=k: dd.pop(k, None) if dd.get(k, (None,))[0] is _r else None)
        dd[k] = (ref, t._version, c)
        return c


_wcast = _WeightCasts()


def _conv_code(dt):
    if dt == torch.bfloat16:
        return 0
    if dt == torch.float32:
        return 3 if CONV_BF16_FP32 else 1
    if dt == torch.float64:
        return 2
    return None


GEMM_DNN_FILL = int(os.environ.get("SYSML_GEMM_DNN_FILL", "240"))   # workgroups that count as a full chip
GEMM_DNN_T128 = int(os.environ.get("SYSML_GEMM_DNN_T128", "0"))      # 128-row tiles below this many 256-row tiles


def _gemm_img(A, B, out, M, K, nimg, hw, hwb=None, bias=None, relu=False):
    """out[n] (M x hw, bf16) = A (M x K, bf16 K-major) . B[n] (K x hw) for every image n as ONE
    image-blocked GEMM launch (gemm.hip sysml_gemm_dnn); B's images are `hwb` pixels apart
    (hwb % 8 == 0; B is padded here when hw is not a multiple of 8), pixels past hw are padding.
    bias (M) and relu are applied in the epilogue."""
    L = load(required=True)
    dev = out.device
    st = _stream()
    if hwb is None:
        hwb = hw
        if hw % 8:
            hwb = (hw + 7) & ~7
            Bp = torch.empty((nimg * K * hwb,), dtype=torch.bfloat16, device=dev)
            rc = L.sysml_pad_pixels(B.data_ptr(), Bp.data_ptr(), nimg * K, hw, hwb, st)
            if rc != 0:
                raise RuntimeError(f"sysml_pad_pixels failed: {rc}")
            B = Bp
    Ncol = nimg * hwb
    # row tile: 64 rows for M <= 128 (a 256-row tile would be mostly padding), else 256; split K
    # only when fewer than half the CUs would get a workgroup
    # (measured, tools/bench_gemm_dnn.py: a 256-row tile on 200 workgroups beats the 64-row tile
    # on 800 for deep K -- the 64-row tile is LDS-bound)
    nt = (Ncol + 255) // 256
    te = 64 if M <= 128 else 256
    if te == 256 and GEMM_DNN_T128 and ((M + 255) // 256) * nt < GEMM_DNN_T128:
        te = 128                      # 256-row tiles would leave CUs idle: twice the workgroups
    tiles = ((M + te - 1) // te) * nt
    ksplit = 1
    if tiles < GEMM_DNN_FILL // 2 and K >= 1024:
        ksplit = max(1, min((GEMM_DNN_FILL + tiles - 1) // tiles, K // 512, 4))
    slab = torch.empty((ksplit * M * Ncol,), dtype=torch.float32, device=dev) if ksplit > 1 else None
    bb = None
    if bias is not None:
        bb = bias.to(device=dev, dtype=torch.float32).reshape(-1).contiguous()
    rc = L.sysml_gemm_dnn(A.data_ptr(), A.stride(0), B.data_ptr(), hwb, K * hwb, out.data_ptr(), hw, M * hw,
                          M, Ncol, K, hwb, hw, bb.data_ptr() if bb is not None else None, int(bool(relu)), 1,
                          ksplit, slab.data_ptr() if slab is not None else None, te, st)
    if rc != 0:
        raise RuntimeError(f"sysml_gemm_dnn failed: {rc}")
    _count("gemm_dnn")
    return out


def _bias_epilogue(y, bias, relu, F, dev):
    """bias_add (+ relu) over a convolution result.  bias_op writes into `out` only on its bf16
    fast path; otherwise it returns a new fp32 tensor, which is taken (cast back to y's dtype)
    instead of silently keeping the un-biased y."""
    bb = bias if bias is not None else torch.zeros(F, device=dev)
    r = bias_op(y, bb, relu=relu, out=y)
    if r is None:
        raise RuntimeError(f"conv2d bias epilogue: {bb.numel()} channels do not divide a row of {y.shape[1]}")
    return r if r is y else r.to(y.dtype)


def conv2d(mode, X, W, D, N, C, H, Wd, F, KH, KW, sh, sw, ph, pw, bias=None, relu=False):
    """Implicit-GEMM convolution (mode 0 forward, 1 backward data, 2 backward filter).  X / W /
    D are the DML 2-D matrices (NCHW rows); returns the DML 2-D result.  bf16 operands compute
    on bf16 MFMA with an fp32 result; fp32 / fp64 on exact MFMA."""
    L = load(required=True)
    ref = X if X is not None else D
    dt = ref.dtype
    code = _conv_code(dt)
    if code is None:
        return None
    odt = torch.float32 if dt == torch.bfloat16 else dt
    dev = ref.device

    def prep(t):
        return None if t is None else t.to(device=dev, dtype=dt).contiguous()
    X, D = prep(X), prep(D)
    W0 = W
    W = _wcast.get(W, dev, dt) if W is not None and W.dtype != dt and dt == torch.bfloat16 else prep(W)
    Ho = (H + 2 * ph - KH) // sh + 1
    Wo = (Wd + 2 * pw - KW) // sw + 1
    if mode == 0:
        shape = (N, F * Ho * Wo)
    elif mode == 1:
        shape = (N, C * H * Wd)
    else:
        shape = (F, C * KH * KW)
    Wsrc = W0 if W0 is not None else W         # the filter as given (cache key of its transposed bf16 copy)
    if CONV1X1_GEMM and mode == 2 and KH == 1 and KW == 1 and sh == 1 and sw == 1 and ph == 0 and pw == 0 \
            and dt == torch.bfloat16:
        # 1x1 stride-1 filter gradient: dW = sum_img dout[img] . t(X[img]) as one batched NT GEMM
        # (wgrad.hip: 16-B pixel-vector loads, images as the split-K axis, slab reduction)
        HW = H * Wd
        S = L.sysml_wgrad_splits(F, C, HW, N)
        slab = torch.empty((S * F * C,), dtype=torch.float32, device=dev) if S > 1 else None
        y = torch.empty((F, C), dtype=torch.float32, device=dev)
        rc = L.sysml_wgrad_nt(D.data_ptr(), X.data_ptr(), y.data_ptr(), _ptr(slab), F, C, HW, N, F * HW, C * HW,
                              _stream())
        if rc != 0:
            raise RuntimeError(f"sysml_wgrad_nt failed: {rc}")
        _count("conv2d_bwd_filter")
        _count("wgrad_1x1")
        return y
    if WGRAD3 and mode == 2 and KH == 3 and KW == 3 and sh == 1 and sw == 1 and ph == 1 and pw == 1 \
            and dt == torch.bfloat16 and Wd <= 64:
        # 3x3 stride-1 filter gradient (wgrad.hip: 8-pixel runs of padded rows, the input patch as
        # three column-shifted LDS copies, chunks split over blocks with a slab reduction)
        S = L.sysml_wgrad3_splits(N, C, H, Wd, F)
        if S >= 1:
            slab = torch.empty((S * F * C * 9,), dtype=torch.float32, device=dev) if S > 1 else None
            y = torch.empty((F, C * 9), dtype=torch.float32, device=dev)
            rc = L.sysml_wgrad3(X.data_ptr(), D.data_ptr(), y.data_ptr(), _ptr(slab), N, C, H, Wd, F, _stream())
            if rc == 0:
                _count("conv2d_bwd_filter")
                _count("wgrad_3x3")
                return y
            if rc != -1:
                raise RuntimeError(f"sysml_wgrad3 failed: {rc}")
    if CONV3_DIRECT and mode != 2 and KH == 3 and KW == 3 and sh == 1 and sw == 1 and ph == 1 and pw == 1 \
            and dt == torch.bfloat16 and (C if mode == 0 else F) % 32 == 0 \
            and 0 < backend.act_bf16_min_cells <= shape[0] * shape[1]:
        # 3x3 stride-1 layers: the direct convolution of conv3.hip (input patch staged in LDS once
        # per 32 channels, the nine taps as LDS offsets); backward data is the forward convolution
        # of dout with the flipped, transposed filter
        y = torch.empty(shape, dtype=torch.bfloat16, device=dev)
        inp, Cin, M = (X, C, F) if mode == 0 else (D, F, C)
        A = _wcast.get(Wsrc, dev, dt, taps=1 + mode)
        bb = None
        if mode == 0 and bias is not None:
            bb = bias.to(device=dev, dtype=torch.float32).reshape(-1).contiguous()
        rc = L.sysml_conv3s1(inp.data_ptr(), A.data_ptr(), _ptr(bb), y.data_ptr(), 0, N, Cin, H, Wd, M,
                             int(bool(relu and mode == 0)), _stream())
        if rc == 0:
            _count(("conv2d", "conv2d_bwd_data")[mode])
            _count("conv3_direct")
            return y
        if rc != -1:
            raise RuntimeError(f"sysml_conv3s1 failed: {rc}")
    if CONV1X1_GEMM and mode != 2 and KH == 1 and KW == 1 and sh == 1 and sw == 1 and ph == 0 and pw == 0 \
            and dt == torch.bfloat16 and 0 < backend.act_bf16_min_cells <= shape[0] * shape[1]:
        # a 1x1 stride-1 convolution of bf16 activations is ONE GEMM over all images (gemm.hip
        # image-blocked columns): forward W . X[n], backward data t(W) . dY[n]; bias + relu in
        # the epilogue, bf16 out / fp32 accumulate
        HW = H * Wd
        y = torch.empty(shape, dtype=torch.bfloat16, device=dev)
        if mode == 0:
            _gemm_img(_wcast.get(Wsrc, dev, dt, pad8=True), X, y, F, C, N, HW, bias=bias, relu=relu)
        else:
            _gemm_img(_wcast.get(Wsrc, dev, dt, trans=True, pad8=True), D, y, C, F, N, HW)
        _count(("conv2d", "conv2d_bwd_data")[mode])
        _count("conv1x1_gemm")
        return y
    if CONV1X1_GEMM and mode == 0 and KH * KW > 1 and Ho * Wo <= IM2COL_MAX_HW and C > 8 \
            and dt == torch.bfloat16 and 0 < backend.act_bf16_min_cells <= shape[0] * shape[1]:
        # small-image convolutions: an im2col gather (pixels padded to a multiple of 8) and ONE
        # image-blocked GEMM over all images
        CKK, P = C * KH * KW, Ho * Wo
        Pp = (P + 7) & ~7
        cols = torch.empty((N, CKK, Pp), dtype=torch.bfloat16, device=dev)
        L.sysml_im2col_pad.restype = ctypes.c_int
        L.sysml_im2col_pad.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int] * 11 + \
            [ctypes.c_void_p]
        rc = L.sysml_im2col_pad(3, X.data_ptr(), cols.data_ptr(), N, C, H, Wd, KH, KW, sh, sw, ph, pw, Pp, _stream())
        if rc != 0:
            raise RuntimeError(f"sysml_im2col failed: {rc}")
        y = torch.empty(shape, dtype=torch.bfloat16, device=dev)
        _gemm_img(_wcast.get(Wsrc, dev, dt, pad8=True), cols, y, F, CKK, N, P, hwb=Pp, bias=bias, relu=relu)
        _count("conv2d")
        _count("conv_im2col")
        return y
    if CONV1X1_GEMM and mode == 1 and (sh > 1 or sw > 1 or (KH > 1 and H * Wd <= COL2IM_MAX_HW)) \
            and dt == torch.bfloat16 and 0 < backend.act_bf16_min_cells <= shape[0] * shape[1]:
        # backward data as cols = t(W) . dY[n] (one image-blocked GEMM, bf16) + a col2im gather:
        # a strided convolution's taps land on the stride grid for a quarter of the (pixel, tap)
        # pairs, which the implicit GEMM would multiply as zeros
        CKK, P = C * KH * KW, Ho * Wo
        cols = torch.empty((N, CKK, P), dtype=torch.bfloat16, device=dev)
        _gemm_img(_wcast.get(Wsrc, dev, dt, trans=True, pad8=True), D, cols, CKK, F, N, P)
        y = torch.empty(shape, dtype=torch.bfloat16, device=dev)
        L.sysml_col2im.restype = ctypes.c_int
        L.sysml_col2im.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int] * 10 + \
            [ctypes.c_void_p]
        rc = L.sysml_col2im(3, cols.data_ptr(), y.data_ptr(), N, C, H, Wd, KH, KW, sh, sw, ph, pw, _stream())
        if rc != 0:
            raise RuntimeError(f"sysml_col2im failed: {rc}")
        _count("conv2d_bwd_data")
        _count("conv_col2im")
        return y
    # GEMM view (M x Ncol, depth K); split K when the output tiles alone cannot fill the chip:
    # ~2k blocks in flight, each reducing >= CONV_SPLIT_MINK products per output (slab traffic stays small)
    M, Nc, K = {0: (F, N * Ho * Wo, C * KH * KW), 1: (C, N * H * Wd, F * KH * KW),
                2: (F, C * KH * KW, N * Ho * Wo)}[mode]
    L.sysml_conv2d_tile_mode.restype = ctypes.c_int
    L.sysml_conv2d_tile_mode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64]
    te = L.sysml_conv2d_tile_mode(code, mode, M, Nc)   # the launcher's output tile edge
    tiles = ((M + te - 1) // te) * ((Nc + te - 1) // te)
    ksplit = 1
    if tiles < CONV_SPLIT_BLOCKS:
        ksplit = max(1, min(256, CONV_SPLIT_BLOCKS // max(tiles, 1), K // CONV_SPLIT_MINK))
    bdt = odt
    if code == 0 and mode != 2 and ksplit == 1 and not (mode == 1 and C <= 8) and \
            0 < backend.act_bf16_min_cells <= shape[0] * shape[1]:
        code, odt = 4, torch.bfloat16              # bf16 activations: the output is stored bf16
    out = torch.empty(shape, dtype=odt, device=dev)
    ws = None
    if mode == 2 and ksplit > 1 and CONV_SLAB and ksplit * M * Nc * out.element_size() <= (256 << 20):
        # deterministic split-K: per-split slices summed in a fixed order (no fp32 atomics)
        ws = torch.empty((ksplit * M * Nc,), dtype=odt, device=dev)
    b = None if bias is None else bias.to(device=dev, dtype=bdt).contiguous().reshape(-1)
    rc = L.sysml_conv2d(code, mode, _ptr(X), _ptr(W), _ptr(D), _ptr(b), out.data_ptr(), _ptr(ws), ksplit,
                        N, C, H, Wd, F, KH, KW, sh, sw, ph, pw, int(bool(relu)), _stream())
    if rc == -1:
        return None
    if rc != 0:
        raise RuntimeError(f"sysml_conv2d failed: {rc}")
    _count(("conv2d", "conv2d_bwd_data", "conv2d_bwd_filter")[mode])
    return out


def _ptr(t):
    return None if t is None else t.data_ptr()


def pool2d(backward, avg, X, D, N, C, H, W, KH, KW, sh, sw, ph, pw):
    L = load(required=True)
    dt = X.dtype if X.dtype in (torch.float32, torch.float64) else torch.float32
    if X.dtype == torch.bfloat16 and backend.act_bf16_min_cells > 0:
        dt = torch.bfloat16                        # bf16 activations stay bf16 (fp32 math)
    code = {torch.float32: 1, torch.float64: 2, torch.bfloat16: 3}[dt]
    X = X.to(dt).contiguous()
    D = None if D is None else D.to(device=X.device, dtype=dt).contiguous()
    Ho = (H + 2 * ph - KH) // sh + 1
    Wo = (W + 2 * pw - KW) // sw + 1
    out = torch.empty((N, C * (H * W if backward else Ho * Wo)), dtype=dt, device=X.device)
    # max-pooling backward: window argmax positions (one byte per window) found in a first pass
    ws = torch.empty((N * C * Ho * Wo,), dtype=torch.uint8, device=X.device) \
        if backward and not avg and KH * KW <= 255 else None
    rc = L.sysml_pool2d_ws(code, int(bool(backward)), int(bool(avg)), X.data_ptr(), _ptr(D), out.data_ptr(),
                           _ptr(ws), N, C, H, W, KH, KW, sh, sw, ph, pw, _stream())
    if rc == -1:
        return None
    if rc != 0:
        raise RuntimeError(f"sysml_pool2d failed: {rc}")
    _count("pool_bwd" if backward else "pool")
    return out


def bias_op(X, b, mult=False, relu=False, out=None):
    L = load(required=True)
    if X.dtype == torch.bfloat16 and backend.act_bf16_min_cells > 0 and X.numel() % 4 == 0 and X.is_contiguous():
        # bf16 activations stay bf16 (fp32 bias and arithmetic); out may alias X
        bf = b.to(device=X.device, dtype=torch.float32).contiguous().reshape(-1)
        C = bf.numel()
        if X.shape[1] % C == 0:
            o = torch.empty_like(X) if out is None else out
            rc = L.sysml_bias_op(3, X.data_ptr(), bf.data_ptr(), o.data_ptr(), X.numel(), C, X.shape[1] // C,
                                 int(bool(mult)), int(bool(relu)), _stream())
            if rc == 0:
                _count("bias_mult" if mult else "bias_add")
                return o
            if rc != -1:
                raise RuntimeError(f"sysml_bias_op failed: {rc}")
    dt = X.dtype if X.dtype in (torch.float32, torch.float64) else torch.float32
    X = X.to(dt).contiguous()
    b = b.to(device=X.device, dtype=dt).contiguous().reshape(-1)
    C = b.numel()
    if X.shape[1] % C:
        return None
    out = torch.empty_like(X)
    rc = L.sysml_bias_op(1 if dt == torch.float32 else 2, X.data_ptr(), b.data_ptr(), out.data_ptr(), X.numel(),
                         C, X.shape[1] // C, int(bool(mult)), int(bool(relu)), _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_bias_op failed: {rc}")
    _count("bias_mult" if mult else "bias_add")
    return out


def relu_backward(X, D):
    L = load(required=True)
    dt = torch.promote_types(X.dtype, D.dtype)
    if dt not in (torch.float32, torch.float64):
        dt = torch.float32
    X = X.to(dt).contiguous()
    D = D.to(device=X.device, dtype=dt).contiguous()
    out = torch.empty_like(X)
    rc = L.sysml_relu_backward(1 if dt == torch.float32 else 2, X.data_ptr(), D.data_ptr(), out.data_ptr(),
                               X.numel(), _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_relu_backward failed: {rc}")
    _count("relu_backward")
    return out


# ----------------------------------------------------------------------------
# Column-wise cumulative aggregates (ops/hip/scan.hip)
# ----------------------------------------------------------------------------
_CUM = {"cumsum": 0, "cumprod": 1, "cummin": 2, "cummax": 3}


_AGG_OPS = {"sum": 0, "sumsq": 1, "mean": 2, "min": 3, "max": 4, "prod": 5, "var": 6, "sd": 7, "imax": 8, "imin": 9}
_AGG_DIR = {"all": 0, "row": 1, "col": 2}
_AGG_XDT = {torch.bfloat16: 0, torch.float32: 1, torch.float64: 2}


def agg(o, d, X, ydt=None):
    """Unary aggregate of a dense device matrix on ops/hip/agg.hip (fp64 accumulation, bf16 /
    fp32 / fp64 read as stored).  d = 'all' -> 0-d fp64 tensor; 'row' -> N x 1; 'col' -> 1 x D
    (stored as `ydt` when given, fp32 or fp64).  None when the operator / layout is not covered."""
    op, dr, xdt = _AGG_OPS.get(o), _AGG_DIR.get(d), _AGG_XDT.get(X.dtype)
    if op is None or dr is None or xdt is None or X.dim() != 2 or (op >= 8 and dr != 1):
        return None
    L = load(required=True)
    N, D = X.shape
    if N == 0 or D == 0:
        return None
    X = _dense(X)
    if ydt is None:
        ydt = torch.float64 if (X.dtype == torch.float64 or (X.dtype == torch.bfloat16
                                                             and backend.dtype == torch.float64)) else torch.float32
    if dr == 0:
        Y = torch.empty((), dtype=torch.float64, device=X.device)
    elif dr == 1:
        Y = torch.empty((N, 1), dtype=ydt, device=X.device)
    else:
        Y = torch.empty((1, D), dtype=ydt, device=X.device)
    nscr = L.sysml_agg_scratch(dr, N, D)
    scr = torch.empty((max(nscr, 8),), dtype=torch.uint8, device=X.device)
    rc = L.sysml_agg(op, dr, xdt, 2 if (dr == 0 or ydt == torch.float64) else 1, X.data_ptr(), Y.data_ptr(),
                     scr.data_ptr(), N, D, _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_agg failed: {rc}")
    _count("agg." + o)
    return Y


_ESIZE = {torch.bfloat16: 2, torch.float32: 4, torch.float64: 8}


def csr_transpose_plan(crow, col, m, n):
    """Transposed pattern of an m x n CSR pattern by counting sort (csrt.hip): (crowT int64,
    colT int64, perm int64) with colT sorted inside every row of t(A) -- the arrays a stable key
    sort gives.  The int32 copy of colT the kernels read is registered with idx32_of.  None when
    a column is longer than the in-LDS segment sort handles."""
    L = load(required=True)
    nnz = col.numel()
    dev = col.device
    idx32 = int(col.dtype == torch.int32)
    colc = col.contiguous() if idx32 else col.to(torch.int64).contiguous()
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    mx = torch.zeros(1, dtype=torch.int32, device=dev)
    rc = L.sysml_csrt_count(colc.data_ptr(), idx32, nnz, cnt.data_ptr(), mx.data_ptr(), _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_csrt_count failed: {rc}")
    if int(mx.item()) > 0:
        return None
    crowT = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(cnt, 0, dtype=torch.int64, out=crowT[1:])
    cursor = torch.zeros(n, dtype=torch.int32, device=dev)
    rows32 = torch.empty(nnz, dtype=torch.int32, device=dev)
    perm = torch.empty(nnz, dtype=torch.int64, device=dev)
    rc = L.sysml_csrt_fill(crow.to(torch.int64).contiguous().data_ptr(), colc.data_ptr(), idx32, m, n,
                           crowT.data_ptr(), cursor.data_ptr(), rows32.data_ptr(), perm.data_ptr(), _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_csrt_fill failed: {rc}")
    colT = rows32.to(torch.int64)
    if len(_IDX32) >= 8:
        _IDX32.pop(next(iter(_IDX32), None), None)
    _IDX32[(colT.data_ptr(), colT.numel(), colT._version)] = (colT, rows32)
    _count("csr_transpose")
    return crowT, colT, perm


def gather(v, perm):
    """v[perm] for a 1-D device tensor and an int64 index vector (csrt.hip gather)."""
    es = v.element_size()
    if es not in (2, 4, 8) or not v.is_cuda or perm.dtype != torch.int64:
        return v[perm]
    L = load(required=True)
    v = v.contiguous()
    out = torch.empty(perm.numel(), dtype=v.dtype, device=v.device)
    rc = L.sysml_gather(es, v.data_ptr(), perm.contiguous().data_ptr(), out.data_ptr(), perm.numel(), _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_gather failed: {rc}")
    return out


def fold_rows(part, op="sum", ydt=torch.float32):
    """1 x n column result of an nb x n fp64 block of row-block partials (sum / min / max),
    stored as ydt (fp32 / fp64): one agg.hip pass (fold_rows)."""
    code = {"sum": 0, "min": 3, "max": 4}.get(op)
    if code is None or part.dtype != torch.float64 or not part.is_cuda or ydt not in (torch.float32, torch.float64):
        return None
    L = load(required=True)
    part = part.contiguous()
    nb, n = part.shape[0], part[0].numel()
    y = torch.empty((1, n), dtype=ydt, device=part.device)
    rc = L.sysml_fold_rows(code, 1 if ydt == torch.float32 else 2, part.data_ptr(), y.data_ptr(), nb, n, _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_fold_rows failed: {rc}")
    return y


def dot(A, B):
    """sum(A * B) of two same-shaped dense device matrices as a 0-d fp64 device tensor
    (agg.hip dot_part, fp64 accumulation; one pass, no product materialised); None when the
    dtypes differ or are not covered."""
    code = _AGG_XDT.get(A.dtype)
    if code is None or B.dtype != A.dtype or A.shape != B.shape or not A.is_cuda or A.device != B.device:
        return None
    L = load(required=True)
    n = A.numel()
    if n == 0:
        return None
    A, B = A.contiguous(), B.contiguous()
    y = torch.empty((), dtype=torch.float64, device=A.device)
    scr = torch.empty((L.sysml_agg_scratch(0, n, 1),), dtype=torch.uint8, device=A.device)
    rc = L.sysml_dot(code, A.data_ptr(), B.data_ptr(), y.data_ptr(), scr.data_ptr(), n, _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_dot failed: {rc}")
    _count("dot")
    return y


def cat(rows, mats):
    """cbind (rows=False) / rbind (rows=True) of dense device matrices of one dtype in one pass
    (ops/hip/reorg.hip); None when not covered (mixed dtypes / devices, > 16 operands)."""
    if not mats or len(mats) > 16:
        return None
    dt, dev = mats[0].dtype, mats[0].device
    if dt not in _ESIZE or any(m.dtype != dt or m.device != dev or not m.is_cuda or m.dim() != 2
                               or m.layout != torch.strided for m in mats):
        return None
    L = load(required=True)
    mats = [m.contiguous() for m in mats]
    if rows:
        N, D = sum(m.shape[0] for m in mats), mats[0].shape[1]
        sizes = [m.shape[0] for m in mats]
    else:
        N, D = mats[0].shape[0], sum(m.shape[1] for m in mats)
        sizes = [m.shape[1] for m in mats]
    out = torch.empty((N, D), dtype=dt, device=dev)
    if N == 0 or D == 0:
        return out
    keep = [m for m in mats if m.numel() > 0]
    n = len(keep)
    srcs = (ctypes.c_void_p * n)(*[m.data_ptr() for m in keep])
    offs, acc = [], 0
    for m in keep:
        offs.append(acc)
        acc += m.shape[0] if rows else m.shape[1]
    offs.append(acc)
    off = (ctypes.c_int64 * (n + 1))(*offs)
    ld = (ctypes.c_int64 * n)(*[m.shape[1] for m in keep])
    del sizes
    rc = L.sysml_cat(int(bool(rows)), _ESIZE[dt], n, srcs, off, ld, out.data_ptr(), N, D, _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_cat failed: {rc}")
    _count("rbind" if rows else "cbind")
    return out


def lix(X, Y, out, r0, r1, c0, c1, sdev=None):
    """out = X with out[r0:r1, c0:c1] = Y (0-based, half-open; Y a wr x wc tensor or a Python
    number; sdev instead: a device fp64 scalar read by the kernel) in one pass; out may be X
    itself (only the window is written).  False when not covered."""
    if X.dtype not in _ESIZE or not X.is_cuda or X.dim() != 2 or not X.is_contiguous() or out.dtype != X.dtype \
            or not out.is_contiguous():
        return False
    L = load(required=True)
    import struct
    scalar = not isinstance(Y, torch.Tensor)
    sbits = 0
    yp = None
    sp = None
    if sdev is not None:
        if not sdev.is_cuda or sdev.device != X.device:
            return False
        sd = sdev.reshape(1)
        if sd.dtype != torch.float64:
            sd = sd.double()
        sp = sd.data_ptr()
    elif scalar:
        v = float(Y)
        if X.dtype == torch.float64:
            sbits = struct.unpack("<Q", struct.pack("<d", v))[0]
        elif X.dtype == torch.float32:
            sbits = struct.unpack("<I", struct.pack("<f", v))[0]
        else:
            sbits = int(torch.tensor([v], dtype=torch.bfloat16).view(torch.int16).item()) & 0xFFFF
    else:
        Y = Y.to(device=X.device, dtype=X.dtype).contiguous()
        yp = Y.data_ptr()
    rc = L.sysml_lix2(_ESIZE[X.dtype], X.data_ptr(), yp, out.data_ptr(), X.shape[0], X.shape[1], r0, r1, c0, c1,
                      int(scalar), sbits, sp, _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_lix failed: {rc}")
    _count("lix")
    return True


def cumagg(op, X):
    """cumsum / cumprod / cummin / cummax down the rows of a device matrix (three-phase chunked
    scan).  bf16 inputs scan in fp32."""
    L = load(required=True)
    if X.dtype not in (torch.float32, torch.float64):
        X = X.float()
    X = X.contiguous()
    N, D = X.shape
    out = torch.empty_like(X)
    if N == 0 or D == 0:
        return out
    rows = ctypes.c_int64(0)
    nchunk = L.sysml_cumagg_chunks(N, D, ctypes.byref(rows))
    tot = torch.empty((nchunk, D), dtype=X.dtype, device=X.device)
    rc = L.sysml_cumagg(0 if X.dtype == torch.float32 else 1, _CUM[op], X.data_ptr(), out.data_ptr(),
                        tot.data_ptr(), N, D, nchunk, rows.value, _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_cumagg failed: {rc}")
    _count(op)
    return out


# ----------------------------------------------------------------------------
# CSR sparse x dense (ops/hip/spmm.hip)
# ----------------------------------------------------------------------------
_IDX32 = {}


def csr_idx32(A):
    """int32 copy of a CSR matrix's column indices (half the index bytes of every sparse
    product), cached per pattern; None when the matrix has >= 2^31 columns."""
    col = A.col_indices()
    if A.shape[1] >= 2 ** 31:
        return None
    if col.dtype == torch.int32:
        return col.contiguous()
    return idx32_of(col)


def idx32_of(col):
    """int32 copy of an int64 index tensor, cached by storage address, length and version.
    The cache holds the original tensor, so its storage (the key's address) cannot be
    recycled for another tensor while the entry lives."""
    if col.dtype == torch.int32:
        return col.contiguous()
    key = (col.data_ptr(), col.numel(), col._version)
    e = _IDX32.get(key)
    if e is None:
        if len(_IDX32) >= 8:
            _IDX32.pop(next(iter(_IDX32), None), None)   # tolerant of a concurrent parfor worker's eviction
        e = (col, col.to(torch.int32).contiguous())
        _IDX32[key] = e
    return e[1]


def spmm_bal(A, B):
    """C = A %*% B for CSR A and dense B on the nnz-balanced kernel (int32 column indices,
    skew-tolerant: ops/hip/spgemm.hip); None if unsupported."""
    L = load(required=True)
    if A.layout != torch.sparse_csr or B.dim() != 2 or B.shape[0] != A.shape[1]:
        return None
    dt = torch.promote_types(A.dtype, B.dtype)
    if dt not in (torch.float32, torch.float64):
        dt = torch.float32
    m, n = A.shape
    K = B.shape[1]
    crow = A.crow_indices().to(torch.int64).contiguous()
    c32 = csr_idx32(A)
    col = c32 if c32 is not None else A.col_indices().to(torch.int64).contiguous()
    val = A.values().to(dt).contiguous()
    B = B.to(device=val.device, dtype=dt).contiguous()
    C = torch.zeros((m, K), dtype=dt, device=val.device)
    nnz = int(val.numel())
    rc = L.sysml_spmm_bal(1 if dt == torch.float32 else 2, int(c32 is not None), crow.data_ptr(), col.data_ptr(),
                          val.data_ptr(), B.data_ptr(), K, C.data_ptr(), K, m, K, nnz, _stream())
    if rc == -1:
        return None
    if rc != 0:
        raise RuntimeError(f"sysml_spmm_bal failed: {rc}")
    _count("spmm_bal")
    return C


SPGEMM_MAXN = 32768


def spgemm(A, B):
    """C = A %*% B for two CSR matrices (fp32, n = ncol(B) <= 32768): Gustavson rows with an LDS
    dense accumulator, count pass + fill pass; canonical CSR result.  None if unsupported."""
    L = load(required=True)
    if A.layout != torch.sparse_csr or B.layout != torch.sparse_csr or A.shape[1] != B.shape[0]:
        return None
    m, n = A.shape[0], B.shape[1]
    if n > SPGEMM_MAXN or n < 1 or m < 1:
        return None
    if torch.float64 in (A.values().dtype, B.values().dtype, backend.dtype):
        return None          # the LDS accumulator is fp32: double-precision products keep the fp64 path
    dev = A.values().device
    ac, bc = A.crow_indices().to(torch.int64).contiguous(), B.crow_indices().to(torch.int64).contiguous()
    a32, b32 = csr_idx32(A), csr_idx32(B)
    acol = a32 if a32 is not None else A.col_indices().to(torch.int64).contiguous()
    bcol = b32 if b32 is not None else B.col_indices().to(torch.int64).contiguous()
    av = A.values().to(torch.float32).contiguous()
    bv = B.values().to(device=dev, dtype=torch.float32).contiguous()
    cnt = torch.empty(m, dtype=torch.int64, device=dev)
    st = _stream()
    rc = L.sysml_spgemm_count(int(a32 is not None), int(b32 is not None), ac.data_ptr(), acol.data_ptr(),
                              bc.data_ptr(), bcol.data_ptr(), m, n, cnt.data_ptr(), st)
    if rc != 0:
        return None
    ccrow = torch.zeros(m + 1, dtype=torch.int64, device=dev)
    ccrow[1:] = torch.cumsum(cnt, 0)
    nnz = int(ccrow[-1].item())
    ccol = torch.empty(max(nnz, 1), dtype=torch.int64, device=dev)
    cval = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
    fcnt = torch.empty(m, dtype=torch.int64, device=dev)
    rc = L.sysml_spgemm_fill(int(a32 is not None), int(b32 is not None), ac.data_ptr(), acol.data_ptr(),
                             av.data_ptr(), bc.data_ptr(), bcol.data_ptr(), bv.data_ptr(), m, n, ccrow.data_ptr(),
                             ccol.data_ptr(), cval.data_ptr(), fcnt.data_ptr(), _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_spgemm_fill failed: {rc}")
    if not torch.equal(fcnt, cnt):
        raise RuntimeError("sysml_spgemm: fill pass disagrees with the count pass")
    _count("spgemm")
    return torch.sparse_csr_tensor(ccrow, ccol[:nnz], cval[:nnz], (m, n), device=dev)


TSMM_SP_MAXD = 8192


def tsmm_sparse(X):
    """t(X) %*% X for CSR X (D = ncol <= 8192) as a dense D x D matrix: pair products of
    every row's non-zeros scattered into the upper triangle, then mirrored."""
    L = load(required=True)
    if X.layout != torch.sparse_csr:
        return None
    m, D = X.shape
    if D > TSMM_SP_MAXD or D < 1:
        return None
    dt = X.dtype if X.dtype in (torch.float32, torch.float64) else torch.float32
    crow = X.crow_indices().to(torch.int64).contiguous()
    c32 = csr_idx32(X)
    col = c32 if c32 is not None else X.col_indices().to(torch.int64).contiguous()
    val = X.values().to(dt).contiguous()
    C = torch.zeros((D, D), dtype=dt, device=val.device)
    rc = L.sysml_tsmm_sparse(1 if dt == torch.float32 else 2, int(c32 is not None), crow.data_ptr(), col.data_ptr(),
                             val.data_ptr(), m, C.data_ptr(), D, _stream())
    if rc != 0:
        return None
    _count("tsmm_sparse")
    return C


def spmm(A, B, transA=False):
    """A (CSR, m x n) %*% B (dense n x K), or t(A) %*% B (B: m x K) without transposing A.
    Computed in the wider of the two dtypes (fp32 / fp64); None if unsupported."""
    L = load(required=True)
    if A.layout != torch.sparse_csr or B.dim() != 2:
        return None
    dt = torch.promote_types(A.dtype, B.dtype)
    if dt not in (torch.float32, torch.float64):
        dt = torch.float32
    m, n = A.shape
    K = B.shape[1]
    if B.shape[0] != (m if transA else n):
        return None
    crow = A.crow_indices().to(torch.int64).contiguous()
    col = A.col_indices().to(torch.int64).contiguous()
    val = A.values().to(dt).contiguous()
    B = B.to(device=val.device, dtype=dt).contiguous()
    if transA:
        C = torch.zeros((n, K), dtype=dt, device=val.device)
    else:
        C = torch.empty((m, K), dtype=dt, device=val.device)
    rc = L.sysml_spmm(1 if dt == torch.float32 else 2, int(bool(transA)), crow.data_ptr(), col.data_ptr(),
                      val.data_ptr(), B.data_ptr(), K, C.data_ptr(), K, m, K, _stream())
    if rc == -1:
        return None
    if rc != 0:
        raise RuntimeError(f"sysml_spmm failed: {rc}")
    _count("spmm_t" if transA else "spmm")
    return C


# ----------------------------------------------------------------------------
# right indexing / transpose / tri / row gathers / sort (ops/hip/reorg.hip, ops/hip/sort.hip)
# ----------------------------------------------------------------------------
_TCODE = {torch.bfloat16: 0, torch.float32: 1, torch.float64: 2}


def _rowpitch(x):
    """Row pitch of a 2-D view whose rows are unit-stride (a slice of a row-major matrix), else
    None."""
    if x.dim() != 2 or x.layout != torch.strided:
        return None
    r, c = x.shape
    if c == 1 or x.stride(1) == 1:
        ld = x.stride(0) if r > 1 else c
        return ld if ld >= c else None
    return None


def copy2d(x, dtype=None):
    """Dense row-major copy of a 2-D device view x (a right-indexing window, any row pitch),
    converted to `dtype` in the same pass; None when not covered (not a row-major view)."""
    dtype = dtype or x.dtype
    if not x.is_cuda or x.dtype not in _TCODE or dtype not in _TCODE:
        return None
    ld = _rowpitch(x)
    if ld is None:
        return None
    L = load(required=True)
    nr, nc = x.shape
    out = torch.empty((nr, nc), dtype=dtype, device=x.device)
    if out.numel() == 0:
        return out
    rc = L.sysml_copy2d(_TCODE[x.dtype], _TCODE[dtype], x.data_ptr(), ld, out.data_ptr(), nc, nr, nc, _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_copy2d failed: {rc}")
    _count("slice" if dtype == x.dtype else "cast")
    return out


def transpose(x):
    """t(x) of a 2-D device matrix (row-major, any row pitch) as a dense matrix (LDS-tiled);
    None when not covered."""
    if not x.is_cuda or x.dtype not in _ESIZE:
        return None
    ld = _rowpitch(x)
    if ld is None:
        return None
    L = load(required=True)
    N, D = x.shape
    out = torch.empty((D, N), dtype=x.dtype, device=x.device)
    if out.numel() == 0:
        return out
    rc = L.sysml_transpose(_ESIZE[x.dtype], x.data_ptr(), ld, out.data_ptr(), N, D, _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_transpose failed: {rc}")
    _count("transpose")
    return out


def tri(x, lower, diag, values):
    """lower.tri / upper.tri of a dense device matrix in one pass; None when not covered."""
    if not x.is_cuda or x.dtype not in _ESIZE or x.dim() != 2 or x.layout != torch.strided:
        return None
    L = load(required=True)
    x = x.contiguous()
    out = torch.empty_like(x)
    if x.numel():
        rc = L.sysml_tri(_ESIZE[x.dtype], x.data_ptr(), out.data_ptr(), x.shape[0], x.shape[1], int(bool(lower)),
                         int(bool(diag)), int(bool(values)), _stream())
        if rc != 0:
            raise RuntimeError(f"sysml_tri failed: {rc}")
    _count("tri")
    return out


def gather_rows(x, idx):
    """x[idx, ] for a 0-based int32 / int64 device index vector; None when not covered."""
    if not x.is_cuda or x.dtype not in _ESIZE or idx.dtype not in (torch.int32, torch.int64) or not idx.is_cuda:
        return None
    ld = _rowpitch(x)
    if ld is None:
        return None
    L = load(required=True)
    idx = idx.reshape(-1).contiguous()
    n, D = idx.numel(), x.shape[1]
    out = torch.empty((n, D), dtype=x.dtype, device=x.device)
    if out.numel():
        rc = L.sysml_gather_rows(_ESIZE[x.dtype], int(idx.dtype == torch.int64), x.data_ptr(), ld, idx.data_ptr(),
                                 out.data_ptr(), n, D, _stream())
        if rc != 0:
            raise RuntimeError(f"sysml_gather_rows failed: {rc}")
    _count("gather_rows")
    return out


def slice_csr(x, r0, r1, c0, c1):
    """Dense window x[r0:r1, c0:c1] (0-based, half-open) of a device CSR matrix; None when not
    covered."""
    if not x.is_cuda or x.layout != torch.sparse_csr or x.dtype not in (torch.float32, torch.float64):
        return None
    L = load(required=True)
    crow, col, val = x.crow_indices(), x.col_indices(), x.values()
    if crow.dtype != col.dtype or crow.dtype not in (torch.int32, torch.int64):
        return None
    out = torch.zeros((r1 - r0, c1 - c0), dtype=x.dtype, device=x.device)
    if out.numel() and val.numel():
        rc = L.sysml_slice_csr(_TCODE[x.dtype], int(crow.dtype == torch.int64), crow.data_ptr(), col.data_ptr(),
                               val.contiguous().data_ptr(), out.data_ptr(), r0, r1, c0, c1, _stream())
        if rc != 0:
            raise RuntimeError(f"sysml_slice_csr failed: {rc}")
    _count("slice_csr")
    return out


_sort_scratch = {}


def _scratch(n, dev):
    key = (dev, n)
    b = _sort_scratch.get(key)
    if b is None:
        L = load(required=True)
        nb = L.sysml_sort_pairs_scratch(n)
        if nb < 0:
            raise RuntimeError("sysml_sort_pairs_scratch failed")
        b = torch.empty((max(nb, 1),), dtype=torch.uint8, device=dev)
        if len(_sort_scratch) > 8:
            _sort_scratch.clear()
        _sort_scratch[key] = b
    return b


def order_perm(x, cols, decreasing):
    """0-based int32 row permutation that sorts the rows of device matrix x by the 1-based key
    columns `cols` (first most significant), stable, on the device: one radix pair sort per key
    from the last to the first.  None when not covered."""
    if not x.is_cuda or x.dtype not in _TCODE or x.shape[0] >= (1 << 31):
        return None
    ld = _rowpitch(x)
    if ld is None:
        return None
    L = load(required=True)
    n = x.shape[0]
    dev = x.device
    keys = torch.empty((n,), dtype=torch.float64, device=dev)
    kout = torch.empty_like(keys)
    perm = None
    tmp = torch.empty((n,), dtype=torch.int32, device=dev)
    vout = torch.empty((n,), dtype=torch.int32, device=dev)
    scr = _scratch(n, dev)
    for k in reversed(list(cols)):
        # keys of the current order and positions 0..n-1 in it (remapped through perm after the sort)
        rc = L.sysml_sort_keys_prep(_TCODE[x.dtype], x.data_ptr(), ld, int(k) - 1,
                                    perm.data_ptr() if perm is not None else None, keys.data_ptr(),
                                    tmp.data_ptr(), n, _stream())
        if rc != 0:
            raise RuntimeError(f"sysml_sort_keys_prep failed: {rc}")
        rc = L.sysml_sort_pairs(keys.data_ptr(), kout.data_ptr(), tmp.data_ptr(), vout.data_ptr(), n,
                                int(bool(decreasing)), scr.data_ptr(), scr.numel(), _stream())
        if rc != 0:
            raise RuntimeError(f"sysml_sort_pairs failed: {rc}")
        if perm is None:
            perm, vout = vout, torch.empty((n,), dtype=torch.int32, device=dev)
        else:
            newp = torch.empty((n,), dtype=torch.int32, device=dev)
            rc = L.sysml_perm_compose(vout.data_ptr(), perm.data_ptr(), newp.data_ptr(), None, 0, n, _stream())
            if rc != 0:
                raise RuntimeError(f"sysml_perm_compose failed: {rc}")
            perm = newp
    _count("order")
    return perm


def perm_index(perm, dtype):
    """(perm + 1) as an n x 1 matrix of `dtype` (order(..., index.return=TRUE))."""
    L = load(required=True)
    n = perm.numel()
    out = torch.empty((n, 1), dtype=dtype, device=perm.device)
    if n:
        rc = L.sysml_perm_compose(perm.data_ptr(), None, None, out.data_ptr(), _TCODE[dtype], n, _stream())
        if rc != 0:
            raise RuntimeError(f"sysml_perm_compose failed: {rc}")
    return out


def sort_values(v):
    """Ascending sort of a device vector's values (quantile / median): (sorted fp64 values,
    0-based int32 permutation)."""
    x = v.reshape(-1, 1)
    if not x.is_contiguous():
        x = x.contiguous()
    perm = order_perm(x, [1], False)
    if perm is None:
        return None
    L = load(required=True)
    n = x.shape[0]
    vals = torch.empty((n,), dtype=torch.float64, device=x.device)
    rc = L.sysml_sort_keys_prep(_TCODE[x.dtype], x.data_ptr(), 1, 0, perm.data_ptr(), vals.data_ptr(), None, n,
                                _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_sort_keys_prep failed: {rc}")
    return vals, perm


COMMIT_MAX = 16


def commit_live(pairs, live_enc):
    """Copy each (src, dst) tensor pair (same byte size) when the encoded run-ahead live flag
    (address | inverted bit) is live -- one launch (chain4.hip commit_live_kernel)."""
    L = load(required=True)
    n = len(pairs)
    if n > COMMIT_MAX or not live_enc:
        raise ValueError("commit_live: at most 16 pairs and a live flag")
    src = (ctypes.c_void_p * COMMIT_MAX)(*[s.data_ptr() for s, _ in pairs])
    dst = (ctypes.c_void_p * COMMIT_MAX)(*[d.data_ptr() for _, d in pairs])
    nb = (ctypes.c_longlong * COMMIT_MAX)(*[s.numel() * s.element_size() for s, _ in pairs])
    for s, d in pairs:
        if s.numel() * s.element_size() != d.numel() * d.element_size() or not (s.is_contiguous() and d.is_contiguous()):
            raise ValueError("commit_live: pairs must be contiguous and of one byte size")
    rc = L.sysml_commit_live(n, src, dst, nb, live_enc, _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_commit_live failed: {rc}")
    _count("commit_live")


def live_and(prev_enc, q_enc):
    """Device fp64 flag: 1.0 when neither encoded run-ahead live flag (address | inverted bit;
    0 = none) is dead (chain4.hip live_and_kernel)."""
    L = load(required=True)
    out = torch.empty((), dtype=torch.float64, device="cuda")
    rc = L.sysml_live_and(prev_enc or None, q_enc or None, out.data_ptr(), _stream())
    if rc != 0:
        raise RuntimeError(f"sysml_live_and failed: {rc}")
    return out
