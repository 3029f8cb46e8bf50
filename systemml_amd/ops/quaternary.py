"""Weighted quaternary operators (reference: hops/QuaternaryOp.java, lops/Weighted*.java,
runtime/matrix/data/LibMatrixMult.java#matrixMultW{SLoss,Sigmoid,DivMM,CeMM,UMM} and the
ALS-CG / GNMF / PNMF scripts that use them).

Every operator is a function of a low-rank product ``U %*% t(V)`` (U: m x r, V: n x r)
that is only needed at the non-zeros of a sparse weight / data matrix:

  wsloss    sum(W * (X - U%*%t(V))^2)      post     (also (X!=0) -> post_nz)
            sum((X - W * (U%*%t(V)))^2)    pre
            sum((X - U%*%t(V))^2)          none
  wsigmoid  W * sigmoid(+-U%*%t(V))        optionally log(sigmoid(...))
  wdivmm    (W / (U%*%t(V) [+ eps])) %*% V     t(U) %*% (W / (U%*%t(V) [+ eps]))
            (W * (U%*%t(V))) %*% V         t(U) %*% (W * (U%*%t(V)))
  wcemm     sum(X * log(U%*%t(V) [+ eps]))
  wumm      X * f(U%*%t(V)),  X / f(U%*%t(V))   (f unary)

MI355X design: with a CSR W / X the m x n product is never materialised — the sampled
product ``uv_k = <U[i_k], V[j_k]>`` is evaluated only at the nnz positions (SDDMM: row
gathers of U and V in nnz chunks, an r-wide dot per non-zero; both gathers hit HBM at
streaming bandwidth because r is small) and the result is either reduced to a scalar, kept
as a CSR with W's pattern, or multiplied by V / U through the sparse product.  wsloss "none"
over a sparse X uses sum(X^2) - 2 sum(U .* (X V)) + sum((U'U) .* (V'V)), which reads X once.
Dense operands (or row-partitioned / compressed ones) run the equivalent unfused operator
sequence of ops/core.py, so results never depend on the representation.
"""
from __future__ import annotations

import torch

from . import sparse as SP

_CHUNK = 1 << 22          # non-zeros per SDDMM chunk (chunk x r gathers of U and V)


def _C():
    from . import core
    return core


def _csr(x):
    if x.layout == torch.sparse_csr:
        return x
    return x.to_sparse_csr()


def _coo_idx(x):
    """(row, col, values) of a CSR matrix."""
    x = _csr(x)
    crow, col, val = x.crow_indices(), x.col_indices(), x.values()
    counts = crow[1:] - crow[:-1]
    row = torch.repeat_interleave(torch.arange(x.shape[0], device=x.device), counts)
    return row, col, val


def sddmm(row, col, U, V):
    """<U[row_k], V[col_k]> for every k (fp32 accumulate); on the GPU the hand-written
    wave-per-row kernel of ops/hip/sddmm.hip (row must be sorted, as CSR order gives)."""
    if U.is_cuda and row.numel() > 0:
        from . import kernels
        crow = torch.searchsorted(row, torch.arange(U.shape[0] + 1, device=row.device))
        out = kernels.sddmm(crow, col, U, V)
        if out is not None:
            return out
    U = U.float()
    V = V.float()
    out = torch.empty(row.numel(), dtype=torch.float32, device=U.device)
    for s in range(0, row.numel(), _CHUNK):
        e = min(s + _CHUNK, row.numel())
        out[s:e] = (U.index_select(0, row[s:e]) * V.index_select(0, col[s:e])).sum(1)
    return out


def _plain(x):
    return isinstance(x, torch.Tensor) and x.layout == torch.strided


def _dense_ok(*xs):
    return all(_plain(x) or SP.is_sparse(x) for x in xs)


def _uvt(U, V):
    C = _C()
    return C.mm(U, C.transpose(V))


def _sparse_like(pattern, vals):
    p = _csr(pattern)
    return torch.sparse_csr_tensor(p.crow_indices(), p.col_indices(), vals.to(torch.float32),
                                   size=p.shape, device=p.device)


def _check(U, V, m, n):
    from ..parser.errors import DMLRuntimeError
    if U.shape[1] != V.shape[1] or U.shape[0] != m or V.shape[0] != n:
        raise DMLRuntimeError(f"weighted quaternary op: dimension mismatch U{tuple(U.shape)} "
                              f"V{tuple(V.shape)} for a {m} x {n} matrix")


# ----------------------------------------------------------------------------- wsloss
def wsloss(kind, X, U, V, W=None):
    C = _C()
    if _dense_ok(X, U, V) and (W is None or _dense_ok(W)) and _plain(U) and _plain(V):
        _check(U, V, X.shape[0], X.shape[1])
        if kind == "post_nz" and SP.is_sparse(X):
            r, c, xv = _coo_idx(X)
            d = xv.float() - sddmm(r, c, U, V)
            return float((d * d).sum().item())
        if kind == "post" and W is not None and SP.is_sparse(W):
            r, c, wv = _coo_idx(W)
            xd = SP.densify(X).float()
            d = xd[r, c] - sddmm(r, c, U, V)
            return float((wv.float() * d * d).sum().item())
        if kind == "pre" and W is not None and SP.is_sparse(W) and _plain(X):
            r, c, wv = _coo_idx(W)
            wuv = wv.float() * sddmm(r, c, U, V)
            xf = X.float()
            return float(((xf * xf).sum() - 2.0 * (xf[r, c] * wuv).sum() + (wuv * wuv).sum()).item())
        if kind == "none" and SP.is_sparse(X):
            Uf, Vf = U.float(), V.float()
            xs = _csr(X).float() if X.dtype != torch.float32 else _csr(X)
            xv = xs.values()
            xvu = (torch.sparse.mm(xs, Vf) * Uf).sum()          # sum(X .* U V')
            uv2 = ((Uf.t() @ Uf) * (Vf.t() @ Vf)).sum()          # sum((U V')^2)
            return float(((xv * xv).sum() - 2.0 * xvu + uv2).item())
    # unfused (dense, row-partitioned or compressed operands)
    X = SP.densify(X)
    uv = _uvt(U, V)
    if kind == "pre":
        d = C.binary("-", X, C.binary("*", SP.densify(W), uv))
        return C.agg("sumsq", "all", d)
    d = C.binary("-", X, uv)
    if kind == "none":
        return C.agg("sumsq", "all", d)
    w = C.binary("!=", X, 0.0) if kind == "post_nz" else SP.densify(W)
    return C.tak(w, C.binary("*", d, d))


# ---------------------------------------------------------------------------- wsigmoid
def _sig(uv, minus, log):
    s = torch.sigmoid(-uv if minus else uv)
    return torch.log(s) if log else s


def wsigmoid(W, U, V, minus=False, log=False):
    C = _C()
    if SP.is_sparse(W) and _plain(U) and _plain(V):
        _check(U, V, W.shape[0], W.shape[1])
        r, c, wv = _coo_idx(W)
        return _sparse_like(W, wv.float() * _sig(sddmm(r, c, U, V), minus, log))
    uv = _uvt(U, V)
    if minus:
        uv = C.unary("neg", uv)
    s = C.unary("sigmoid", uv)
    if log:
        s = C.unary("log", s)
    return C.binary("*", SP.densify(W), s)


# ------------------------------------------------------------------------------ wdivmm
def wdivmm(W, U, V, left, mult=False, eps=None):
    """left=False: (W op UV') %*% V  (m x r);  left=True: t(U) %*% (W op UV')  (r x n)."""
    C = _C()
    if SP.is_sparse(W) and _plain(U) and _plain(V):
        _check(U, V, W.shape[0], W.shape[1])
        r, c, wv = _coo_idx(W)
        uv = sddmm(r, c, U, V)
        if mult:
            q = wv.float() * uv
        else:
            q = wv.float() / (uv + eps if eps is not None else uv)
        S = _sparse_like(W, q)
        if left:
            return torch.sparse.mm(S.t().to_sparse_csr(), U.float()).t().contiguous()
        return torch.sparse.mm(S, V.float())
    uv = _uvt(U, V)
    if eps is not None:
        uv = C.binary("+", uv, eps)
    q = C.binary("*" if mult else "/", SP.densify(W), uv)
    return C.mm(U, q, True) if left else C.mm(q, V)


# ------------------------------------------------------------------------------- wcemm
def wcemm(X, U, V, eps=None):
    C = _C()
    if SP.is_sparse(X) and _plain(U) and _plain(V):
        _check(U, V, X.shape[0], X.shape[1])
        r, c, xv = _coo_idx(X)
        uv = sddmm(r, c, U, V)
        if eps is not None:
            uv = uv + eps
        return float((xv.float() * torch.log(uv)).sum().item())
    uv = _uvt(U, V)
    if eps is not None:
        uv = C.binary("+", uv, eps)
    return C.tak(SP.densify(X), C.unary("log", uv))


# -------------------------------------------------------------------------------- wumm
def wumm(X, U, V, uop, op="*"):
    """X op f(U %*% t(V)) for a unary f (reference WeightedUnaryMM)."""
    C = _C()
    if SP.is_sparse(X) and op == "*" and _plain(U) and _plain(V):
        _check(U, V, X.shape[0], X.shape[1])
        r, c, xv = _coo_idx(X)
        f = C.unary(uop, sddmm(r, c, U, V)) if uop != "^2" else sddmm(r, c, U, V) ** 2
        return _sparse_like(X, xv.float() * f)
    uv = _uvt(U, V)
    f = C.binary("^", uv, 2.0) if uop == "^2" else C.unary(uop, uv)
    return C.binary(op, SP.densify(X), f)


def execute(p, a):
    """Dispatch of a `wquat` hop (compiler/rewrites.py#_match_wquat)."""
    k = p["kind"]
    eps = a[3] if p.get("eps") else None
    if k == "wsloss":
        return wsloss(p["type"], a[0], a[1], a[2], a[3] if len(a) > 3 else None)
    if k == "wsigmoid":
        return wsigmoid(a[0], a[1], a[2], p.get("minus", False), p.get("log", False))
    if k == "wdivmm":
        return wdivmm(a[0], a[1], a[2], p["left"], p.get("mult", False), eps)
    if k == "wcemm":
        return wcemm(a[0], a[1], a[2], eps)
    if k == "wumm":
        return wumm(a[0], a[1], a[2], p["uop"], p.get("op", "*"))
    raise ValueError(k)
