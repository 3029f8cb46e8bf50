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
Dense operands (or compressed ones) run the equivalent unfused operator sequence of
ops/core.py, so results never depend on the representation: the operators are sparse-safe
as in the reference (cells where W / X is zero contribute 0, even where f(U V') is +-inf or
NaN), and everything computes in the engine precision (fp64 by default; the SDDMM kernel has
fp32 and fp64 variants).  Row-partitioned operands run the same code per rank
(parallel/dist.wquat).
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


_ROWS = {}


def _coo_idx(x):
    """(row, col, values) of a CSR matrix; the expanded row indices are cached per pattern
    (the cache holds the row-pointer tensor, so its address -- the key -- stays unique)."""
    x = _csr(x)
    crow, col, val = x.crow_indices(), x.col_indices(), x.values()
    key = (crow.data_ptr(), crow.numel(), crow._version, col.numel())
    e = _ROWS.get(key)
    if e is None:
        counts = crow[1:] - crow[:-1]
        row = torch.repeat_interleave(torch.arange(x.shape[0], device=x.device), counts)
        if len(_ROWS) >= 4:
            _ROWS.pop(next(iter(_ROWS), None), None)   # tolerant of a concurrent parfor worker's eviction
        e = _ROWS[key] = (crow, row)
    return e[1], col, val


def _cdt(*xs):
    """Compute dtype: the engine's precision (fp64 unless `precision=single`); bf16-stored
    factors compute in fp32 (reference: the weighted operators compute in double)."""
    from .backend import backend
    dts = {x.dtype for x in xs if isinstance(x, torch.Tensor)}
    if torch.float64 in dts or backend.dtype == torch.float64:
        return torch.float64
    return torch.float32


def sddmm(row, col, U, V, crow=None, dtype=None):
    """<U[row_k], V[col_k]> for every k in `dtype`; on the GPU the hand-written grouped-lane
    kernel of ops/hip/sddmm.hip (row must be sorted, as CSR order gives)."""
    from .backend import backend
    dt = dtype or _cdt(U, V)
    if U.is_cuda and row.numel() > 0 and backend.use_kernels:
        from . import kernels
        if crow is None:
            crow = torch.searchsorted(row, torch.arange(U.shape[0] + 1, device=row.device))
        out = kernels.sddmm(crow, kernels.idx32_of(col) if V.shape[0] < 2 ** 31 else col, U, V, dt)
        if out is not None:
            return out
    U = U.to(dt)
    V = V.to(dt)
    out = torch.empty(row.numel(), dtype=dt, device=U.device)
    for s in range(0, row.numel(), _CHUNK):
        e = min(s + _CHUNK, row.numel())
        out[s:e] = (U.index_select(0, row[s:e]) * V.index_select(0, col[s:e])).sum(1)
    return out


def _sd(x, U, V, dt):
    """(row, col, values as dt, sampled U V' as dt) at the non-zeros of CSR x."""
    x = _csr(x)
    r, c, v = _coo_idx(x)
    return r, c, v.to(dt), sddmm(r, c, U, V, crow=x.crow_indices(), dtype=dt)


def _plain(x):
    return isinstance(x, torch.Tensor) and x.layout == torch.strided


def _dense_ok(*xs):
    return all(_plain(x) or SP.is_sparse(x) for x in xs)


def _uvt(U, V):
    C = _C()
    return C.mm(U, C.transpose(V))


def _sparse_like(pattern, vals):
    p = _csr(pattern)
    return torch.sparse_csr_tensor(p.crow_indices(), p.col_indices(), vals, size=p.shape, device=p.device)


def _check(U, V, m, n):
    from ..parser.errors import DMLRuntimeError
    if U.shape[1] != V.shape[1] or U.shape[0] != m or V.shape[0] != n:
        raise DMLRuntimeError(f"weighted quaternary op: dimension mismatch U{tuple(U.shape)} "
                              f"V{tuple(V.shape)} for a {m} x {n} matrix")


def _values_at(X, W, r, c, dt):
    """X's values at W's non-zero positions (r, c in CSR order).  A sparse X is looked up by
    sorted linear index (same pattern: its values directly) -- never densified."""
    if SP.is_sparse(X):
        xs, ws = _csr(X), _csr(W)
        if xs.col_indices().numel() == ws.col_indices().numel() and \
                torch.equal(xs.crow_indices(), ws.crow_indices()) and torch.equal(xs.col_indices(), ws.col_indices()):
            return xs.values().to(dt)
        xr, xc, xv = _coo_idx(xs)
        n = X.shape[1]
        kx = xr * n + xc                              # sorted (CSR order)
        kw = r * n + c
        pos = torch.searchsorted(kx, kw).clamp_(max=max(kx.numel() - 1, 0))
        hit = (kx.numel() > 0) & (kx[pos] == kw) if kx.numel() else torch.zeros_like(kw, dtype=torch.bool)
        return torch.where(hit, xv[pos].to(dt), torch.zeros((), dtype=dt, device=xv.device)) if kx.numel() \
            else torch.zeros(kw.numel(), dtype=dt, device=kw.device)
    return X[r, c].to(dt)


# ----------------------------------------------------------------------------- wsloss
def wsloss(kind, X, U, V, W=None):
    C = _C()
    if _dense_ok(X, U, V) and (W is None or _dense_ok(W)) and _plain(U) and _plain(V):
        _check(U, V, X.shape[0], X.shape[1])
        dt = _cdt(X, U, V, W)
        if kind == "post_nz" and SP.is_sparse(X):
            _, _, xv, uv = _sd(X, U, V, dt)
            d = xv - uv
            return float((d * d).sum().item())
        if kind == "post" and W is not None and SP.is_sparse(W):
            r, c, wv, uv = _sd(W, U, V, dt)
            d = _values_at(X, W, r, c, dt) - uv
            return float((wv * d * d).sum().item())
        if kind == "pre" and W is not None and SP.is_sparse(W) and _plain(X):
            # sum((X - W*UV')^2): residual at W's non-zeros plus X^2 where W is zero -- both
            # sums of squares, no cancelling subtraction
            r, c, wv, uv = _sd(W, U, V, dt)
            xrc = X[r, c].to(dt)
            d = xrc - wv * uv
            xz = X.to(dt).clone()
            xz[r, c] = 0
            return float(((d * d).sum() + (xz * xz).sum()).item())
        if kind == "none" and SP.is_sparse(X):
            # sum((X - UV')^2) = sum_nz (x - uv)^2 + sum_zero uv^2, the second term as
            # sum((U'U) .* (V'V)) - sum_nz uv^2 (a sum over cells X does not hold, fp64)
            _, _, xv, uv = _sd(X, U, V, dt)
            Uf, Vf = U.to(dt), V.to(dt)
            d = xv - uv
            zero_part = ((Uf.t() @ Uf) * (Vf.t() @ Vf)).sum() - (uv * uv).sum()
            return float(((d * d).sum() + zero_part).item())
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


def _sparse_safe(W, f):
    """W * f with f only where W != 0: the operators are sparse-safe in the reference (they
    iterate over W's non-zeros), so zeros of W stay 0 even where f is +-inf or NaN."""
    C = _C()
    Wd = SP.densify(W)
    prod = C.binary("*", Wd, f)
    if isinstance(prod, torch.Tensor) and isinstance(Wd, torch.Tensor):
        return torch.where(Wd != 0, prod, torch.zeros((), dtype=prod.dtype, device=prod.device))
    return prod


def wsigmoid(W, U, V, minus=False, log=False):
    C = _C()
    if SP.is_sparse(W) and _plain(U) and _plain(V):
        _check(U, V, W.shape[0], W.shape[1])
        dt = _cdt(W, U, V)
        _, _, wv, uv = _sd(W, U, V, dt)
        return _sparse_like(W, wv * _sig(uv, minus, log))
    uv = _uvt(U, V)
    if minus:
        uv = C.unary("neg", uv)
    s = C.unary("sigmoid", uv)
    if log:
        s = C.unary("log", s)
    return _sparse_safe(W, s)


# ------------------------------------------------------------------------------ wdivmm
def wdivmm(W, U, V, left, mult=False, eps=None, X=None):
    """left=False: (W op UV') %*% V  (m x r);  left=True: t(U) %*% (W op UV')  (r x n);
    with X (mult only): W * (UV' - X), the residual of the ALS gradients."""
    C = _C()
    if SP.is_sparse(W) and _plain(U) and _plain(V) and (X is None or _plain(X) or SP.is_sparse(X)):
        _check(U, V, W.shape[0], W.shape[1])
        dt = _cdt(W, U, V)
        r = _wdivmm_fused(W, U, V, left, mult, eps, X, dt)
        if r is not None:
            return r
        r, c, wv, uv = _sd(W, U, V, dt)
        if X is not None:
            if tuple(X.shape) != tuple(W.shape):
                from ..parser.errors import DMLRuntimeError
                raise DMLRuntimeError(f"wdivmm: X {tuple(X.shape)} does not match W {tuple(W.shape)}")
            uv = uv - _values_at(X, W, r, c, dt)
        if mult:
            q = wv * uv
        else:
            q = wv / (uv + eps if eps is not None else uv)
        S = _sparse_like(W, q)
        # the sampled matrix times a factor: CSR SpMM (ops/hip/spmm.hip on the MI355X; t(S)
        # by atomic scatter, no transposed copy)
        if left:
            return SP.mm(S, U.to(dt), transA=True).t().contiguous()
        return SP.mm(S, V.to(dt))
    uv = _uvt(U, V)
    if eps is not None:
        uv = C.binary("+", uv, eps)
    if X is not None:
        uv = C.binary("-", uv, SP.densify(X))
    q = C.binary("*", SP.densify(W), uv) if mult else _sparse_safe(W, C.binary("/", 1.0, uv))
    return C.mm(U, q, True) if left else C.mm(q, V)


_PATEQ = {}


def _same_pattern(A, B):
    """A and B are CSR with the same pattern (shared index tensors, or equal ones -- compared
    once per pair of index storages)."""
    if A.layout != torch.sparse_csr or B.layout != torch.sparse_csr or A.shape != B.shape:
        return False
    ca, cb = A.crow_indices(), B.crow_indices()
    ia, ib = A.col_indices(), B.col_indices()
    if ca.data_ptr() == cb.data_ptr() and ia.data_ptr() == ib.data_ptr():
        return True
    if ia.numel() != ib.numel():
        return False
    key = (ca.data_ptr(), cb.data_ptr(), ia.data_ptr(), ib.data_ptr(), ia.numel(), ca._version, ia._version)
    r = _PATEQ.get(key)
    if r is None:
        if len(_PATEQ) >= 8:
            _PATEQ.pop(next(iter(_PATEQ), None), None)
        r = _PATEQ[key] = (bool(torch.equal(ca, cb)) and bool(torch.equal(ia, ib)), (ca, cb, ia, ib))
    return r[0]


def _wdivmm_fused(W, U, V, left, mult, eps, X, dt):
    """The fused kernel (ops/hip/sddmm.hip wdivmm_kernel) for a CSR W on the MI355X: one pass
    over W's pattern gathering each V (U for the left form) row once; the left form runs on
    the transposed pattern of W, which -- with W's values and X's values in its order -- is
    cached per pattern (ALS: W and X are fixed across all iterations).  None: not applicable
    (X of another pattern, rank > 64, host operands)."""
    from .backend import backend
    if not (backend.use_kernels and W.is_cuda and W.layout == torch.sparse_csr and U.is_cuda and V.is_cuda):
        return None
    if X is not None and not (mult and SP.is_sparse(X) and X.is_cuda and _same_pattern(W, X)):
        return None
    from . import kernels
    mode = 1 if X is not None else (0 if mult else 2)
    e = float(eps) if (eps is not None and not mult) else 0.0
    if not left:
        xv = X.values() if X is not None else None
        col = kernels.idx32_of(W.col_indices()) if W.shape[1] < 2 ** 31 else W.col_indices()
        return kernels.wdivmm(W.crow_indices(), col, W.values(), xv, U, V, mode, e, dt)
    Wt = SP._transposed(W)
    xt = SP._transposed(X).values() if X is not None else None
    col = kernels.idx32_of(Wt.col_indices()) if Wt.shape[1] < 2 ** 31 else Wt.col_indices()
    r = kernels.wdivmm(Wt.crow_indices(), col, Wt.values(), xt, V, U, mode, e, dt)
    return r.t().contiguous() if r is not None else None


# ------------------------------------------------------------------------------- wcemm
def wcemm(X, U, V, eps=None):
    C = _C()
    if SP.is_sparse(X) and _plain(U) and _plain(V):
        _check(U, V, X.shape[0], X.shape[1])
        dt = _cdt(X, U, V)
        _, _, xv, uv = _sd(X, U, V, dt)
        if eps is not None:
            uv = uv + eps
        return float((xv * torch.log(uv)).sum().item())
    uv = _uvt(U, V)
    if eps is not None:
        uv = C.binary("+", uv, eps)
    return C.agg("sum", "all", _sparse_safe(X, C.unary("log", uv)))


# -------------------------------------------------------------------------------- wumm
def wumm(X, U, V, uop, op="*"):
    """X op f(U %*% t(V)) for a unary f (reference WeightedUnaryMM)."""
    C = _C()
    if SP.is_sparse(X) and op == "*" and _plain(U) and _plain(V):
        _check(U, V, X.shape[0], X.shape[1])
        dt = _cdt(X, U, V)
        _, _, xv, uv = _sd(X, U, V, dt)
        f = C.unary(uop, uv) if uop != "^2" else uv * uv
        return _sparse_like(X, xv * f)
    uv = _uvt(U, V)
    f = C.binary("^", uv, 2.0) if uop == "^2" else C.unary(uop, uv)
    if op == "*":
        return _sparse_safe(X, f)
    return C.binary(op, SP.densify(X), f)


def execute(p, a):
    """Dispatch of a `wquat` hop (compiler/rewrites.py#_match_wquat)."""
    C = _C()
    if any(C.is_dist(x) for x in a):
        return C._dist().wquat(p, a)
    k = p["kind"]
    eps = a[3] if p.get("eps") else None
    if k == "wsloss":
        return wsloss(p["type"], a[0], a[1], a[2], a[3] if len(a) > 3 else None)
    if k == "wsigmoid":
        return wsigmoid(a[0], a[1], a[2], p.get("minus", False), p.get("log", False))
    if k == "wdivmm":
        return wdivmm(a[0], a[1], a[2], p["left"], p.get("mult", False), eps,
                      X=a[-1] if p.get("minus") else None)
    if k == "wcemm":
        return wcemm(a[0], a[1], a[2], eps)
    if k == "wumm":
        return wumm(a[0], a[1], a[2], p["uop"], p.get("op", "*"))
    raise ValueError(k)
