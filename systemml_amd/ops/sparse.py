"""Sparse matrices (reference: runtime/matrix/data/{SparseBlock,SparseBlockCSR,SparseBlockMCSR}
and the sparse paths of LibMatrixMult / LibMatrixAgg; MatrixBlock.evalSparseFormatInMemory
decides dense vs sparse with a 0.4 sparsity turn point).

Representation: a torch CSR tensor (`torch.sparse_csr`) on the backend device; on the
MI355X sparse x dense products (and row / column sums) run the in-tree SpMM / SpMV kernel
(ops/hip/spmm.hip) and the sampled products of the weighted quaternary operators the SDDMM
kernel (ops/hip/sddmm.hip).  Only the operations that benefit from sparsity keep the CSR form (matrix products incl. tsmm / mmchain, sum-type
aggregates, transpose, scaling by a scalar, shape queries, write); every other operator
receives a densified operand (instructions.make_impl), so semantics never depend on the
format.
"""
from __future__ import annotations

import torch

SPARSITY_TURN_POINT = 0.4          # reference: MatrixBlock.SPARSITY_TURN_POINT
MIN_CELLS = 1 << 16                # small matrices always stay dense


def is_sparse(x) -> bool:
    return isinstance(x, torch.Tensor) and x.layout in (torch.sparse_csr, torch.sparse_csc, torch.sparse_coo)


def densify(x):
    """Dense tensor of a sparse (CSR) or compressed (ops/compress.py) matrix."""
    if is_sparse(x):
        return x.to_dense()
    n = type(x).__name__
    if n == "CompressedMatrix":
        return x.decompress()
    if n == "ConstCol":
        return x.materialize()
    return x


def is_special(x) -> bool:
    """Sparse, compressed or constant-column (ops/augmented.py) representation: operators
    without a native path densify it."""
    return is_sparse(x) or type(x).__name__ in ("CompressedMatrix", "ConstCol")


def canonical(x):
    """CSR with strictly increasing column indices within every row (duplicate cells summed,
    as a dense conversion would): the sparse-at-non-zeros operators (weighted quaternaries,
    sparse-safe cellwise ops) assume one stored entry per cell."""
    if x.layout == torch.sparse_coo:
        return x.coalesce().to_sparse_csr()
    if x.layout != torch.sparse_csr:
        return x
    crow, col = x.crow_indices(), x.col_indices()
    if col.numel() < 2:
        return x
    inc = col[1:] > col[:-1]
    starts = torch.zeros(col.numel(), dtype=torch.bool, device=col.device)
    b = crow[1:-1]
    starts[b[b < col.numel()]] = True                 # first entry of each row
    if bool((inc | starts[1:]).all()):
        return x
    rows = torch.repeat_interleave(torch.arange(x.shape[0], device=crow.device), crow[1:] - crow[:-1])
    return from_ijv(rows, col, x.values(), x.shape[0], x.shape[1], x.values().dtype, x.device)


def nnz(x) -> int:
    if is_sparse(x):
        return int(x._nnz()) if x.layout != torch.sparse_coo else int(x.coalesce()._nnz())
    return int(torch.count_nonzero(x).item())


def want_sparse(rows, cols, nz) -> bool:
    cells = rows * cols
    return cells >= MIN_CELLS and nz < SPARSITY_TURN_POINT * cells


def maybe_sparse(x: torch.Tensor):
    """Convert a dense matrix to CSR when it is sparse enough to pay off."""
    if is_sparse(x) or x.dim() != 2 or x.dtype == torch.bfloat16:
        return x
    r, c = x.shape
    if r * c < MIN_CELLS:
        return x
    nz = int(torch.count_nonzero(x).item())
    return x.to_sparse_csr() if want_sparse(r, c, nz) else x


def from_ijv(i, j, v, rows, cols, dtype, device):
    """CSR matrix from 0-based COO triplets (duplicates summed)."""
    idx = torch.stack([torch.as_tensor(i, dtype=torch.int64), torch.as_tensor(j, dtype=torch.int64)])
    coo = torch.sparse_coo_tensor(idx, torch.as_tensor(v, dtype=dtype), (rows, cols)).coalesce()
    return coo.to_sparse_csr().to(device)


def rand_csr(rows, cols, sparsity, lo, hi, pdf, gen, dtype, device, chunk_cells=1 << 26):
    """rand(..., sparsity < 0.4) generated directly in CSR, row-chunked so the dense
    intermediate never exceeds `chunk_cells` cells."""
    crow = [torch.zeros(1, dtype=torch.int64, device=device)]
    cols_l, vals_l = [], []
    step = max(1, chunk_cells // max(cols, 1))
    base = 0
    for r0 in range(0, rows, step):
        r1 = min(rows, r0 + step)
        mask = torch.rand((r1 - r0, cols), generator=gen, device=device, dtype=torch.float32) < sparsity
        nzr, nzc = mask.nonzero(as_tuple=True)
        k = nzr.numel()
        if pdf == "normal":
            v = torch.randn(k, generator=gen, device=device, dtype=dtype)
        else:
            v = torch.rand(k, generator=gen, device=device, dtype=dtype) * (hi - lo) + lo
        counts = mask.sum(1, dtype=torch.int64)
        crow.append(base + torch.cumsum(counts, 0))
        base += k
        cols_l.append(nzc.to(torch.int64))
        vals_l.append(v)
    crow_t = torch.cat(crow)
    col_t = torch.cat(cols_l) if cols_l else torch.zeros(0, dtype=torch.int64, device=device)
    val_t = torch.cat(vals_l) if vals_l else torch.zeros(0, dtype=dtype, device=device)
    return torch.sparse_csr_tensor(crow_t, col_t, val_t, (rows, cols), device=device)


def csr_rows(x, r0, r1):
    """Rows [r0, r1) of a CSR matrix, still CSR (no densification)."""
    crow = x.crow_indices()
    a, b = int(crow[r0].item()), int(crow[r1].item())
    return torch.sparse_csr_tensor((crow[r0:r1 + 1] - a).contiguous(), x.col_indices()[a:b].contiguous(),
                                   x.values()[a:b].contiguous(), (r1 - r0, x.shape[1]), device=x.device)


def csr_vstack(parts):
    """rbind of CSR matrices with equal column counts, still CSR."""
    crows, cols, vals, base, rows = [], [], [], 0, 0
    for i, p in enumerate(parts):
        cr = p.crow_indices()
        crows.append(cr[(0 if i == 0 else 1):] + base)
        cols.append(p.col_indices())
        vals.append(p.values())
        base += int(cr[-1].item())
        rows += p.shape[0]
    return torch.sparse_csr_tensor(torch.cat(crows), torch.cat(cols), torch.cat(vals), (rows, parts[0].shape[1]),
                                   device=parts[0].device)


# ----------------------------------------------------------------------------
# sparse-aware operators (dense operands pass through untouched)
# ----------------------------------------------------------------------------
def _dense_rhs(b, dtype):
    b = densify(b)
    return b.to(dtype) if b.dtype != dtype else b


_TPLANS = {}        # CSR pattern -> (crow of t(A), col of t(A), permutation), see _transpose_plan


def _transpose_plan(a):
    """Structure of t(A) for CSR A and the permutation taking A's values to t(A)'s CSR order,
    cached per pattern: a pattern that is multiplied transposed again and again (the ratings
    of ALS, the sampled matrices of wdivmm built on it) pays the sort once, and every product
    is a gather plus the row-parallel SpMM instead of an atomic scatter.  The entry holds the
    pattern tensors, so their storage (the key) cannot be reused while it is cached."""
    crow, col = a.crow_indices(), a.col_indices()
    key = (crow.data_ptr(), col.data_ptr(), tuple(a.shape), col.numel())
    p = _TPLANS.get(key)
    if p is None and a.is_cuda:
        from .backend import backend
        if backend.use_kernels:
            # counting sort on the device (ops/hip/csrt.hip), no key sort
            from . import kernels
            t = kernels.csr_transpose_plan(crow, col, a.shape[0], a.shape[1])
            if t is not None:
                p = (t[0], t[1], t[2], crow, col)
                if len(_TPLANS) >= 4:
                    _TPLANS.pop(next(iter(_TPLANS), None), None)
                _TPLANS[key] = p
    if p is None:
        r, c = a.shape
        rows = torch.repeat_interleave(torch.arange(r, device=crow.device), crow[1:] - crow[:-1])
        perm = torch.argsort(col * r + rows)
        crowT = torch.zeros(c + 1, dtype=torch.int64, device=crow.device)
        crowT[1:] = torch.cumsum(torch.bincount(col, minlength=c), 0)
        p = (crowT, rows[perm].contiguous(), perm, crow, col)
        if len(_TPLANS) >= 4:
            _TPLANS.pop(next(iter(_TPLANS), None), None)   # tolerant of a concurrent parfor worker's eviction
        _TPLANS[key] = p
    return p


def mm(a, b, transA=False):
    """a %*% b (or t(a) %*% b) with a and/or b sparse.  On the MI355X a CSR left operand with
    a dense right operand runs the hand-written SpMM / SpMV kernel of ops/hip/spmm.hip; t(A)
    uses the cached transposed structure of A's pattern (_transpose_plan) when the product
    is wide enough to pay for the value gather, else the kernel's atomic scatter."""
    from .backend import backend
    if is_sparse(a) and a.layout == torch.sparse_csr and a.is_cuda and not is_sparse(b):
        if backend.use_kernels:
            from . import kernels
            bd = densify(b)
            if transA and bd.dim() == 2 and bd.shape[1] >= 4:
                at = _transposed(a)
                r = kernels.spmm_bal(at, bd)
                if r is not None:
                    return r
            r = kernels.spmm_bal(a, bd) if not transA else kernels.spmm(a, bd, True)
            if r is not None:
                return r
    if backend.use_kernels and is_sparse(a) and is_sparse(b) and a.is_cuda and b.is_cuda and \
            a.layout == torch.sparse_csr and b.layout == torch.sparse_csr:
        # sparse x sparse: Gustavson SpGEMM with an LDS accumulator (ops/hip/spgemm.hip)
        from . import kernels
        r = kernels.spgemm(_transposed(a) if transA else a, b)
        if r is not None:
            return r
    if backend.use_kernels and not is_sparse(a) and is_sparse(b) and b.layout == torch.sparse_csr and b.is_cuda \
            and isinstance(a, torch.Tensor) and a.is_cuda and a.dim() == 2:
        # dense x sparse: D %*% S = t(t(S) %*% t(D)), t(S) from the cached transpose plan and
        # the nnz-balanced SpMM over it
        from . import kernels
        at = a.t() if transA else a
        r = kernels.spmm_bal(_transposed(b), at.t().contiguous())
        if r is not None:
            return r.t().contiguous()
    if is_sparse(a):
        if transA:
            a = a.t()                                  # CSR^T = CSC, consumed by spmm
        return (a @ _dense_rhs(b, a.dtype)).contiguous()
    # dense %*% sparse = t(t(b) %*% t(a))
    at = a.t() if not transA else a
    return (b.t() @ at.t().contiguous().to(b.dtype)).t().contiguous() if is_sparse(b) else None


_TVALS = {}


def _transposed(a):
    """t(A) as CSR from the cached transpose plan of A's pattern (values gathered); the
    gathered values are cached too while A's value storage is unchanged (a fixed input such
    as the ratings of ALS is transposed once, not once per product)."""
    crowT, colT, perm, _, _ = _transpose_plan(a)
    v = a.values()
    key = (v.data_ptr(), v.numel(), v._version, perm.data_ptr())
    e = _TVALS.get(key)
    if e is None:
        if len(_TVALS) >= 2:
            _TVALS.pop(next(iter(_TVALS), None), None)   # tolerant of a concurrent parfor worker's eviction
        from .backend import backend
        if a.is_cuda and backend.use_kernels:
            from . import kernels
            vt = kernels.gather(v, perm)
        else:
            vt = v[perm]
        e = _TVALS[key] = (v, torch.sparse_csr_tensor(crowT, colT, vt, (a.shape[1], a.shape[0]),
                                                      device=a.device))
    return e[1]


def tsmm(x, left=True):
    """t(X) %*% X (left) or X %*% t(X) as a sparse x sparse product; the (small) result is dense.
    On the MI355X the left form is the pair-scatter kernel (ops/hip/spgemm.hip), the right
    form the SpGEMM of X and t(X) when its columns fit the LDS accumulator."""
    from .backend import backend
    if backend.use_kernels and x.is_cuda and x.layout == torch.sparse_csr:
        from . import kernels
        r = kernels.tsmm_sparse(x) if left else None
        if r is None and not left:
            r = kernels.spgemm(x, _transposed(x))
            if r is not None:
                r = r.to_dense()
        if r is not None:
            return r
    xt = x.t().to_sparse_csr()
    r = (xt @ x) if left else (x @ xt)
    return densify(r).contiguous()


def agg(o, d, x):
    """sum / sumsq / mean over all, rows or columns of a sparse matrix; None if unsupported."""
    r, c = x.shape
    if o not in ("sum", "sumsq", "mean"):
        return None
    vals = x.values()
    if o == "sumsq":
        xs = torch.sparse_csr_tensor(x.crow_indices(), x.col_indices(), vals * vals, x.shape) \
            if x.layout == torch.sparse_csr else None
        if xs is None:
            return None
        x = xs
        vals = x.values()
    if d == "all":
        s = float(vals.sum().item())
        return s / (r * c) if o == "mean" else s
    if d == "row":
        out = mm(x, torch.ones((c, 1), dtype=vals.dtype, device=vals.device))
        return out / c if o == "mean" else out
    out = mm(x, torch.ones((r, 1), dtype=vals.dtype, device=vals.device), transA=True).t().contiguous()
    return out / r if o == "mean" else out


def scale(x, s, op):
    v = x.values()
    nv = v * s if op == "*" else v / s
    return torch.sparse_csr_tensor(x.crow_indices(), x.col_indices(), nv, x.shape)


def transpose(x):
    return x.t().to_sparse_csr()


# ----------------------------------------------------------------------------
# sparse-safe cellwise operators (reference: LibMatrixBincell / LibMatrixUnary sparse paths,
# BinaryOperator.isSparseSafe / UnaryOperator.sparseSafe): when f(0[, .]) = 0 the result keeps
# the operand's non-zero pattern and only its stored values are transformed
# ----------------------------------------------------------------------------
SAFE_UNARY = {"abs", "sqrt", "round", "floor", "ceil", "sign", "sin", "tan", "asin", "atan", "sinh", "tanh",
              "neg"}


def _with_values(x, vals, prune=False):
    """CSR with x's pattern and new stored values; `prune` drops cells that became zero
    (comparisons, sign, round) so nnz() counts true non-zeros."""
    if prune and bool((vals == 0).any()):
        keep = vals != 0
        rows, cols = _rows_of(x)[keep], x.col_indices()[keep]
        return from_ijv(rows, cols, vals[keep], x.shape[0], x.shape[1], vals.dtype, vals.device)
    return torch.sparse_csr_tensor(x.crow_indices(), x.col_indices(), vals, x.shape)


def _rows_of(x):
    crow = x.crow_indices()
    counts = crow[1:] - crow[:-1]
    return torch.repeat_interleave(torch.arange(x.shape[0], device=crow.device), counts)


def unary(op, x, fn):
    """f(X) for a sparse-safe unary f on a CSR matrix (None if f is not sparse-safe)."""
    if op not in SAFE_UNARY or x.layout != torch.sparse_csr:
        return None
    return _with_values(x, fn(x.values()), prune=op in ("round", "floor", "ceil", "sign"))


def _scalar_safe(op, s, fn):
    """Is `X op s` zero wherever X is zero (so the result keeps X's pattern)?"""
    try:
        z = fn(torch.zeros((), dtype=torch.float64), torch.tensor(float(s), dtype=torch.float64))
    except Exception:   # noqa: BLE001
        return False
    return bool(z == 0)


def binary(op, a, b, fn):
    """Sparse-safe `a op b` with CSR `a`; None if the operation must densify.

    * sparse op scalar for any op with 0 op s == 0 (X * s, X / s (s != 0), X ^ s (s > 0),
      X > s (s >= 0), X != 0, max(X, s <= 0) ...);
    * sparse * dense (same shape, column or row vector broadcast): the dense operand is
      gathered at the stored cells;
    * sparse * sparse (intersection) and sparse +/- sparse (union) of equal shape."""
    if a.layout != torch.sparse_csr:
        return None
    if not isinstance(b, torch.Tensor):
        if isinstance(b, bool) or not isinstance(b, (int, float)):
            return None
        if not _scalar_safe(op, b, fn):
            return None
        v = a.values()
        return _with_values(a, fn(v, torch.tensor(float(b), dtype=v.dtype, device=v.device)).to(v.dtype), prune=True)
    if is_sparse(b):
        if b.layout != torch.sparse_csr or tuple(b.shape) != tuple(a.shape):
            return None
        if op in ("+", "-"):
            ac, bc = a.to_sparse_coo(), b.to_sparse_coo()
            r = ((ac + bc) if op == "+" else (ac - bc)).coalesce().to_sparse_csr()
            return _with_values(r, r.values(), prune=True)      # cells that cancelled are not stored
        if op == "*":
            if torch.equal(a.crow_indices(), b.crow_indices()) and torch.equal(a.col_indices(), b.col_indices()):
                return _with_values(a, a.values() * b.values(), prune=True)
            r = (a.to_sparse_coo() * b.to_sparse_coo()).coalesce().to_sparse_csr()
            return _with_values(r, r.values(), prune=True)
        return None
    if op != "*" or b.dim() != 2:
        return None
    r, c = a.shape
    if tuple(b.shape) == (r, c):
        g = b[_rows_of(a), a.col_indices()]
    elif tuple(b.shape) == (r, 1):
        g = b[_rows_of(a), 0]
    elif tuple(b.shape) == (1, c):
        g = b[0, a.col_indices()]
    else:
        return None
    v = a.values()
    return _with_values(a, v * g.to(v.dtype))
