"""Generated Outer-product-template operators (reference: hops/codegen/template/
TemplateOuterProduct.java, cplan/CNodeOuterProduct.java and runtime/codegen/
SpoofOuterProduct.java with its output types CELLWISE_OUTER_PRODUCT, AGG_OUTER_PRODUCT,
LEFT_OUTER_PRODUCT and RIGHT_OUTER_PRODUCT).

An `OuterProgram` is a fused cellwise DAG f(W, U %*% t(V), ...) that is sparse-safe in a
driver matrix W: wherever W is zero, f is zero (the compiler proves it structurally,
compiler/codegen.fuse_outer).  The low-rank product is therefore only needed at W's
non-zeros, and the program ends in
  cell   f itself (m x n, W's sparsity pattern),
  all    sum(f),
  left   f %*% B   (m x k, e.g. B = V: the wdivmm left form),
  right  t(f) %*% B (n x k, e.g. B = U).
The weighted quaternary operators of ops/quaternary.py are fixed instances; this is the
general template with any cellwise body (the fused cell program of ops/cell.py).

MI355X execution with a CSR driver: U %*% t(V) is sampled at the non-zeros by the
hand-written SDDMM kernel (ops/hip/sddmm.hip), the other cell inputs are gathered at the same
positions, the cell program runs once over the nnz values (one generated cell kernel,
ops/cell.py), and the sparse result feeds the CSR SpMM kernels (ops/hip/spmm.hip) for the
left / right forms -- the m x n product is never materialised.  A dense driver computes the
product with the MFMA GEMM and then runs the same cell program over the full matrix; off the
GPU (and for operands the sparse path does not cover) the original operators run one by one.
"""
from __future__ import annotations

import torch

from . import core as C
from . import sparse as SP
from .cell import CellProgram, evaluate as cell_eval, sequential as cell_seq

OTYPES = ("cell", "all", "left", "right")
stats = {"sparse": 0, "dense": 0, "sequential": 0}


class OuterProgram:
    """cell: CellProgram over the cell inputs; uv: index of the U %*% t(V) value among them;
    w: index of the sparse-safe driver among them; otype; inputs of the operator are
    [U, V] + the cell inputs except uv (+ B for left / right)."""
    __slots__ = ("cell", "uv", "w", "otype")

    def __init__(self, cell: CellProgram, uv, w, otype):
        if otype not in OTYPES:
            raise ValueError(otype)
        self.cell = cell
        self.uv = uv
        self.w = w
        self.otype = otype

    def key(self):
        return (self.cell.key(), self.uv, self.w, self.otype)

    def __eq__(self, other):
        return isinstance(other, OuterProgram) and self.key() == other.key()

    def __hash__(self):
        return hash(self.key())

    def describe(self):
        return f"outer[{self.cell.describe()}]|{self.otype}"

    def __repr__(self):
        return self.describe()

    def split(self, args):
        """(U, V, cell inputs with the uv slot empty, B or None)."""
        U, V = args[0], args[1]
        n = self.cell.n_in - 1
        rest = list(args[2:2 + n])
        B = args[2 + n] if self.otype in ("left", "right") else None
        cin = rest[:self.uv] + [None] + rest[self.uv:]
        return U, V, cin, B


def _finish(prog, r, B):
    ot = prog.otype
    if ot == "cell":
        return r
    if ot == "all":
        return C.agg("sum", "all", r)
    if ot == "left":
        return C.mm(r, B)
    return C.mm(r, B, True)


def sequential(prog: OuterProgram, args):
    """The original operators: the full product U %*% t(V), the cell DAG, the output operator."""
    U, V, cin, B = prog.split(args)
    cin[prog.uv] = C.mm(U, C.transpose(V))
    return _finish(prog, cell_seq(prog.cell, cin), B)


def evaluate(prog: OuterProgram, args):
    from .backend import backend
    U, V, cin, B = prog.split(args)
    W = cin[prog.w]
    dense = lambda x: isinstance(x, torch.Tensor) and x.layout == torch.strided
    if backend.use_kernels and SP.is_sparse(W) and dense(U) and dense(V) and W.is_cuda:
        r = _sparse(prog, U, V, cin, W, B)
        if r is not None:
            stats["sparse"] += 1
            return r
    if backend.use_kernels and dense(W) and dense(U) and dense(V) and W.is_cuda:
        stats["dense"] += 1
        cin[prog.uv] = C.mm(U, C.transpose(V))             # MFMA GEMM
        return _finish(prog, cell_eval(prog.cell, cin), B)
    stats["sequential"] += 1
    return sequential(prog, args)


def _sparse(prog, U, V, cin, W, B):
    """CSR driver: sample U V' at W's non-zeros, evaluate the cell program over the nnz values."""
    from . import quaternary as Q
    from ..runtime.scalars import DevScalar
    m, n = W.shape
    if U.dim() != 2 or V.dim() != 2 or U.shape[0] != m or V.shape[0] != n or U.shape[1] != V.shape[1]:
        return None                                           # the sequential path raises
    Wc = Q._csr(W)
    row, col, _ = Q._coo_idx(Wc)
    dt = Q._cdt(U, V)
    vals = []
    for k, x in enumerate(cin):
        if k == prog.uv:
            vals.append(Q.sddmm(row, col, U, V, crow=Wc.crow_indices(), dtype=dt).reshape(-1, 1))
            continue
        if x is W:
            vals.append(Wc.values().to(dt).reshape(-1, 1))
            continue
        if isinstance(x, (int, float, bool)) or type(x) is DevScalar:
            vals.append(x)
            continue
        if not isinstance(x, torch.Tensor) or x.device != W.device:
            return None
        if SP.is_sparse(x):
            if tuple(x.shape) != (m, n):
                return None
            vals.append(Q._values_at(x, Wc, row, col, dt).reshape(-1, 1))
            continue
        r, c = x.shape
        if (r, c) == (m, n):
            vals.append(x[row, col].to(dt).reshape(-1, 1))
        elif (r, c) == (1, 1):
            vals.append(x.to(dt))
        elif (r, c) == (m, 1):
            vals.append(x[row, 0].to(dt).reshape(-1, 1))
        elif (r, c) == (1, n):
            vals.append(x[0, col].to(dt).reshape(-1, 1))
        else:
            return None
    if row.numel() == 0:
        v = torch.zeros((0, 1), dtype=dt, device=W.device)
    else:
        v = cell_eval(prog.cell, vals)
        if not isinstance(v, torch.Tensor) or v.shape != (row.numel(), 1):
            return None
    f = torch.sparse_csr_tensor(Wc.crow_indices(), Wc.col_indices(), v.reshape(-1).to(dt), size=(m, n),
                                device=W.device)
    ot = prog.otype
    if ot == "all":
        return C._lazy_out(v.sum()) if v.numel() else 0.0
    if ot == "cell":
        return f
    return _finish(prog, f, B)
