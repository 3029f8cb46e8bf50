"""Builtin function implementations dispatched by name from `bi` / `sink` HOPs.

Reference: parser/BuiltinFunctionExpression.java + ParameterizedBuiltinFunctionExpression.java
(signatures/defaults) and the CP instructions implementing them
(runtime/instructions/cp/{DataGenCPInstruction,AppendCPInstruction,CtableCPInstruction,
ParameterizedBuiltinCPInstruction,MultiReturnBuiltinCPInstruction,QuantilePickCPInstruction,
CentralMomentCPInstruction,CovarianceCPInstruction,...}.java, LibCommonsMath.java).

Every function takes the ExecutionContext first, then DML arguments (positional
and named, with the reference's parameter names).
"""
from __future__ import annotations

import math
import time as _time

import numpy as np
import torch

from ..parser.errors import DMLRuntimeError, DMLScriptStop
from ..ops import core as C
from ..ops.backend import backend, place
from . import scalars as S
from .data import ListObject, FrameBlock

Tensor = torch.Tensor
REGISTRY = {}
MULTI_RETURN = set()


def builtin(*names, multi=False):
    def deco(fn):
        for n in names:
            REGISTRY[n] = fn
            if multi:
                MULTI_RETURN.add(n)
        return fn
    return deco


def _dev():
    return backend.device


def _dt():
    return backend.dtype


def _matk(x, what="argument"):
    """_mat for the DNN builtins: a bf16 activation in HBM stays bf16 (the dnn.hip kernels read
    bf16 directly; a conversion would be one more pass over it)."""
    if isinstance(x, Tensor) and x.dtype == torch.bfloat16 and x.is_cuda and backend.use_kernels:
        return x
    return _mat(x, what)


def _mat(x, what="argument"):
    if isinstance(x, Tensor):
        return C.cvt(x)
    if C.is_dist(x):
        import sys
        return C._dist()._fallback(x, "builtin:" + sys._getframe(1).f_code.co_name)
    if isinstance(x, FrameBlock):
        return place(x.to_matrix())
    if isinstance(x, (int, float, bool)):
        return torch.full((1, 1), float(x), dtype=_dt(), device=_dev())
    raise DMLRuntimeError(f"{what}: expected a matrix")


def _int(v, name="argument"):
    if isinstance(v, Tensor):
        v = v.reshape(-1)[0].item()
    try:
        return int(S.as_double(v)) if not isinstance(v, int) else v
    except DMLRuntimeError:
        raise DMLRuntimeError(f"{name}: expected an integer, got {v!r}")


def _float(v):
    if isinstance(v, Tensor):
        return float(v.reshape(-1)[0].item())
    return S.as_double(v)


def _bool(v):
    if isinstance(v, Tensor):
        return bool(v.reshape(-1)[0].item() != 0)
    return S.as_bool(v)


# ============================================================================
# printing / control
# ============================================================================
@builtin("print")
def b_print(ctx, x="", *rest, **kw):
    buf = getattr(ctx, "_ra_prints", None)
    if buf is not None and not rest:
        # a run-ahead loop iteration (runtime/program.py): printed once the iteration is
        # known to be live, in order; a deferred string is resolved then
        buf.append(x if type(x) is S.LazyStr else to_display_string(x))
        return None
    if rest:
        # printf-style print("fmt %d", a, b)
        s = _format(x, rest)
    else:
        s = to_display_string(x)
    ctx.print(s)
    return None


def _format(fmt, args):
    try:
        vals = [(_float(a) if isinstance(a, Tensor) else a) for a in args]
        return str(fmt) % tuple(vals)
    except TypeError as e:
        raise DMLRuntimeError(f"print format error: {e}")


@builtin("printf")
def b_printf(ctx, fmt, *args):
    ctx.print(_format(fmt, args))


def to_display_string(x):
    if isinstance(x, Tensor) or C.is_dist(x):
        return b_toString(None, x)
    if isinstance(x, FrameBlock):
        return b_toString(None, x)
    if isinstance(x, ListObject):
        return b_toString(None, x)
    return S.to_str(x)


@builtin("stop")
def b_stop(ctx, msg=""):
    raise DMLScriptStop(S.to_str(msg))


@builtin("assert")
def b_assert(ctx, cond):
    if not _bool(cond):
        raise DMLRuntimeError("assertion failed")


@builtin("time")
def b_time(ctx):
    return int(_time.time_ns())


@builtin("exists")
def b_exists(ctx, name, *a, **kw):
    """exists("X") with a computed name: probes the current frame's variables (statically
    named variables are resolved by the translator, compiler/translator.py)."""
    if isinstance(name, str):
        return name in ctx.vars
    return True


@builtin("toString")
def b_toString(ctx, target, rows=100, cols=100, decimal=3, sparse=False, sep=" ", linesep="\n"):
    if isinstance(target, ListObject):
        parts = []
        for i, v in enumerate(target.data):
            nm = target.names[i] if target.names else str(i + 1)
            parts.append(f"[{nm}]: {to_display_string(v)}")
        return "\n".join(parts)
    if isinstance(target, FrameBlock):
        r, c = target.shape
        lines = ["# FRAME: nrow = %d, ncol = %d" % (r, c),
                 "# " + sep.join(target.names), "# " + sep.join(target.schema)]
        for i in range(min(r, _int(rows))):
            lines.append(sep.join(S.to_str(v) if v is not None else "" for v in target.row(i)[:_int(cols)]))
        return linesep.join(lines) + linesep
    if not isinstance(target, Tensor) and not C.is_dist(target):
        return S.to_str(target)
    m = _mat(target).detach().cpu().double().numpy()
    r, c = m.shape
    r = min(r, _int(rows))
    c = min(c, _int(cols))
    d = _int(decimal)
    out = []
    if _bool(sparse):
        for i in range(r):
            for j in range(c):
                if m[i, j] != 0:
                    out.append(f"{i + 1}{sep}{j + 1}{sep}{_fmt_dec(m[i, j], d)}")
        return linesep.join(out) + linesep
    for i in range(r):
        out.append(sep.join(_fmt_dec(m[i, j], d) for j in range(c)))
    return linesep.join(out) + linesep


def _fmt_dec(v, d):
    if v != v:
        return "NaN"
    if v == math.inf:
        return "Infinity"
    if v == -math.inf:
        return "-Infinity"
    s = f"{v:.{d}f}"
    if s.startswith("-") and float(s) == 0:
        s = s[1:]
    return s


# ============================================================================
# data generation (reference: LibMatrixDatagen.java, DataGenCPInstruction.java)
# ============================================================================
def _seed(ctx, seed):
    """Resolve `seed = -1` (draw a fresh one).  In an SPMD run every rank must draw the same
    value for a replicated result, and a fixed `sysml.random.seed` makes runs repeatable:
    both come from the execution context's SeedSource (runtime/program.py)."""
    seed = _int(seed) if seed is not None else -1
    if seed != -1 or ctx is None or getattr(ctx, "seeds", None) is None:
        return seed
    return ctx.seeds.next()


def _gen(seed):
    seed = _int(seed) if seed is not None else -1
    g = torch.Generator(device="cpu")
    if seed is None or seed == -1:
        g.seed()
    else:
        g.manual_seed(seed)
    return g


def _devgen(seed):
    seed = _int(seed) if seed is not None else -1
    dev = _dev()
    g = torch.Generator(device=dev)
    if seed == -1:
        g.seed()
    else:
        g.manual_seed(seed)
    return g


@builtin("rand", "Rand")
def b_rand(ctx, rows=None, cols=None, min=0.0, max=1.0, sparsity=1.0, pdf="uniform", seed=-1,
           **kw):
    lam = kw.get("lambda", 1.0)
    if "dims" in kw:
        raise DMLRuntimeError("tensor rand not supported")
    r, c = _int(rows, "rows"), _int(cols, "cols")
    lo, hi = _float(min), _float(max)
    sp = _float(sparsity)
    pdf = str(pdf).lower()
    seed = _seed(ctx, seed)
    if ctx is not None and ctx.dist is not None and r >= ctx.config.dist_min_rows:
        return C._dist().rand(ctx, r, c, lo, hi, sp, pdf, seed, _float(lam))
    return _rand_local(r, c, lo, hi, sp, pdf, seed, _float(lam))


RAND_CHUNK_CELLS = 1 << 22


def rand_chunk_rows(c):
    """Rows per generator chunk: a seeded rand is produced in chunks of whole rows, chunk k
    from its own seed, so any row range of it can be generated alone and a row-partitioned
    rand equals the single-process one (reference: LibMatrixDatagen seeds per block)."""
    return max(1, RAND_CHUNK_CELLS // max(c, 1))


def _chunk_seed(seed, k):
    return seed if k == 0 else (seed + k * 1000003) % (1 << 62)


def _rand_local(r, c, lo, hi, sp, pdf, seed, lam, device=None, row_offset=0, total_rows=None):
    """Rows [row_offset, row_offset + r) of a (total_rows x c) rand matrix."""
    device = device or _dev()
    dt = _dt()
    total = r + row_offset if total_rows is None else total_rows
    if r == 0 or c == 0:
        return torch.zeros((r, c), dtype=dt, device=device)
    if seed == -1:
        seed = int(torch.randint(0, 1 << 62, (1,)).item())
    ch = rand_chunk_rows(c)
    k0, k1 = row_offset // ch, (row_offset + r - 1) // ch
    from ..ops import sparse as SP
    sparse = sp < SP.SPARSITY_TURN_POINT and total * c >= SP.MIN_CELLS and pdf in ("uniform", "normal") \
        and not (pdf == "uniform" and lo == hi == 0)
    parts = []
    for k in range(k0, k1 + 1):
        a, b = k * ch, min(total, (k + 1) * ch)
        g = torch.Generator(device=device)
        g.manual_seed(_chunk_seed(seed, k))
        blk = _rand_block(b - a, c, lo, hi, sp, pdf, lam, g, dt, device, sparse)
        lo_r, hi_r = max(a, row_offset) - a, min(b, row_offset + r) - a
        if lo_r != 0 or hi_r != b - a:
            blk = SP.csr_rows(blk, lo_r, hi_r) if sparse else blk[lo_r:hi_r]
        parts.append(blk)
    if len(parts) == 1:
        return parts[0] if sparse or parts[0].is_contiguous() else parts[0].contiguous()
    return SP.csr_vstack(parts) if sparse else torch.cat(parts, 0)


def _rand_block(r, c, lo, hi, sp, pdf, lam, g, dt, device, sparse):
    from ..ops import sparse as SP
    if sparse:
        # sparse rand: CSR generated directly (reference: sparse MatrixBlocks below the turn point)
        return SP.rand_csr(r, c, sp, lo, hi, pdf, g, dt, device)
    if pdf == "uniform":
        if lo == hi:
            m = torch.full((r, c), lo, dtype=dt, device=device)
        else:
            m = torch.rand((r, c), generator=g, dtype=dt, device=device) * (hi - lo) + lo
    elif pdf == "normal":
        m = torch.randn((r, c), generator=g, dtype=dt, device=device)
    elif pdf == "poisson":
        m = torch.poisson(torch.full((r, c), lam, dtype=dt, device=device), generator=g)
    else:
        raise DMLRuntimeError(f"unsupported pdf '{pdf}'")
    if sp < 1.0:
        mask = torch.rand((r, c), generator=g, dtype=dt, device=device) < sp
        m = m * mask
    return m


@builtin("matrix")
def b_matrix(ctx, data=None, rows=None, cols=None, byrow=True, dimnames=False, **kw):
    if isinstance(data, str):
        toks = data.replace(",", " ").split()
        vals = [float(t) for t in toks]
        r = _int(rows) if rows is not None else None
        c = _int(cols) if cols is not None else None
        if r is None and c is None:
            r, c = len(vals), 1
        elif r is None:
            r = len(vals) // c
        elif c is None:
            c = len(vals) // r
        if len(vals) != r * c:
            if len(vals) == 1:
                vals = vals * (r * c)
            else:
                raise DMLRuntimeError(f"matrix(): {len(vals)} values do not match {r}x{c}")
        t = torch.tensor(vals, dtype=torch.float64).reshape(r, c) if _bool(byrow) else \
            torch.tensor(vals, dtype=torch.float64).reshape(c, r).t()
        return place(t.contiguous())
    if isinstance(data, (Tensor,)) or C.is_dist(data):
        m = _mat(data)
        nr, nc = m.shape
        r = _int(rows) if rows is not None else None
        c = _int(cols) if cols is not None else None
        if r is None:
            r = nr * nc // c
        if c is None:
            c = nr * nc // r
        if r * c != nr * nc:
            raise DMLRuntimeError(f"reshape: cannot reshape {nr}x{nc} to {r}x{c}")
        if _bool(byrow):
            return m.contiguous().reshape(r, c)
        return m.t().contiguous().reshape(c, r).t().contiguous()
    if isinstance(data, FrameBlock):
        return place(data.to_matrix())
    v = _float(data if data is not None else 0.0)
    r, c = _int(rows, "rows"), _int(cols, "cols")
    if ctx is not None and ctx.dist is not None and r >= ctx.config.dist_min_rows:
        return C._dist().full(ctx, r, c, v)
    return torch.full((r, c), v, dtype=_dt(), device=_dev())


@builtin("seq")
def b_seq(ctx, frm=None, to=None, incr=None, **kw):
    frm = kw.get("from", frm)
    a, b = _float(frm), _float(to)
    if incr is None:
        inc = 1.0 if a <= b else -1.0
    else:
        inc = _float(incr)
    if inc == 0 or (b - a) * inc < 0:
        if a == b:
            n = 1
        else:
            raise DMLRuntimeError(f"seq: wrong sign for increment ({a}, {b}, {inc})")
    else:
        n = int(math.floor((b - a) / inc + 1e-10)) + 1
    if ctx is not None and ctx.dist is not None and n >= ctx.config.dist_min_rows:
        return C._dist().seq(ctx, a, inc, n)
    from ..ops.backend import home
    t = a + inc * torch.arange(n, dtype=torch.float64, device=home(n))   # generated where it lives
    return place(t.reshape(n, 1))


@builtin("sample")
def b_sample(ctx, range_=None, size=None, replace=False, seed=-1, **kw):
    rng = _int(kw.get("range", range_))
    n = _int(size)
    rep = _bool(replace) if not isinstance(replace, (int, float)) or isinstance(replace, bool) else False
    if isinstance(replace, (int, float)) and not isinstance(replace, bool) and seed == -1:
        seed = replace
        rep = False
    g = _gen(_seed(ctx, seed))
    if rep:
        v = torch.randint(1, rng + 1, (n,), generator=g, dtype=torch.int64)
    else:
        if n > rng:
            raise DMLRuntimeError("sample: size > range without replacement")
        v = torch.randperm(rng, generator=g)[:n] + 1
    return place(v.double().reshape(n, 1))


# ============================================================================
# append / reorg
# ============================================================================
def _one_device(ms):
    """Operands of an append on one device: a small host operand (e.g. the 1 x 1 constant of
    GLM's rbind(t(X) %*% w, matrix(sw, 1, 1))) joins the device of the largest operand."""
    dev = ms[0].device
    if all(m.device == dev for m in ms):
        return ms
    big = max(ms, key=lambda m: m.numel()).device
    return [m if m.device == big else m.to(big) for m in ms]


@builtin("cbind", "append")
def b_cbind(ctx, *args, **kw):
    if any(C.is_dist(a) for a in args):
        return C._dist().cbind(args)
    if isinstance(args[0], (str, S.LazyStr)):
        # string append (reference: StringObject append joins with a newline)
        if any(type(a) is S.LazyStr or type(a) is S.DevScalar for a in args) and backend.defer:
            r = args[0]
            for a in args[1:]:
                r = S.lazy_concat(r, a, "\n")
            return r
        return "\n".join(S.to_str(a) for a in args)
    if isinstance(args[0], ListObject):
        out = ListObject(args[0].data, args[0].names)
        for a in args[1:]:
            out.data.append(a)
            if out.names is not None:
                out.names.append("")
        return out
    if isinstance(args[0], FrameBlock):
        return FrameBlock.cbind([a if isinstance(a, FrameBlock) else C.unary("cast_frame", a) for a in args])
    ms = _one_device([_mat(a) for a in args])
    r = ms[0].shape[0]
    for m in ms[1:]:
        if m.shape[0] != r:
            raise DMLRuntimeError(f"cbind: number of rows do not match ({r} vs {m.shape[0]})")
    if backend.use_kernels and ms[0].is_cuda:
        from ..ops import kernels
        out = kernels.cat(False, ms)
        if out is not None:
            return out
    return torch.cat(ms, dim=1)


@builtin("_cbind_const")
def b_cbind_const(ctx, X, c, rows=None):
    """cbind(X, matrix(c, rows=nrow(X), cols=1)) as a constant-column view (ops/augmented.py)."""
    from ..ops import augmented as AUG
    n = X.shape[0] if hasattr(X, "shape") else None
    if rows is not None and n is not None and _int(rows) != n:
        return b_cbind(ctx, X, b_matrix(ctx, c, rows, 1))     # shapes differ: the cbind's own error
    return AUG.make(X, c)


@builtin("rbind")
def b_rbind(ctx, *args, **kw):
    if any(C.is_dist(a) for a in args):
        return C._dist().rbind(args)
    if isinstance(args[0], FrameBlock):
        cols = [list(c) for c in args[0].columns]
        for a in args[1:]:
            for j, c in enumerate(a.columns):
                cols[j] += c
        return FrameBlock(cols, args[0].schema, args[0].names)
    ms = _one_device([_mat(a) for a in args])
    c = ms[0].shape[1]
    for m in ms[1:]:
        if m.shape[1] != c:
            raise DMLRuntimeError(f"rbind: number of columns do not match ({c} vs {m.shape[1]})")
    if backend.use_kernels and ms[0].is_cuda:
        from ..ops import kernels
        out = kernels.cat(True, ms)
        if out is not None:
            return out
    return torch.cat(ms, dim=0)


@builtin("rev")
def b_rev(ctx, x):
    return torch.flip(_mat(x), dims=[0])


@builtin("diag")
def b_diag(ctx, x):
    m = _mat(x)
    r, c = m.shape
    if c == 1:
        return torch.diag(m.reshape(-1))
    if r == c:
        return torch.diagonal(m).reshape(-1, 1).clone()
    raise DMLRuntimeError("diag requires a square matrix or a column vector")


def _tri_kernel(m, lower, diag, values):
    """lower.tri / upper.tri of a device matrix in one pass (reorg.hip; SystemML.cu:425-429)."""
    if isinstance(m, Tensor) and m.is_cuda and backend.use_kernels and m.layout == torch.strided:
        from ..ops import kernels
        return kernels.tri(m, lower, diag, values)
    return None


@builtin("lower.tri")
def b_lower_tri(ctx, target=None, diag=False, values=False):
    m = _mat(target)
    r = _tri_kernel(m, True, _bool(diag), _bool(values))
    if r is not None:
        return r
    k = 0 if _bool(diag) else -1
    out = torch.tril(m, diagonal=k)
    if not _bool(values):
        out = (torch.tril(torch.ones_like(m), diagonal=k))
    return out


@builtin("upper.tri")
def b_upper_tri(ctx, target=None, diag=False, values=False):
    m = _mat(target)
    r = _tri_kernel(m, False, _bool(diag), _bool(values))
    if r is not None:
        return r
    k = 0 if _bool(diag) else 1
    out = torch.triu(m, diagonal=k)
    if not _bool(values):
        out = torch.triu(torch.ones_like(m), diagonal=k)
    return out


@builtin("order")
def b_order(ctx, target=None, by=1, decreasing=False, **kw):
    m = _mat(target)
    idx_ret = _bool(kw.get("index.return", False))
    dec = _bool(decreasing)
    keys = [int(v) for v in by.reshape(-1).tolist()] if isinstance(by, Tensor) else [_int(by)]
    for k in keys:
        if k < 1 or k > m.shape[1]:
            raise DMLRuntimeError(f"order: by column {k} out of range [1, {m.shape[1]}]")
    if isinstance(m, Tensor) and m.is_cuda and backend.use_kernels and m.layout == torch.strided:
        # device radix sort (sort.hip): stable key passes, then one row gather / index output
        from ..ops import kernels
        perm = kernels.order_perm(m, keys, dec)
        if perm is not None:
            if idx_ret:
                return kernels.perm_index(perm, m.dtype if m.dtype != torch.bfloat16 else backend.dtype)
            r = kernels.gather_rows(m, perm)
            if r is not None:
                return r
    if isinstance(by, Tensor) and by.numel() > 1:
        # several key columns (a column vector of indices): lexicographic, first column major --
        # stable sorts from the last key to the first
        keys = [int(v) for v in by.reshape(-1).tolist()]
        perm = torch.arange(m.shape[0], device=m.device)
        for k in reversed(keys):
            if k < 1 or k > m.shape[1]:
                raise DMLRuntimeError(f"order: by column {k} out of range [1, {m.shape[1]}]")
            p = torch.sort(m[perm, k - 1], descending=dec, stable=True).indices
            perm = perm[p]
    else:
        col = m[:, _int(by) - 1]
        # stable sort (ties keep input order), as the reference
        perm = torch.sort(col, descending=dec, stable=True).indices
    if idx_ret:
        return (perm + 1).to(m.dtype).reshape(-1, 1)
    return m[perm]


@builtin("removeEmpty")
def b_removeEmpty(ctx, target=None, margin="rows", select=None, **kw):
    if C.is_dist(target) and margin == "rows" and (select is None or C.is_dist(select)
                                                   or isinstance(select, Tensor)):
        return C._dist().remove_empty_rows(target, select)
    m = _mat(target)
    empty_return = _bool(kw.get("empty.return", True))
    if margin == "rows":
        keep = (m != 0).any(dim=1) if select is None else (_mat(select).reshape(-1) != 0)
        out = m[keep]
        if out.shape[0] == 0 and empty_return:
            return torch.zeros((1, m.shape[1]), dtype=m.dtype, device=m.device)
        return out
    if margin == "cols":
        keep = (m != 0).any(dim=0) if select is None else (_mat(select).reshape(-1) != 0)
        out = m[:, keep]
        if out.shape[1] == 0 and empty_return:
            return torch.zeros((m.shape[0], 1), dtype=m.dtype, device=m.device)
        return out
    raise DMLRuntimeError(f"removeEmpty: invalid margin '{margin}'")


@builtin("replace")
def b_replace(ctx, target=None, pattern=None, replacement=None):
    m = _mat(target).clone()
    p = _float(pattern)
    r = _float(replacement)
    if p != p:
        m[torch.isnan(m)] = r
    else:
        m[m == p] = r
    return m


@builtin("ifelse")
def b_ifelse(ctx, test, yes, no):
    if not any(isinstance(a, Tensor) or C.is_dist(a) for a in (test, yes, no)):
        return yes if _bool(test) else no
    t = test if isinstance(test, Tensor) else None
    shape_src = next(a for a in (test, yes, no) if isinstance(a, Tensor))
    def full(a):
        if isinstance(a, Tensor):
            return C.cvt(a)
        return torch.full(shape_src.shape, float(C._num(a)), dtype=_dt(), device=shape_src.device)
    tt, yy, nn = full(test), full(yes), full(no)
    return torch.where(tt != 0, yy, nn)


# ----------------------------------------------------------------------------
# data-parallel training across SPMD ranks (Caffe2DML allreduce algorithms, reference
# Caffe2DML.scala:396-405; here one rank per GPU with an RCCL gradient all-reduce)
# ----------------------------------------------------------------------------
@builtin("_dp_world")
def b_dp_world(ctx):
    return int(ctx.dist.world) if ctx.dist is not None else 1


@builtin("_dp_rank")
def b_dp_rank(ctx):
    return int(ctx.dist.rank) if ctx.dist is not None else 0


@builtin("_dp_allreduce", multi=True)
def b_dp_allreduce(ctx, *grads):
    """Sum over the ranks of every operand (the training script weights each rank's
    gradients by its share of the step's rows first), as ONE bucketed all-reduce: the
    matrices are packed into a flat fp32 / fp64 buffer in HBM (one RCCL call over xGMI
    instead of one per parameter), reduced and unpacked.  Single process: identity."""
    dist = ctx.dist
    if dist is None or dist.world <= 1:
        return tuple(grads)
    mats = [_mat(g) for g in grads]
    dev = dist._coll_device()
    dt = torch.float64 if any(m.dtype == torch.float64 for m in mats) else torch.float32
    flat = torch.cat([m.reshape(-1).to(device=dev, dtype=dt) for m in mats])
    dist.allreduce_(flat, "sum")
    out, off = [], 0
    for m in mats:
        n = m.numel()
        out.append(flat[off:off + n].reshape(m.shape).to(device=m.device, dtype=m.dtype))
        off += n
    return tuple(out)


# sparse-safe fused operators of compiler/rewrites.py (reference: the nnz / minus-nz / log-nz
# fusions of RewriteAlgebraicSimplification{Dynamic,Static}.java): on CSR operands they touch the
# stored values only, so a sparse X stays sparse
def _nz_apply(x, fn):
    if isinstance(x, Tensor) and x.layout == torch.sparse_csr:
        v = fn(x.values())
        return torch.sparse_csr_tensor(x.crow_indices(), x.col_indices(), v, x.shape, device=v.device)
    m = _mat(x)
    return torch.where(m != 0, fn(m), torch.zeros((), dtype=m.dtype, device=m.device))


@builtin("_nnz")
def b_nnz(ctx, x):
    """sum(X != 0) without the boolean matrix."""
    if isinstance(x, Tensor) and x.layout == torch.sparse_csr:
        return float(torch.count_nonzero(x.values()).item())     # a sum: DOUBLE, as before the rewrite
    if C.is_dist(x):
        return C.agg("sum", "all", C.binary("!=", x, 0))
    return float(torch.count_nonzero(_mat(x)).item())


@builtin("_minus_nz")
def b_minus_nz(ctx, x, s):
    """X - s * (X != 0)."""
    if C.is_dist(x):
        return C.binary("-", x, C.binary("*", s, C.binary("!=", x, 0)))
    sv = _float(s)
    return _nz_apply(x, lambda v: v - sv)


@builtin("_log_nz")
def b_log_nz(ctx, x, base=None):
    """(X != 0) * log(X [, base])."""
    if C.is_dist(x):
        lg = C.unary("log", x) if base is None else C.binary("log", x, base)
        return C.binary("*", C.binary("!=", x, 0), lg)
    if base is None:
        return _nz_apply(x, torch.log)
    lb = float(np.log(_float(base)))
    return _nz_apply(x, lambda v: torch.log(v) / lb)


@builtin("_axpy")
def b_axpy(ctx, x, s, y, sign):
    """X + sign * s * Y (reference TernaryOp PLUS_MULT / MINUS_MULT from
    fuseAxpyBinaryOperationChain): one pass over equally shaped dense host operands; anything
    else -- broadcasting, sparse, device or row-partitioned operands -- the two operators."""
    sg = _float(sign)
    if type(x) is Tensor and type(y) is Tensor and x.shape == y.shape and not x.is_cuda and not y.is_cuda \
            and x.layout == torch.strided and y.layout == torch.strided and x.dtype == y.dtype \
            and not isinstance(s, Tensor):
        return torch.add(x, y, alpha=sg * _float(s))
    return C.binary("+" if sg > 0 else "-", x, C.binary("*", s, y))


@builtin("_sel")
def b_sel(ctx, test, yes, no):
    """Select of an if-converted branch (compiler/ifconv.py): a scalar test picks one operand
    as is; a matrix test selects cellwise."""
    if isinstance(test, Tensor) or C.is_dist(test):
        return b_ifelse(ctx, test, yes, no)
    return yes if _bool(test) else no


@builtin("outer")
def b_outer(ctx, a, b, op):
    x = _mat(a)
    y = _mat(b)
    if x.shape[1] != 1 or y.shape[0] != 1:
        raise DMLRuntimeError("outer requires a column vector and a row vector")
    return C.binary(str(op), x, y)


@builtin("_gather_rows")
def b_gather_rows(ctx, idx, B, nrows, ncols=-1):
    """Rows of B selected by idx (1-based; rows with idx out of range are 0): the
    permutation-matrix product table(seq(1,n), idx, n, L) %*% B without the n x L matrix."""
    if C.is_dist(idx):
        idx = C._dist().gather(idx)
    if C.is_dist(B):
        B = C._dist().gather(B)
    I = _mat(idx).reshape(-1)
    M = _mat(B)
    n = int(nrows)
    L = int(ncols) if ncols is not None and int(ncols) >= 0 else M.shape[0]
    if L != M.shape[0]:
        raise DMLRuntimeError(f"matrix multiplication: dimension mismatch ({n}x{L} %*% {M.shape[0]}x{M.shape[1]})")
    if I.shape[0] != n:
        raise DMLRuntimeError("table: seq length does not match the category vector")
    k = I.round().long()
    ok = (k >= 1) & (k <= L)
    out = M.index_select(0, (k.clamp(1, max(L, 1)) - 1).to(M.device))
    return out * ok.to(device=M.device, dtype=M.dtype).reshape(-1, 1)


@builtin("table", "ctable")
def b_table(ctx, A=None, B=None, W=None, odim1=None, odim2=None, *rest, **kw):
    # table(A, B, [W], [d1, d2])
    args = [a for a in (A, B, W, odim1, odim2) + rest if a is not None]
    if "weights" in kw:
        args.insert(2, kw["weights"])
    A_, B_ = args[0], args[1]
    w = None
    dims = None
    rem = args[2:]
    if len(rem) in (1, 3):
        w = rem[0]
        rem = rem[1:]
    if len(rem) == 2:
        dims = (_int(rem[0]), _int(rem[1]))
    if C.is_dist(A_) or C.is_dist(B_):
        return C._dist().table(ctx, A_, B_, w, dims)
    a = _mat(A_).reshape(-1) if isinstance(A_, Tensor) else None
    b = _mat(B_).reshape(-1) if isinstance(B_, Tensor) else None
    n = a.numel() if a is not None else b.numel()
    if a is None:
        a = torch.full((n,), float(A_), dtype=_dt(), device=_dev())
    if b is None:
        b = torch.full((n,), float(B_), dtype=_dt(), device=_dev())
    # hybrid placement can leave one operand on the host and another in HBM
    if b.device != a.device:
        dev = a.device if a.is_cuda else b.device
        a, b = a.to(dev), b.to(dev)
    if w is None:
        wv = torch.ones(n, dtype=_dt(), device=a.device)
    elif isinstance(w, Tensor):
        wv = C.cvt(w).reshape(-1).to(a.device)
    else:
        wv = torch.full((n,), float(w), dtype=_dt(), device=a.device)
    return _ctable(a, b, wv, dims)


@builtin("_seq_expand")
def b_seq_expand(ctx, v, m):
    """outer(v, t(seq(1, m)), "==") without the sequence (rewrites.py simplifyOuterSeqExpand,
    reference rexpand with ignore=TRUE, cast=FALSE): cell (i, j) is 1 where v[i] == j exactly;
    values outside 1..m or not integral give a zero row."""
    yv = _mat(v).reshape(-1)
    k = _int(m)
    cols = torch.arange(1, k + 1, dtype=yv.dtype, device=yv.device)
    return (yv.reshape(-1, 1) == cols.reshape(1, -1)).to(_dt())


@builtin("_onehot")
def b_onehot(ctx, y, n=None, k=None):
    """table(seq(1, N), y [, N, K]) without materialising seq (rewrites.py _match_onehot):
    row i gets a 1 in column round(y[i]); rows beyond N / categories beyond K are dropped.
    Non-positive categories are an error, as in ctable."""
    if C.is_dist(y):
        return C._dist().onehot(ctx, y, n, k)
    yv = _mat(y).reshape(-1)
    yi = torch.round(yv).long()
    if yi.numel() and bool((yi <= 0).any()):
        raise DMLRuntimeError("ctable: invalid (non-positive) category values")
    rows = yi.numel() if n is None or _int(n) < 0 else _int(n)
    cols = (int(yi.max().item()) if yi.numel() else 0) if k is None or _int(k) < 0 else _int(k)
    m = min(rows, yi.numel())
    yi = yi[:m]
    out = torch.zeros((rows, cols), dtype=_dt(), device=yv.device)
    keep = yi <= cols
    if not bool(keep.all()):
        idx = torch.nonzero(keep).reshape(-1)
        out[idx, yi[idx] - 1] = 1.0
    else:
        out[:m].scatter_(1, (yi - 1).reshape(-1, 1), 1.0)
    return out


def _ctable(a, b, wv, dims):
    ai = torch.round(a).long()
    bi = torch.round(b).long()
    valid = (ai > 0) & (bi > 0)
    if not bool(valid.all()):
        if bool(((ai <= 0) | (bi <= 0)).any()):
            raise DMLRuntimeError("ctable: invalid (non-positive) category values")
    if dims is None:
        d1 = int(ai.max().item()) if ai.numel() else 0
        d2 = int(bi.max().item()) if bi.numel() else 0
    else:
        d1, d2 = dims
        keep = (ai <= d1) & (bi <= d2)
        ai, bi, wv = ai[keep], bi[keep], wv[keep]
    out = torch.zeros(d1 * d2, dtype=_dt(), device=a.device)
    out.index_add_(0, (ai - 1) * d2 + (bi - 1), wv.to(out.dtype))
    return out.reshape(d1, d2)


# ============================================================================
# statistics (reference: CentralMomentCPInstruction, CovarianceCPInstruction,
# QuantilePickCPInstruction, LibMatrixAgg grouped aggregates)
# ============================================================================
def _weights(w, n, like):
    if w is None:
        return None
    return _mat(w).reshape(-1).to(like.dtype)


@builtin("moment", "centralMoment")
def b_moment(ctx, x, a2=None, a3=None):
    v = _mat(x).reshape(-1)
    if a3 is not None:
        w = _mat(a2).reshape(-1).to(v.dtype)
        order = _int(a3)
    else:
        w = None
        order = _int(a2)
    if w is None:
        mu = v.mean()
        return float(((v - mu) ** order).mean().item())
    W = w.sum()
    mu = (v * w).sum() / W
    return float((w * (v - mu) ** order).sum().item() / W.item())


@builtin("cov")
def b_cov(ctx, x, y, w=None):
    a = _mat(x).reshape(-1)
    b = _mat(y).reshape(-1).to(a.dtype)
    if w is None:
        n = a.numel()
        return float(((a - a.mean()) * (b - b.mean())).sum().item() / (n - 1))
    wv = _mat(w).reshape(-1).to(a.dtype)
    W = wv.sum()
    ma = (a * wv).sum() / W
    mb = (b * wv).sum() / W
    return float(((a - ma) * (b - mb) * wv).sum().item() / (W.item() - 1))


def _sorted_weighted(x, w):
    m = _mat(x)
    if isinstance(m, Tensor) and m.is_cuda and backend.use_kernels and m.layout == torch.strided:
        from ..ops import kernels
        r = kernels.sort_values(m)
        if r is not None:
            vals, perm = r
            if w is None:
                return vals, None
            wm = _mat(w).reshape(-1, 1)
            wg = kernels.gather_rows(wm.contiguous(), perm) if wm.is_cuda else None
            if wg is not None:
                return vals, C.cvt(wg).reshape(-1).to(vals.dtype)
    v = m.reshape(-1)
    if w is None:
        return torch.sort(v).values, None
    wv = _mat(w).reshape(-1).to(v.dtype)
    s = torch.sort(v)
    return s.values, wv[s.indices]


def _quantile_pick(vals, wts, p):
    """Reference semantics (QuantilePickCPInstruction): value at position ceil(p*n) in sorted order."""
    if wts is None:
        n = vals.numel()
        pos = int(math.ceil(p * n)) - 1
        pos = min(max(pos, 0), n - 1)
        return float(vals[pos].item())
    cw = torch.cumsum(wts, 0)
    total = float(cw[-1].item())
    target = math.ceil(p * total)
    idx = int(torch.searchsorted(cw, torch.tensor(target, dtype=cw.dtype, device=cw.device)).item())
    idx = min(max(idx, 0), vals.numel() - 1)
    return float(vals[idx].item())


@builtin("quantile")
def b_quantile(ctx, x, a2, a3=None):
    if a3 is not None:
        vals, wts = _sorted_weighted(x, a2)
        p = a3
    else:
        vals, wts = _sorted_weighted(x, None)
        p = a2
    if isinstance(p, Tensor):
        ps = C.cvt(p).reshape(-1).tolist()
        out = [_quantile_pick(vals, wts, q) for q in ps]
        return place(torch.tensor(out, dtype=torch.float64).reshape(-1, 1))
    return _quantile_pick(vals, wts, _float(p))


@builtin("median")
def b_median(ctx, x, w=None):
    vals, wts = _sorted_weighted(x, w)
    n = vals.numel() if wts is None else float(wts.sum().item())
    if wts is None and n % 2 == 0:
        # reference: average of the two middle values for even counts
        return float((vals[n // 2 - 1] + vals[n // 2]).item() / 2)
    return _quantile_pick(vals, wts, 0.5)


@builtin("interQuantile")
def b_interquantile(ctx, x, a2, a3=None):
    if a3 is not None:
        vals, wts = _sorted_weighted(x, a2)
        p = _float(a3)
    else:
        vals, wts = _sorted_weighted(x, None)
        p = _float(a2)
    n = vals.numel()
    lo = int(math.ceil(n * p))
    hi = int(math.ceil(n * (1 - p)))
    return place(vals[lo:hi].reshape(-1, 1).clone())


@builtin("interQuartileMean")
def b_iqm(ctx, x, w=None):
    vals, wts = _sorted_weighted(x, w)
    n = vals.numel()
    if wts is None:
        q1 = n * 0.25
        q3 = n * 0.75
        lo = int(math.ceil(q1))
        hi = int(math.ceil(q3))
        s = vals[lo:hi].sum().item()
        # partial weights of boundary elements (reference: IQM with fractional ends)
        s += (lo - q1) * vals[lo - 1].item() if lo > 0 else 0.0
        s -= (hi - q3) * vals[hi - 1].item() if hi > 0 else 0.0
        return float(s / (q3 - q1))
    # weighted (reference MatrixBlock.interQuartileMean, weights as frequencies): walk the sorted
    # values by cumulative weight to the 25% / 75% marks, sum value * weight in between and
    # correct for the fractional weight of the two boundary values
    cw = torch.cumsum(wts.double(), 0)
    v = vals.double()
    sum_wt = float(cw[-1].item())
    q25d, q75d = 0.25 * sum_wt, 0.75 * sum_wt
    q25i, q75i = math.ceil(q25d), math.ceil(q75d)
    i25 = min(int(torch.searchsorted(cw, torch.tensor(float(q25i), dtype=cw.dtype, device=cw.device)).item()), n - 1)
    i75 = min(int(torch.searchsorted(cw, torch.tensor(float(q75i), dtype=cw.dtype, device=cw.device)).item()), n - 1)
    mid = (v[i25 + 1:i75 + 1] * wts.double()[i25 + 1:i75 + 1]).sum().item() if i75 > i25 else 0.0
    q25part, q25val = float(cw[i25].item()) - q25d, float(v[i25].item())
    q75part, q75val = float(cw[i75].item()) - q75d, float(v[i75].item())
    return float((mid + q25part * q25val - q75part * q75val) / (sum_wt * 0.5))


@builtin("aggregate")
def b_aggregate(ctx, target=None, groups=None, fn="sum", weights=None, ngroups=None, **kw):
    """Grouped aggregates (reference: ParameterizedBuiltin GROUPEDAGG); a multi-column
    target is aggregated column-wise (result ngroups x ncol)."""
    T = _mat(target)
    g = torch.round(_mat(groups).reshape(-1)).long()
    if T.shape[0] != g.numel() and T.shape[1] == g.numel() and T.shape[0] == 1:
        T = T.t()
    k = _int(ngroups) if ngroups is not None else int(g.max().item())
    keep = (g >= 1) & (g <= k)
    T, g = T[keep], g[keep] - 1
    w = _mat(weights).reshape(-1)[keep].to(T.dtype) if weights is not None else None
    fn = str(fn)
    dev, dt = T.device, T.dtype
    m = T.shape[1]
    ww = (w if w is not None else torch.ones(T.shape[0], dtype=dt, device=dev)).reshape(-1, 1)

    def gsum(v):
        return torch.zeros((k, m), dtype=dt, device=dev).index_add_(0, g, v)

    cnt = gsum(ww.expand(-1, m).contiguous())
    if fn == "count":
        out = cnt
    elif fn == "sum":
        out = gsum(T * ww)
    elif fn == "mean":
        out = gsum(T * ww) / cnt
    elif fn in ("variance", "var"):
        mu = gsum(T * ww) / cnt
        out = gsum(ww * (T - mu[g]) ** 2) / (cnt - 1)
    elif fn in ("min", "max"):
        init = math.inf if fn == "min" else -math.inf
        out = torch.full((k, m), init, dtype=dt, device=dev)
        out = out.scatter_reduce(0, g.reshape(-1, 1).expand(-1, m), T, reduce="amin" if fn == "min" else "amax")
    elif fn.startswith("centralmoment") or fn == "moment":
        order = _int(kw.get("order", 2))
        mu = gsum(T) / cnt
        out = gsum((T - mu[g]) ** order) / cnt
    else:
        raise DMLRuntimeError(f"aggregate: unsupported fn '{fn}'")
    return out


# ============================================================================
# distributions (reference: ParameterizedBuiltinCPInstruction cdf/invcdf)
# ============================================================================
def _num(v):
    """Distribution parameter: a float, or (matrix parameter, an extension over the
    reference's scalar-only cdf) an fp64 numpy array broadcast cell-wise against the target."""
    if isinstance(v, Tensor) and v.numel() != 1:
        return C.cvt(v).detach().double().cpu().numpy()
    return _float(v)


def _dist_fns(dist, prm):
    """(cdf, sf, ppf) of a distribution as plain scipy.special ufuncs: no frozen
    scipy.stats object per call, so scalar p-value loops (e.g. stratstats' fStat_tailprob)
    cost microseconds per call."""
    from scipy import special as sp
    _float = _num      # noqa: N806 -- parameters may be matrices
    if dist == "normal":
        mu, sd = _float(prm.get("mean", 0.0)), _float(prm.get("sd", 1.0))
        return (lambda x: sp.ndtr((x - mu) / sd), lambda x: sp.ndtr((mu - x) / sd),
                lambda u: sp.ndtri(u) * sd + mu)
    if dist == "exp":
        r = _float(prm.get("rate", 1.0))
        return (lambda x: -np.expm1(-r * np.maximum(x, 0.0)), lambda x: np.exp(-r * np.maximum(x, 0.0)),
                lambda u: -np.log1p(-u) / r)
    if dist == "chisq":
        k = _float(prm["df"])
        return (lambda x: sp.chdtr(k, np.maximum(x, 0.0)), lambda x: sp.chdtrc(k, np.maximum(x, 0.0)),
                lambda u: sp.chdtri(k, 1.0 - u))
    if dist == "f":
        a, b = _float(prm["df1"]), _float(prm["df2"])
        return (lambda x: sp.fdtr(a, b, np.maximum(x, 0.0)), lambda x: sp.fdtrc(a, b, np.maximum(x, 0.0)),
                lambda u: sp.fdtri(a, b, u))
    if dist == "t":
        k = _float(prm["df"])
        return (lambda x: sp.stdtr(k, x), lambda x: sp.stdtr(k, -x), lambda u: sp.stdtrit(k, u))
    raise DMLRuntimeError(f"unsupported distribution '{dist}'")


def _dist_fn(dist, q=None, p=None, lower=True, **prm):
    dist = str(dist).lower()
    x = q if q is not None else p
    if isinstance(x, torch.Tensor) and dist == "normal":
        # element-wise over a matrix (extension over the reference's scalar-only cdf);
        # the normal family stays on the device via torch.special
        mu, sd = _float(prm.get("mean", 0.0)), _float(prm.get("sd", 1.0))
        if q is not None:
            z = (x - mu) / sd
            return torch.special.ndtr(z if lower else -z)
        return torch.special.ndtri(x) * sd + mu
    cdf, sf, ppf = _dist_fns(dist, prm)
    fn = (cdf if lower else sf) if q is not None else ppf
    if isinstance(x, torch.Tensor):
        xn = C.cvt(x).detach().double().cpu().numpy()
        r = np.array(np.broadcast_to(np.asarray(fn(xn), dtype=np.float64), xn.shape))
        return torch.from_numpy(r).to(device=x.device, dtype=_dt())
    r = fn(_float(x))
    if isinstance(r, np.ndarray) and r.size != 1:      # scalar target, matrix parameters
        return torch.from_numpy(np.ascontiguousarray(r, dtype=np.float64)).to(device=_dev(), dtype=_dt())
    return float(r)


@builtin("cdf")
def b_cdf(ctx, target=None, dist="normal", **kw):
    lower = _bool(kw.pop("lower.tail", True))
    return _dist_fn(dist, q=target, lower=lower, **kw)


@builtin("invcdf", "icdf")
def b_invcdf(ctx, target=None, dist="normal", **kw):
    return _dist_fn(dist, p=target, **kw)


def _mk_dist(name, dist, inverse):
    def fn(ctx, target=None, **kw):
        lower = _bool(kw.pop("lower.tail", True))
        if inverse:
            return _dist_fn(dist, p=target, **kw)
        return _dist_fn(dist, q=target, lower=lower, **kw)
    REGISTRY[name] = fn


for _n, _d in (("pnorm", "normal"), ("pexp", "exp"), ("pchisq", "chisq"), ("pf", "f"), ("pt", "t")):
    _mk_dist(_n, _d, False)
for _n, _d in (("qnorm", "normal"), ("qexp", "exp"), ("qchisq", "chisq"), ("qf", "f"), ("qt", "t")):
    _mk_dist(_n, _d, True)


# ============================================================================
# linear algebra (reference: LibCommonsMath.java)
# ============================================================================
def _la(x):
    m = _mat(x)
    return m.double() if m.dtype != torch.float64 else m


@builtin("solve")
def b_solve(ctx, A, b):
    a, bb = _la(A), _la(b)
    if a.shape[0] != a.shape[1]:
        # least squares (reference: QR-based solve for non-square)
        return torch.linalg.lstsq(a.cpu(), bb.cpu()).solution.to(_dev(), _dt())
    return torch.linalg.solve(a, bb).to(_dt())


@builtin("inv", "inverse")
def b_inv(ctx, A):
    a = _la(A)
    if a.shape[0] != a.shape[1]:
        raise DMLRuntimeError("inv requires a square matrix")
    return torch.linalg.inv(a).to(_dt())


@builtin("cholesky")
def b_cholesky(ctx, A):
    return torch.linalg.cholesky(_la(A)).to(_dt())


@builtin("eigen", multi=True)
def b_eigen(ctx, A):
    a = _la(A)
    w, v = torch.linalg.eigh(a)
    return (w.reshape(-1, 1).to(_dt()), v.to(_dt()))


@builtin("svd", multi=True)
def b_svd(ctx, A):
    a = _la(A)
    U, Sv, Vh = torch.linalg.svd(a, full_matrices=False)
    return (U.to(_dt()), torch.diag(Sv).to(_dt()), Vh.t().contiguous().to(_dt()))


@builtin("qr", multi=True)
def b_qr(ctx, A):
    """[H, R] = qr(A): H (m x n) holds the Householder vectors column by column (lower
    trapezoidal, unit leading entry; reflector j is I - 2 v v'/(v'v)), R (m x n) is upper
    trapezoidal, A = H_1 ... H_n R (reference LibCommonsMath.computeQR semantics)."""
    a = _la(A)
    m, n = a.shape
    f, tau = torch.geqrf(a)
    H = torch.tril(f, -1)
    k = min(m, n)
    idx = torch.arange(k, device=H.device)
    H[idx, idx] = torch.where(tau[:k] != 0, torch.ones_like(tau[:k]), torch.zeros_like(tau[:k]))
    return (H.to(_dt()), torch.triu(f).to(_dt()))


@builtin("lu", multi=True)
def b_lu(ctx, A):
    a = _la(A)
    P, L, U = torch.linalg.lu(a)
    return (P.t().contiguous().to(_dt()), L.to(_dt()), U.to(_dt()))


# ============================================================================
# lists / eval
# ============================================================================
@builtin("list")
def b_list(ctx, *args, **kw):
    if kw and not args:
        return ListObject(list(kw.values()), list(kw.keys()))
    if kw:
        return ListObject(list(args) + list(kw.values()), [""] * len(args) + list(kw.keys()))
    return ListObject(list(args))


# ============================================================================
# IO
# ============================================================================
@builtin("read")
def b_read(ctx, fname, **kw):
    from ..io import readers
    return readers.read(ctx, S.to_str(fname), **kw)


@builtin("write")
def b_write(ctx, x, fname, **kw):
    from ..io import writers
    writers.write(ctx, x, S.to_str(fname), **kw)


# ============================================================================
# DNN builtins (reference: LibMatrixDNN*, ConvolutionCPInstruction)
# ============================================================================
def _nchw(x, C_, H, W):
    return _mat(x).reshape(-1, C_, H, W)


def _shape4(v):
    if isinstance(v, ListObject):
        return [_int(a) for a in v.data]
    if isinstance(v, (list, tuple)):
        return [_int(a) for a in v]
    raise DMLRuntimeError("expected a list of 4 integers (e.g. input_shape=[N,C,H,W])")


def _conv_params(kw):
    ishape = _shape4(kw["input_shape"])
    stride = _shape4(kw.get("stride", [1, 1]))
    padding = _shape4(kw.get("padding", [0, 0]))
    return ishape, stride, padding


@builtin("conv2d")
def b_conv2d(ctx, input=None, filter=None, bias=None, **kw):
    """conv2d; `bias` (F x 1) is set by the conv2d + bias_add fusion rewrite and added in the
    convolution kernel's epilogue (reference: DnnOp CONV2D_BIAS_ADD)."""
    from ..ops import dnn
    b = None if bias is None else _matk(bias).reshape(-1)
    return dnn.conv2d(_matk(input), _matk(filter), bias=b, **_conv_kw(kw))


@builtin("conv2d_backward_filter")
def b_conv2d_bwd_filter(ctx, input=None, dout=None, **kw):
    from ..ops import dnn
    return dnn.conv2d_backward_filter(_matk(input), _matk(dout), **_conv_kw(kw))


@builtin("conv2d_backward_data")
def b_conv2d_bwd_data(ctx, filter=None, dout=None, **kw):
    from ..ops import dnn
    return dnn.conv2d_backward_data(_matk(filter), _matk(dout), **_conv_kw(kw))


def _conv_kw(kw):
    out = {}
    for k in ("input_shape", "filter_shape", "stride", "padding", "pool_size"):
        if k in kw:
            out[k] = _shape4(kw[k])
    return out


@builtin("max_pool", "avg_pool")
def b_pool(ctx, input=None, **kw):
    from ..ops import dnn
    return dnn.pool(_matk(input), kind=kw.get("__name__", "max"), **_conv_kw(kw))


def _pool_factory(kind, backward):
    def fn(ctx, input=None, dout=None, **kw):
        from ..ops import dnn
        if backward:
            return dnn.pool_backward(_matk(input), _matk(dout), kind=kind, **_conv_kw(kw))
        return dnn.pool(_matk(input), kind=kind, **_conv_kw(kw))
    return fn


REGISTRY["max_pool"] = _pool_factory("max", False)
REGISTRY["avg_pool"] = _pool_factory("avg", False)
REGISTRY["max_pool_backward"] = _pool_factory("max", True)
REGISTRY["avg_pool_backward"] = _pool_factory("avg", True)


@builtin("bias_add")
def b_bias_add(ctx, input, bias):
    from ..ops import dnn
    return dnn.bias_op(_matk(input), _matk(bias), mult=False)


@builtin("bias_multiply")
def b_bias_mult(ctx, input, bias):
    from ..ops import dnn
    return dnn.bias_op(_matk(input), _matk(bias), mult=True)


# ============================================================================
# frames / transform (reference: runtime/transform/*)
# ============================================================================
@builtin("transformencode", multi=True)
def b_transformencode(ctx, target=None, spec=None):
    from . import transform
    return transform.encode(ctx, target, spec)


@builtin("transform")
def b_transform(ctx, target=None, **kw):
    from . import transform
    return transform.legacy_transform(ctx, target, **kw)


@builtin("transformapply")
def b_transformapply(ctx, target=None, spec=None, meta=None):
    from . import transform
    return transform.apply(ctx, target, spec, meta)


@builtin("transformdecode")
def b_transformdecode(ctx, target=None, spec=None, meta=None):
    from . import transform
    return transform.decode(ctx, target, spec, meta)


@builtin("transformcolmap")
def b_transformcolmap(ctx, target=None, spec=None):
    from . import transform
    return transform.colmap(ctx, target, spec)


@builtin("transformmeta")
def b_transformmeta(ctx, spec=None, meta=None):
    from . import transform
    return transform.read_meta(ctx, spec, meta)
