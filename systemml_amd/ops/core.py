"""Local matrix operator library (reference: runtime/matrix/data/LibMatrixBincell.java,
LibMatrixAgg.java, LibMatrixReorg.java, LibMatrixMult.java, and the GPU
counterparts LibMatrixCUDA.java / LibMatrixCuMatMult.java).

All functions accept DML runtime values: Python scalars (bool/int/float/str),
2-D torch tensors (host or HBM) and row-partitioned DistMatrix objects (routed
to systemml_amd.parallel.dist).  Hot GPU paths (skinny matmults, mmchain,
row-fused Hessian-vector products, sum-of-squares aggregates, bf16-stored
inputs) go to the hand-written HIP kernels in ops/kernels.py.
"""
from __future__ import annotations

import math

import torch

from ..parser.errors import DMLRuntimeError
from ..runtime import scalars as S
from ..runtime.scalars import DevScalar
from .backend import backend
from . import sparse as SP
from . import compress as CMP

Tensor = torch.Tensor
_DIST = None


def _dist():
    global _DIST
    if _DIST is None:
        from ..parallel import dist as d
        _DIST = d
    return _DIST


def is_dist(x):
    return isinstance(x, _dist().DistMatrix)


def cvt_sp(x):
    if x.dtype != backend.dtype and x.dtype in (torch.float32, torch.float64):
        return x.to(backend.dtype)
    return x


def cvt(x: Tensor) -> Tensor:
    """bf16 storage → compute dtype (materialises; kernels avoid this).  Device matrices widen
    in one pass of reorg.hip's copy2d (any row pitch), not an ATen cast."""
    if x.dtype == torch.bfloat16:
        if x.is_cuda and backend.use_kernels and x.dim() == 2:
            from . import kernels
            r = kernels.copy2d(x, backend.dtype)
            if r is not None:
                return r
        return x.to(backend.dtype)
    return x


def dense_copy(x: Tensor) -> Tensor:
    """A dense row-major copy of a device view (slice windows, strided rows) on reorg.hip; the
    tensor itself when it is already contiguous."""
    if x.is_contiguous():
        return x
    if x.is_cuda and backend.use_kernels and x.dim() == 2:
        from . import kernels
        r = kernels.copy2d(x)
        if r is not None:
            return r
    return x.contiguous()


def _num(v):
    if isinstance(v, bool):
        return 1.0 if v else 0.0
    if isinstance(v, str):
        raise DMLRuntimeError(f"string '{v}' used in a matrix operation")
    return v


def _fdt(x: Tensor):
    return x.dtype if x.dtype in (torch.float32, torch.float64) else backend.dtype


# ----------------------------------------------------------------------------
# binary cellwise
# ----------------------------------------------------------------------------
def _rel(fn):
    def f(a, b):
        r = fn(a, b)
        return r.to(_out_dtype(a, b))
    return f


def _out_dtype(a, b):
    for x in (a, b):
        if isinstance(x, Tensor) and x.dtype in (torch.float32, torch.float64):
            return x.dtype
    return backend.dtype


def _logical(fn):
    def f(a, b):
        a2 = (a != 0) if isinstance(a, Tensor) else bool(a != 0)
        b2 = (b != 0) if isinstance(b, Tensor) else bool(b != 0)
        if not isinstance(a2, Tensor):
            a2 = torch.tensor(a2, device=b.device)
        if not isinstance(b2, Tensor):
            b2 = torch.tensor(b2, device=a.device)
        return fn(a2, b2).to(_out_dtype(a, b))
    return f


def _min(a, b):
    if not isinstance(a, Tensor):
        a, b = b, a
    if not isinstance(b, Tensor):
        b = float(b)
        if b == b:          # clamp: no scalar tensor upload, vectorised; NaN cells of a stay NaN
            return torch.clamp(a, max=b)
        b = torch.tensor(b, dtype=a.dtype, device=a.device)
    return torch.minimum(a, b)


def _max(a, b):
    if not isinstance(a, Tensor):
        a, b = b, a
    if not isinstance(b, Tensor):
        b = float(b)
        if b == b:          # e.g. relu's max(X, 0)
            return torch.clamp(a, min=b)
        b = torch.tensor(b, dtype=a.dtype, device=a.device)
    return torch.maximum(a, b)


def _pow(a, b):
    if isinstance(b, (int, float)) and b == 2:
        return a * a
    if not isinstance(a, Tensor):
        a = torch.tensor(float(a), dtype=b.dtype, device=b.device)
    return torch.pow(a, b)


def _mod(a, b):
    if not isinstance(a, Tensor):
        a = torch.tensor(float(a), dtype=b.dtype, device=b.device)
    return torch.remainder(a, b)


def _intdiv(a, b):
    if not isinstance(a, Tensor):
        a = torch.tensor(float(a), dtype=b.dtype, device=b.device)
    return torch.floor(a / b)


def _log2(a, b):
    la = torch.log(a) if isinstance(a, Tensor) else math.log(a) if a > 0 else (-math.inf if a == 0 else math.nan)
    lb = torch.log(b) if isinstance(b, Tensor) else math.log(b)
    return la / lb


def _bitw(fn):
    def f(a, b):
        ai = a.long() if isinstance(a, Tensor) else int(a)
        bi = b.long() if isinstance(b, Tensor) else int(b)
        return fn(ai, bi).to(_out_dtype(a, b))
    return f


BIN = {
    "+": lambda a, b: a + b,
    "-": lambda a, b: a - b,
    "*": lambda a, b: a * b,
    "/": lambda a, b: a / b,
    "^": _pow,
    "%%": _mod,
    "%/%": _intdiv,
    "==": _rel(lambda a, b: a == b),
    "!=": _rel(lambda a, b: a != b),
    "<": _rel(lambda a, b: a < b),
    "<=": _rel(lambda a, b: a <= b),
    ">": _rel(lambda a, b: a > b),
    ">=": _rel(lambda a, b: a >= b),
    "&": _logical(torch.logical_and),
    "|": _logical(torch.logical_or),
    "xor": _logical(torch.logical_xor),
    "min": _min,
    "max": _max,
    "log": _log2,
    "bitwAnd": _bitw(lambda a, b: a & b),
    "bitwOr": _bitw(lambda a, b: a | b),
    "bitwXor": _bitw(lambda a, b: a ^ b),
    "bitwShiftL": _bitw(lambda a, b: a << b),
    "bitwShiftR": _bitw(lambda a, b: a >> b),
}


def _check_bin_dims(a: Tensor, b: Tensor, op):
    sa, sb = a.shape, b.shape
    if sa == sb:
        return
    (ra, ca), (rb, cb) = sa, sb
    ok = ((ra == rb and (ca == 1 or cb == 1)) or (ca == cb and (ra == 1 or rb == 1)) or
          (ra == 1 and ca == 1) or (rb == 1 and cb == 1) or
          (ca == 1 and rb == 1) or (ra == 1 and cb == 1))
    if not ok:
        raise DMLRuntimeError(f"Block sizes are not matched for binary cell operations: "
                              f"{ra}x{ca} vs {rb}x{cb} (op {op})")


_PYNUM = (int, float, bool)
_STRIDED = torch.strided


# ----------------------------------------------------------------------------
# HBM-resident scalars (runtime/scalars.DevScalar): scalar algebra queued on the device
# ----------------------------------------------------------------------------
_DEV_ARITH = {"+", "-", "*", "/", "^", "min", "max"}
_DEV_CMP = {"==": torch.eq, "!=": torch.ne, "<": torch.lt, "<=": torch.le, ">": torch.gt, ">=": torch.ge}


def _lazy_out(r):
    """A 0-d (or 1x1) device aggregate -> DevScalar on a lazy backend, else a Python float."""
    if backend.lazy and isinstance(r, Tensor) and r.is_cuda:
        return DevScalar(r.reshape(()).to(torch.float64))
    return float(r.item()) if isinstance(r, Tensor) else float(r)


def _dev_bool(x):
    """(x != 0) as a 0-d bool tensor (x DevScalar) or a Python bool."""
    if type(x) is DevScalar:
        return x.t != 0
    return S.as_bool(x)


def _dev_binary(op, a, b):
    # a device scalar whose value the host already read (a branch, a print) is a host value from
    # then on: its further scalar algebra runs on the host, not as tiny device launches between
    # host syncs (the solvers' outer-loop bookkeeping)
    if type(a) is DevScalar and a._v is not None:
        a = a._v
    if type(b) is DevScalar and b._v is not None:
        b = b._v
    if type(a) is not DevScalar and type(b) is not DevScalar:
        return binary(op, a, b)
    da, db = type(a) is DevScalar, type(b) is DevScalar
    other = b if da else a
    if isinstance(other, Tensor) and not (da and db):
        if other.is_cuda and other.layout is _STRIDED and op in BIN and op not in ("log",) \
                and not op.startswith("bitw"):
            m = cvt(other)
            s = (a if da else b).t.to(m.dtype)
            return BIN[op](s, m) if da else BIN[op](m, s)
        return binary(op, S.materialize(a), S.materialize(b))
    if isinstance(other, (str,)) or not (da and db or isinstance(other, (int, float, bool))):
        if op == "+" and type(other) is str and backend.defer:
            return S.lazy_concat(a, b)       # a run-ahead iteration: read the value when it is live
        return binary(op, S.materialize(a), S.materialize(b))
    x = a.t if da else float(S._num(a))
    y = b.t if db else float(S._num(b))
    if op in _DEV_ARITH:
        if op == "+":
            r = x + y
        elif op == "-":
            r = x - y
        elif op == "*":
            r = x * y
        elif op == "/":
            r = x / y
        elif op == "^":
            r = torch.pow(x, y)
        else:
            xt = x if da else torch.full_like(y, x)
            yt = y if db else torch.full_like(x, y)
            r = torch.minimum(xt, yt) if op == "min" else torch.maximum(xt, yt)
        # INT op INT stays INT except for '/' and '^' (runtime/scalars.binary)
        ints = op not in ("/", "^") and (a.vt == "i" if da else type(a) is int) and (b.vt == "i" if db else type(b) is int)
        return DevScalar(r, "i" if ints else "d")
    if op in _DEV_CMP:
        r = _DEV_CMP[op](x, y) if da else _DEV_CMP[op](torch.full_like(y, x), y)
        return DevScalar(r.to(torch.float64), "b")
    if op in ("&", "|", "xor"):
        p, q = _dev_bool(a), _dev_bool(b)
        if not isinstance(p, Tensor):
            p, q = q, p                      # p is the device side
        if not isinstance(q, Tensor):        # fold the host boolean
            if op == "&":
                return DevScalar(p.to(torch.float64), "b") if q else False
            if op == "|":
                return True if q else DevScalar(p.to(torch.float64), "b")
            return DevScalar((~p if q else p).to(torch.float64), "b")
        r = torch.logical_and(p, q) if op == "&" else torch.logical_or(p, q) if op == "|" else torch.logical_xor(p, q)
        return DevScalar(r.to(torch.float64), "b")
    return S.binary(op, S.materialize(a), S.materialize(b))


_DEV_UN = {"neg": torch.neg, "abs": torch.abs, "exp": torch.exp, "log": torch.log, "sqrt": torch.sqrt,
           "floor": torch.floor, "ceil": torch.ceil, "sign": torch.sign, "sin": torch.sin, "cos": torch.cos,
           "tan": torch.tan, "asin": torch.asin, "acos": torch.acos, "atan": torch.atan, "sinh": torch.sinh,
           "cosh": torch.cosh, "tanh": torch.tanh, "sigmoid": torch.sigmoid,
           "round": lambda t: torch.floor(t + 0.5)}


def _dev_unary(op, x):
    if x._v is not None:                 # already read back: host arithmetic (see _dev_binary)
        return unary(op, x._v)
    f = _DEV_UN.get(op)
    if f is not None and x.vt != "b":
        return DevScalar(f(x.t), "i" if (x.vt == "i" and op in ("neg", "abs", "sign", "floor", "ceil", "round"))
                         else "d")
    if op == "not":
        return DevScalar((x.t == 0).to(torch.float64), "b")
    if op in ("ident", "cast_scalar"):
        return x
    if op == "cast_double":
        return DevScalar(x.t) if x.vt == "d" else DevScalar(x.t.clone())
    if op == "cast_bool":
        return DevScalar((x.t != 0).to(torch.float64), "b")
    if op == "cast_matrix":
        return x.t.reshape(1, 1).to(backend.dtype)
    return unary(op, x.value())


from . import augmented as AUG   # noqa: E402  (cbind(X, const) views)
_CC = AUG.ConstCol


def binary(op, a, b):
    if type(a) is _CC or type(b) is _CC:
        return AUG.binary(op, a, b)
    if type(a) is S.LazyStr or type(b) is S.LazyStr:
        if op == "+":
            return S.lazy_concat(a, b)
        a, b = S.materialize(a), S.materialize(b)
    # fast paths: two Python scalars; dense same-device same-dtype tensors (or tensor-scalar)
    ta_, tb_ = type(a), type(b)
    if ta_ in _PYNUM and tb_ in _PYNUM:
        return S.binary(op, a, b)
    if ta_ is DevScalar or tb_ is DevScalar:
        return _dev_binary(op, a, b)
    if ta_ is Tensor and a.layout is _STRIDED and a.dtype is not torch.bfloat16:
        fn = BIN.get(op)
        if fn is not None:
            if tb_ is Tensor:
                if b.layout is _STRIDED and b.dtype is a.dtype and b.device == a.device:
                    _check_bin_dims(a, b, op)
                    return fn(a, b)
            elif tb_ is int or tb_ is float:
                return fn(a, b)
    elif tb_ is Tensor and (ta_ is int or ta_ is float) and b.layout is _STRIDED and b.dtype is not torch.bfloat16:
        fn = BIN.get(op)
        if fn is not None:
            return fn(a, b)
    if CMP.is_compressed(a):
        if op in ("*", "/") and isinstance(b, (int, float)) and not isinstance(b, bool) and (op == "*" or b != 0):
            return a.scale(float(b) if op == "*" else 1.0 / float(b))
        a = a.decompress()
    if CMP.is_compressed(b):
        if op == "*" and isinstance(a, (int, float)) and not isinstance(a, bool):
            return b.scale(float(a))
        b = b.decompress()
    ta, tb = isinstance(a, Tensor), isinstance(b, Tensor)
    if ta and SP.is_sparse(a):
        if not tb and op in ("*", "/") and isinstance(b, (int, float)) and not isinstance(b, bool) \
                and (op == "*" or b != 0):
            return SP.scale(a, float(b), op)
        fn = BIN.get(op)
        r = SP.binary(op, a, b if not tb or SP.is_sparse(b) else cvt(b), fn) if fn is not None else None
        if r is not None:
            return r
        a = SP.densify(a)
    if tb and SP.is_sparse(b):
        if not ta and op == "*" and isinstance(a, (int, float)) and not isinstance(a, bool):
            return SP.scale(b, float(a), "*")
        if op in ("*", "+") and ta:              # commutative: dense * sparse, sparse + sparse
            fn = BIN.get(op)
            r = SP.binary(op, b, cvt(a), fn) if fn is not None and not SP.is_sparse(a) and op == "*" else None
            if r is not None:
                return r
        b = SP.densify(b)
    if not ta and not tb:
        if is_dist(a) or is_dist(b):
            return _dist().binary(op, a, b)
        if hasattr(a, "columns") or hasattr(b, "columns"):
            raise DMLRuntimeError(f"operator {op} not supported on frames")
        return S.binary(op, a, b)
    if is_dist(a) or is_dist(b):
        return _dist().binary(op, a, b)
    fn = BIN.get(op)
    if fn is None:
        raise DMLRuntimeError(f"unknown binary operator {op}")
    if ta and tb:
        a, b = cvt(a), cvt(b)
        if a.device != b.device:
            b = b.to(a.device)
        if a.dtype != b.dtype:
            dt = torch.promote_types(a.dtype, b.dtype)
            a, b = a.to(dt), b.to(dt)
        _check_bin_dims(a, b, op)
        return fn(a, b)
    if ta:
        return fn(cvt(a), _num(b))
    return fn(_num(a), cvt(b))


# ----------------------------------------------------------------------------
# unary cellwise
# ----------------------------------------------------------------------------
def _round(x):
    return torch.floor(x + 0.5)


UN = {
    "neg": lambda x: -x,
    "not": lambda x: (x == 0).to(x.dtype),
    "abs": torch.abs,
    "exp": torch.exp,
    "log": torch.log,
    "sqrt": torch.sqrt,
    "round": _round,
    "floor": torch.floor,
    "ceil": torch.ceil,
    "sign": torch.sign,
    "sin": torch.sin, "cos": torch.cos, "tan": torch.tan,
    "asin": torch.asin, "acos": torch.acos, "atan": torch.atan,
    "sinh": torch.sinh, "cosh": torch.cosh, "tanh": torch.tanh,
    "cumsum": lambda x: _cum("cumsum", x),
    "cumprod": lambda x: _cum("cumprod", x),
    "cummin": lambda x: _cum("cummin", x),
    "cummax": lambda x: _cum("cummax", x),
    "sigmoid": torch.sigmoid,
}

_CUM_HOST = {
    "cumsum": lambda x: torch.cumsum(x, dim=0),
    "cumprod": lambda x: torch.cumprod(x, dim=0),
    "cummin": lambda x: torch.cummin(x, dim=0).values,
    "cummax": lambda x: torch.cummax(x, dim=0).values,
}


def _cum(op, x):
    """Column-wise cumulative aggregates: device matrices take the chunked HIP scan
    (ops/hip/scan.hip), host matrices torch's."""
    if x.is_cuda and backend.use_kernels:
        from . import kernels
        return kernels.cumagg(op, x)
    return _CUM_HOST[op](x)


def unary(op, x):
    if type(x) is _CC:
        return AUG.unary(op, x)
    if type(x) is DevScalar:
        return _dev_unary(op, x)
    if CMP.is_compressed(x):
        if op in ("nrow", "ncol", "length"):
            r, c = x.shape
            return {"nrow": r, "ncol": c, "length": r * c}[op]
        x = x.decompress()
    if isinstance(x, Tensor):
        if op in ("nrow", "ncol", "length"):
            r, c = x.shape
            return {"nrow": r, "ncol": c, "length": r * c}[op]
        if op == "cast_scalar" or op in ("cast_double", "cast_int", "cast_bool"):
            if x.numel() != 1:
                raise DMLRuntimeError(f"cannot cast {x.shape[0]}x{x.shape[1]} matrix to scalar")
            if backend.lazy and x.is_cuda and op in ("cast_scalar", "cast_double"):
                return DevScalar(cvt(x).reshape(()).to(torch.float64))
            v = float(x.reshape(-1)[0].item())
            return S.unary(op, v) if op != "cast_scalar" else v
        if op == "cast_matrix":
            return x
        if op == "cast_frame":
            from ..runtime.data import FrameBlock
            return FrameBlock.from_matrix(x)
        fn = UN.get(op)
        if fn is None:
            raise DMLRuntimeError(f"unknown unary operator {op}")
        if SP.is_sparse(x):
            r = SP.unary(op, x, fn)
            if r is not None:
                return r
            x = SP.densify(x)
        return fn(cvt(x))
    if is_dist(x):
        return _dist().unary(op, x)
    if op in ("nrow", "ncol", "length"):
        if hasattr(x, "columns"):
            r, c = x.shape
            return {"nrow": r, "ncol": c, "length": r * c}[op]
        if hasattr(x, "data") and hasattr(x, "names"):
            return len(x) if op == "length" else (len(x) if op == "nrow" else 1)
        if op == "length":
            return 1
        raise DMLRuntimeError(f"{op}() requires a matrix or frame argument")
    if op == "cast_matrix":
        if hasattr(x, "columns"):
            return x.to_matrix(backend.dtype).to(backend.device)
        if hasattr(x, "data") and hasattr(x, "names"):
            vals = [float(v) for v in x.data]
            return torch.tensor(vals, dtype=backend.dtype, device=backend.device).reshape(-1, 1)
        return torch.full((1, 1), float(_num(x)), dtype=backend.dtype, device=backend.device)
    if op == "cast_frame":
        from ..runtime.data import FrameBlock
        if hasattr(x, "columns"):
            return x
        return FrameBlock([[x]], [S.vtype_of(x)])
    if op == "cast_scalar" and hasattr(x, "columns"):
        return x.columns[0][0]
    if op == "cast_list":
        from ..runtime.data import ListObject
        return x if hasattr(x, "names") and hasattr(x, "data") else ListObject([x])
    return S.unary(op, x)


# ----------------------------------------------------------------------------
# aggregates
# ----------------------------------------------------------------------------
def _var(x, dim=None):
    if dim is None:
        n = x.numel()
        if n <= 1:
            return torch.zeros((), dtype=x.dtype, device=x.device)
        return torch.var(x)
    n = x.shape[dim]
    if n <= 1:
        shape = list(x.shape)
        shape[dim] = 1
        return torch.zeros(shape, dtype=x.dtype, device=x.device)
    return torch.var(x, dim=dim, keepdim=True)


_COLSUM = []


def _colsum_kernel(x):
    from . import cell
    if not _COLSUM:
        _COLSUM.append(cell.CellProgram([], 1, 0, ("sum", "col")))
    return cell._kernel(_COLSUM[0], [x])


_KAGG = {"sum", "sumsq", "mean", "min", "max", "prod", "var", "sd", "imax", "imin"}


def agg(o, d, x):
    # fast path: dense host tensors (the CP backend's solver state) -- no representation checks
    if type(x) is Tensor and x.layout is _STRIDED and not x.is_cuda and x.dtype is not torch.bfloat16 \
            and x.numel() > 0:
        if d == "all":
            if o == "sum":
                return float(torch.sum(x))
            if o == "sumsq":
                return float(torch.sum(x * x))
        elif o == "sum":
            return torch.sum(x, dim=1 if d == "row" else 0, keepdim=True)
    if type(x) is _CC:
        return AUG.agg(o, d, x)
    if CMP.is_compressed(x):
        if o in ("sum", "sumsq", "mean"):
            sq = o == "sumsq"
            r, c = x.shape
            if d == "all":
                v = float(x.colsums(sq).sum().item())
                return v / (r * c) if o == "mean" else v
            out = x.rowsums(sq) if d == "row" else x.colsums(sq)
            return out / (c if d == "row" else r) if o == "mean" else out
        x = x.decompress()
    if isinstance(x, Tensor) and SP.is_sparse(x):
        r = SP.agg(o, d, x)
        if r is not None:
            return r
        x = SP.densify(x)
    if not isinstance(x, Tensor):
        if is_dist(x):
            return _dist().agg(o, d, x)
        if type(x) is DevScalar:
            x = x.value()
        if isinstance(x, (int, float, bool)):
            v = _num(x)
            if o in ("sum", "mean", "min", "max", "prod", "trace"):
                return float(v)
            if o == "sumsq":
                return float(v) * float(v)
            if o in ("var", "sd"):
                return 0.0
        raise DMLRuntimeError(f"aggregate {o} requires a matrix argument")
    if o == "sumsq" and backend.use_kernels and x.is_cuda and x.numel() >= 1 << 16 and d in ("all", "row", "col"):
        from . import kernels
        return kernels.sumsq(x, d)
    if o == "sum" and d == "col" and backend.use_kernels and x.is_cuda and x.shape[1] >= 2048 and x.shape[0] > 1:
        # wide column sums (e.g. the batch-norm channel sums): the generated column-aggregate
        # kernel (fp64 accumulation, 8 rows in flight per lane) instead of torch's strided reduction
        r = _colsum_kernel(x)
        if r is not None:
            return r
    if backend.use_kernels and x.is_cuda and x.layout is _STRIDED and x.numel() > 0 and o in _KAGG \
            and x.dim() == 2 and (d != "all" or o not in ("sum", "sumsq")):
        # the eager long tail on agg.hip (sum / sumsq over all cells mostly arrive fused)
        from . import kernels
        r = kernels.agg(o, d, x)
        if r is not None:
            return _lazy_out(r) if d == "all" else r
    x = cvt(x)
    if d == "all":
        if x.numel() == 0:
            if o in ("sum", "sumsq", "trace"):
                return 0.0
            raise DMLRuntimeError(f"aggregate {o} of an empty matrix")
        if o == "sum":
            r = torch.sum(x)
        elif o == "sumsq":
            r = torch.sum(x * x)
        elif o == "mean":
            r = torch.mean(x)
        elif o == "prod":
            r = torch.prod(x)
        elif o == "min":
            r = torch.min(x)
        elif o == "max":
            r = torch.max(x)
        elif o == "var":
            r = _var(x)
        elif o == "sd":
            r = torch.sqrt(_var(x))
        elif o == "trace":
            if x.shape[0] != x.shape[1]:
                raise DMLRuntimeError("trace requires a square matrix")
            r = torch.trace(x)
        else:
            raise DMLRuntimeError(f"unknown aggregate {o}")
        return _lazy_out(r)
    dim = 1 if d == "row" else 0
    if o == "sum":
        return torch.sum(x, dim=dim, keepdim=True)
    if o == "sumsq":
        return torch.sum(x * x, dim=dim, keepdim=True)
    if o == "mean":
        return torch.mean(x, dim=dim, keepdim=True)
    if o == "prod":
        return torch.prod(x, dim=dim, keepdim=True)
    if o == "min":
        return torch.amin(x, dim=dim, keepdim=True)
    if o == "max":
        return torch.amax(x, dim=dim, keepdim=True)
    if o == "var":
        return _var(x, dim)
    if o == "sd":
        return torch.sqrt(_var(x, dim))
    if o in ("imax", "imin"):
        # 1-based index of the (last) extreme value per row, as LibMatrixAgg
        xf = torch.flip(x, dims=[1])
        idx = torch.argmax(xf, dim=1, keepdim=True) if o == "imax" else torch.argmin(xf, dim=1, keepdim=True)
        return (x.shape[1] - idx).to(x.dtype)
    raise DMLRuntimeError(f"unknown aggregate {o}")


def tak(a, b):
    """sum(a*b) without materialising the product (TernaryAggregate tak+*)."""
    if type(a) is Tensor and type(b) is Tensor and a.layout is _STRIDED and b.layout is _STRIDED and \
            not a.is_cuda and not b.is_cuda and a.dtype is b.dtype and a.dtype is not torch.bfloat16 and \
            a.shape == b.shape:
        return float(torch.dot(a.reshape(-1), b.reshape(-1)))
    if is_dist(a) or is_dist(b):
        return _dist().tak(a, b)
    a, b = SP.densify(a), SP.densify(b)
    if not isinstance(a, Tensor) or not isinstance(b, Tensor):
        return agg("sum", "all", binary("*", a, b))
    a, b = SP.densify(a), SP.densify(b)
    if a.shape != b.shape:
        return agg("sum", "all", binary("*", a, b))
    a, b = cvt(a), cvt(b)
    if b.dtype != a.dtype:
        b = b.to(a.dtype)
    if a.device != b.device:
        b = b.to(a.device)
    if backend.use_kernels and a.is_cuda:
        from . import kernels
        r = kernels.dot(a, b)                   # agg.hip: one pass, fp64 accumulation
        if r is not None:
            return _lazy_out(r)
    return _lazy_out(torch.dot(a.reshape(-1), b.reshape(-1)))


# ----------------------------------------------------------------------------
# matrix multiplication family
# ----------------------------------------------------------------------------
def _need_mat(x, what):
    if not isinstance(x, Tensor):
        if is_dist(x):
            return x
        raise DMLRuntimeError(f"{what}: expected a matrix, got {type(x).__name__}")
    return x


def mm(a, b, transA=False):
    if type(a) is _CC or type(b) is _CC:
        if type(a) is _CC:
            return AUG.mm(a, b, transA)
        b = b.materialize()
    if is_dist(a) or is_dist(b):
        return _dist().mm(a, b, transA)
    if CMP.is_compressed(a):
        b = SP.densify(_need_mat(b, "%*%"))
        k = a.shape[0] if transA else a.shape[1]
        if k != b.shape[0]:
            raise DMLRuntimeError(f"Matrix multiplication dimension mismatch: {a.shape} %*% {tuple(b.shape)}")
        return a.tmatmul(cvt(b)) if transA else a.matmul(cvt(b))
    if CMP.is_compressed(b):
        b = b.decompress()
    a = _need_mat(a, "%*%")
    b = _need_mat(b, "%*%")
    if SP.is_sparse(a) or SP.is_sparse(b):
        ka = a.shape[0] if transA else a.shape[1]
        if ka != b.shape[0]:
            raise DMLRuntimeError(f"Matrix multiplication dimension mismatch: {a.shape} %*% {b.shape}")
        if SP.is_sparse(a):
            return SP.mm(cvt_sp(a), b, transA)
        return mm(cvt(a), SP.densify(b), transA)
    ka = a.shape[0] if transA else a.shape[1]
    if ka != b.shape[0]:
        ra, ca = (a.shape[1], a.shape[0]) if transA else tuple(a.shape)
        raise DMLRuntimeError(f"Matrix multiplication dimension mismatch: {ra}x{ca} %*% {b.shape[0]}x{b.shape[1]}")
    if backend.use_kernels and a.is_cuda:
        from . import kernels
        r = kernels.try_mm(a, b, transA)
        if r is not None:
            return r
    a, b = cvt(a), cvt(b)
    if a.device != b.device:
        b = b.to(a.device)
    if a.dtype != b.dtype:
        dt = torch.promote_types(a.dtype, b.dtype)
        a, b = a.to(dt), b.to(dt)
    return a.t() @ b if transA else a @ b


def tsmm(x, left=True):
    if type(x) is _CC:
        Xp = AUG.padded(x) if left else None
        if Xp is not None:
            D1 = x.X.shape[1] + 1
            return tsmm(Xp, True)[:D1, :D1]
        return AUG.tsmm(x, left)
    if is_dist(x):
        return _dist().tsmm(x, left)
    if CMP.is_compressed(x):
        x = x.decompress()
    x = _need_mat(x, "tsmm")
    if SP.is_sparse(x):
        return SP.tsmm(x, left)
    if backend.use_kernels and x.is_cuda:
        from . import kernels
        r = kernels.try_tsmm(x, left)
        if r is not None:
            return r
    x = cvt(x)
    return x.t() @ x if left else x @ x.t()


def mmchain(ctype, X, v, w=None):
    """t(X) %*% f(X %*% v) fused chains (MapMultChain + codegen row template)."""
    if type(X) is _CC:
        return AUG.mmchain(ctype, X, v, w)
    if is_dist(X):
        return _dist().mmchain(ctype, X, v, w)
    if backend.use_kernels and isinstance(X, Tensor) and X.is_cuda and not SP.is_sparse(X):
        from . import kernels
        r = kernels.try_mmchain(ctype, X, v, w)
        if r is not None:
            return r
    return mmchain_ref(ctype, X, v, w)


def smgrad(X, V, Y, cu=None):
    """Fused multinomial-logreg candidate evaluation: returns (U, G) with U = X %*% V and
    G = t(X) %*% (P[, 1:cu] - Y), P = row-softmax of cbind(U, 0)  (the row template the
    compiler forms from MultiLogReg's line-search step, see rewrites.fuse_softmax_grad)."""
    if type(X) is _CC:
        K = V.shape[1]
        return AUG.smgrad(X, V, Y, K if cu is None else int(S.as_double(cu)))
    if is_dist(X):
        return _dist().smgrad(X, V, Y, cu)
    K = V.shape[1] if hasattr(V, "shape") else None
    kc = K if cu is None else int(S.as_double(cu))
    if backend.use_kernels and isinstance(X, Tensor) and X.is_cuda and not SP.is_sparse(X) and kc == K \
            and isinstance(V, Tensor) and isinstance(Y, Tensor) and not SP.is_sparse(Y):
        from . import kernels
        r = kernels.smgrad(X, V, Y)
        if r is not None:
            return r
    return smgrad_ref(X, V, Y, kc)


def smobj(X, V, Y, cu=None, defer=False):
    """Fused multinomial-logreg candidate evaluation with the objective (compiler op `smobj`,
    rewrites.fuse_softmax_grad): with L = cbind(X %*% V, 0), LT = L - rowMaxs(L), E = exp(LT),
    returns (P, G, s1, s2): P = E / rowSums(E), G = t(X) %*% (P[, 1:cu] - Y[, 1:cu]),
    s1 = sum(Y * LT), s2 = sum(log(rowSums(E))) -- one pass over X on the MI355X."""
    K = V.shape[1] if hasattr(V, "shape") else None
    kc = K if cu is None else int(S.as_double(cu))
    if is_dist(X):
        return _dist().smobj(X, V, Y, kc)
    if type(X) is _CC and isinstance(V, Tensor):
        Xp = AUG.padded(X)            # cbind(X, 1) copy with 16-B rows: the one-pass kernel applies
        if Xp is not None:
            p, g, s1, s2 = smobj(Xp, AUG.padv(V.to(Xp.device), Xp.shape[1]), Y, cu)
            return p, g[:X.X.shape[1] + 1], s1, s2
    if type(X) is not _CC and backend.use_kernels and isinstance(X, Tensor) and X.is_cuda \
            and not SP.is_sparse(X) and kc == K and isinstance(V, Tensor) and isinstance(Y, Tensor) \
            and not SP.is_sparse(Y):
        from . import kernels
        r = kernels.smobj(X, V, Y, defer=defer)
        if r is not None:
            return r
    return smobj_ref(X, V, Y, kc)


def smobj_ref(X, V, Y, kc):
    if type(X) is _CC:
        u, _ = AUG.smgrad(X, V, rix(Y, None, None, 1, kc), kc)
    else:
        u = mm(X, V)
    lt = cvt(u) if not isinstance(u, Tensor) or SP.is_sparse(u) else u
    lt = torch.cat([lt, torch.zeros((lt.shape[0], 1), dtype=lt.dtype, device=lt.device)], dim=1)
    lt = lt - lt.max(dim=1, keepdim=True).values
    e = torch.exp(lt)
    rs = e.sum(dim=1, keepdim=True)
    p = e / rs
    Yd = cvt(SP.densify(Y)).to(device=lt.device, dtype=lt.dtype)
    s1 = float((Yd * lt).sum().item())
    s2 = float(torch.log(rs).sum().item())
    g = binary("-", p[:, :kc], Yd[:, :kc])
    return p, mm(X, g, transA=True), s1, s2


def smgrad_ref(X, V, Y, kc):
    u = mm(X, V)
    lt = cvt(u) if not isinstance(u, Tensor) or SP.is_sparse(u) else u
    lt = torch.cat([lt, torch.zeros((lt.shape[0], 1), dtype=lt.dtype, device=lt.device)], dim=1)
    lt = lt - lt.max(dim=1, keepdim=True).values
    e = torch.exp(lt)
    p = e / e.sum(dim=1, keepdim=True)
    g = binary("-", p[:, :kc], Y)
    return u, mm(X, g, transA=True)


def mmchain_ref(ctype, X, v, w=None):
    u = mm(X, v)
    if ctype == "XtXv":
        g = u
    elif ctype == "XtwXv":
        g = binary("*", w, u)
    elif ctype == "XtXvy":
        g = binary("-", u, w)
    elif ctype == "XtPSXv":
        q = binary("*", w, u)
        g = binary("-", q, binary("*", w, agg("sum", "row", q)))
    else:
        raise DMLRuntimeError(f"unknown mmchain type {ctype}")
    return mm(X, g, transA=True)


# ----------------------------------------------------------------------------
# reorg / indexing
# ----------------------------------------------------------------------------
def transpose(x):
    if type(x) is _CC:
        x = x.materialize()
    if is_dist(x):
        return _dist().transpose(x)
    if CMP.is_compressed(x):
        x = x.decompress()
    x = _need_mat(x, "t")
    if SP.is_sparse(x):
        return SP.transpose(x)
    if x.is_cuda and backend.use_kernels:
        # LDS-tiled transpose of the stored cells (bf16 stays bf16: the consumers widen it)
        from . import kernels
        r = kernels.transpose(x)
        if r is not None:
            return r
    return cvt(x).t().contiguous()


def _bound(v, default):
    if v is None:
        return default
    if isinstance(v, Tensor):
        v = v.reshape(-1)[0].item()
    return int(S.as_double(v)) if not isinstance(v, int) else v


def rix(x, rl, ru, cl, cu, list_mode=False):
    from ..runtime.data import ListObject, FrameBlock
    if isinstance(x, ListObject):
        if isinstance(rl, str):
            return x.get(rl)
        lo = _bound(rl, 1)
        hi = _bound(ru, len(x))
        if lo == hi and (ru is rl or ru is None or list_mode):
            return x.get(lo)
        return x.slice(lo, hi)
    if type(x) is _CC:
        return AUG.rix(x, rl, ru, cl, cu)
    if is_dist(x):
        return _dist().rix(x, rl, ru, cl, cu)
    if isinstance(x, FrameBlock):
        nr, nc = x.shape
        r0, r1 = _bound(rl, 1), _bound(ru, nr)
        c0, c1 = _bound(cl, 1), _bound(cu, nc)
        _check_range(r0, r1, c0, c1, nr, nc)
        return x.slice(r0 - 1, r1, c0 - 1, c1)
    if not isinstance(x, Tensor):
        if getattr(x, "is_part_view", False):           # parfor data partition (runtime/parfor.py)
            return x.part_rix(rl, ru, cl, cu)
        raise DMLRuntimeError("indexing requires a matrix, frame or list")
    nr, nc = x.shape
    r0, r1 = _bound(rl, 1), _bound(ru, nr)
    c0, c1 = _bound(cl, 1), _bound(cu, nc)
    _check_range(r0, r1, c0, c1, nr, nc)
    if x.is_cuda and backend.use_kernels:
        from . import kernels
        if SP.is_sparse(x) and x.layout == torch.sparse_csr:
            # slice_sparse_dense_row (SystemML.cu:301): the window of a CSR matrix as dense cells
            r = kernels.slice_csr(x, r0 - 1, r1, c0 - 1, c1)
            if r is not None:
                return r
        elif x.layout is _STRIDED and (r0, r1, c0, c1) == (1, nr, 1, nc):
            r = kernels.copy2d(x)           # the whole matrix: a copy (X[,] is a new value)
            if r is not None:
                return r
        # windows stay zero-copy views with a row pitch: the chain / row kernels read them in
        # place (e.g. P[, 1:K]); consumers that need dense rows copy them on reorg.hip
    out = x[r0 - 1:r1, c0 - 1:c1]
    return out.clone() if out.data_ptr() == x.data_ptr() and out.shape == x.shape else out


def _check_range(r0, r1, c0, c1, nr, nc):
    if r0 < 1 or r1 > nr or r0 > r1 or c0 < 1 or c1 > nc or c0 > c1:
        raise DMLRuntimeError(f"Invalid values for matrix indexing: [{r0}:{r1},{c0}:{c1}] "
                              f"must be within matrix dimensions [{nr},{nc}]")


def lix(x, y, rl, ru, cl, cu, list_mode=False, owned=None):
    """X[rl:ru, cl:cu] = y.  `owned` (update-in-place loops, compiler/loops.py): a WeakSet of
    buffers this loop execution already copied; those are modified in place, anything else is
    copied once and registered.  y may be a device-resident scalar (DevScalar): written into
    a device matrix without a host round trip."""
    from ..runtime.data import ListObject
    from ..runtime.scalars import DevScalar
    if type(y) is DevScalar and not (type(x) is Tensor and x.is_cuda and y.t.is_cuda):
        y = y.value()
    if isinstance(x, ListObject):
        i = _bound(rl, 1)
        data = list(x.data)
        names = list(x.names) if x.names else None
        if isinstance(rl, str):
            if names and rl in names:
                data[names.index(rl)] = y
            else:
                data.append(y)
                names = (names or [""] * (len(data) - 1)) + [rl]
        else:
            while len(data) < i:
                data.append(None)
            data[i - 1] = y
        return ListObject(data, names)
    if type(x) is _CC:
        x = x.materialize()
    if type(y) is _CC:
        y = y.materialize()
    if is_dist(x) or is_dist(y):
        return _dist().lix(x, y, rl, ru, cl, cu)
    if hasattr(x, "columns") and hasattr(x, "set_slice"):   # frame target
        nr, nc = x.shape
        r0, r1 = _bound(rl, 1), _bound(ru, nr)
        c0, c1 = _bound(cl, 1), _bound(cu, nc)
        _check_range(r0, r1, c0, c1, nr, nc)
        return x.set_slice(r0 - 1, r1, c0 - 1, c1, y.cpu() if isinstance(y, Tensor) else y)
    if not isinstance(x, Tensor):
        if getattr(x, "is_part_view", False):           # parfor data partition (runtime/parfor.py)
            return x.part_lix(y, rl, ru, cl, cu, owned=owned)
        raise DMLRuntimeError("left indexing requires a matrix target")
    nr, nc = x.shape
    r0, r1 = _bound(rl, 1), _bound(ru, nr)
    c0, c1 = _bound(cl, 1), _bound(cu, nc)
    _check_range(r0, r1, c0, c1, nr, nc)
    inplace = owned is not None and type(x) is Tensor and x.layout == torch.strided and x in owned and cvt(x) is x
    if backend.use_kernels and type(x) is Tensor and x.is_cuda and x.layout == torch.strided and x.dim() == 2:
        # one pass on reorg.hip: every output cell written once (or only the window, in place)
        xc = cvt(x).contiguous()
        yv = y
        if type(y) is DevScalar:
            out = xc if (inplace and xc is x) else torch.empty_like(xc)
            from . import kernels
            if kernels.lix(xc, None, out, r0 - 1, r1, c0 - 1, c1, sdev=y.t):
                if owned is not None and out is not x:
                    owned.add(out)
                return out
            y = yv = y.value()
        if isinstance(y, Tensor):
            yv = cvt(y)
            if tuple(yv.shape) != (r1 - r0 + 1, c1 - c0 + 1):
                if yv.numel() != 1:
                    raise DMLRuntimeError(f"left indexing dimension mismatch: target [{r0}:{r1},{c0}:{c1}] "
                                          f"vs source {yv.shape[0]}x{yv.shape[1]}")
                yv = float(yv.reshape(-1)[0].item())
        else:
            yv = float(_num(y))
        out = xc if (inplace and xc is x) else torch.empty_like(xc)
        from . import kernels
        if kernels.lix(xc, yv, out, r0 - 1, r1, c0 - 1, c1):
            if owned is not None and out is not x:
                owned.add(out)
            return out
    if inplace:
        out = x
    else:
        out = cvt(x).clone()
        if owned is not None and type(out) is Tensor:
            owned.add(out)
    if isinstance(y, Tensor):
        y = cvt(y)
        if tuple(y.shape) != (r1 - r0 + 1, c1 - c0 + 1):
            if y.numel() == 1:
                y = y.reshape(())
            else:
                raise DMLRuntimeError(f"left indexing dimension mismatch: target [{r0}:{r1},{c0}:{c1}] "
                                      f"vs source {y.shape[0]}x{y.shape[1]}")
        out[r0 - 1:r1, c0 - 1:c1] = y.to(device=out.device, dtype=out.dtype)
    else:
        out[r0 - 1:r1, c0 - 1:c1] = float(_num(y))
    return out
