"""Instruction binding: HOP → executable closure (reference:
runtime/instructions/InstructionParser + cp/*CPInstruction, gpu/*GPUInstruction).

Each closure has the signature ``fn(ctx, args) -> value`` where ``args`` are the
already-evaluated input values.  Exec-type (host CP vs. HBM GPU vs. row-
partitioned DIST) is resolved by the operator library from where the operands
live, so the same instruction stream runs on every backend.
"""
from __future__ import annotations

import torch

from .bufferpool import Evicted

from ..parser.errors import DMLRuntimeError
from ..ops import core as C
from ..ops import sparse as SP
from . import builtins as B
from .scalars import DevScalar


_SPARSE_OK_OPS = {"lit", "tread", "fout", "fcall", "mm", "tsmm", "mmchain", "t", "agg", "b", "tak", "wquat", "cell",
                  "magg", "row", "outer", "vprog", "hcell"}
# builtins with their own CSR paths (the sparse-safe fused operators of compiler/rewrites.py)
_SPARSE_OK_BI = {"_nnz", "_minus_nz", "_log_nz"}
# operators computing directly on cbind(X, const) views (ops/augmented.ConstCol)
_CC_OK_OPS = {"b", "u", "agg", "mm", "tsmm", "mmchain", "smgrad", "smobj", "rix", "t", "cell", "magg", "row"}
_SPARSE_OK_UNARY = {"nrow", "ncol", "length", "cast_matrix", "abs", "sqrt", "round", "floor", "ceil", "sign",
                    "sin", "tan", "asin", "atan", "sinh", "tanh", "neg"}       # ops/sparse.py SAFE_UNARY
# operators that accept HBM-resident scalars (runtime/scalars.DevScalar) as operands; all others
# receive materialised Python values (one device sync)
_LAZY_OK_OPS = {"lit", "tread", "b", "u", "fcall", "fout", "mm", "tsmm", "mmchain", "smgrad", "smobj", "t", "tak",
                 "cell", "magg", "row", "outer", "vprog", "lix", "hcell"}
# operators that compute on matrix operands (placement applies); the rest move values around
_COMPUTE_OPS = {"b", "u", "agg", "mm", "tsmm", "mmchain", "smgrad", "smobj", "wquat", "tak", "t", "rix", "lix", "bi",
                 "cell", "magg", "row", "outer", "hcell"}
transfer_stats = {"h2d": 0, "d2h": 0, "h2d_bytes": 0, "d2h_bytes": 0}   # -stats (utils/stats.gpu_report)
_NO_PLACE_BI = {"print", "write", "stop", "assert", "printf", "list", "eval", "exists", "time", "toString",
                "read"}


def make_impl(h):
    """Instruction implementation; operators that have no sparse path receive densified
    operands (sparse matrices: ops/sparse.py), and compute operators run under the
    hybrid host/HBM placement of `_placed` on a GPU backend."""
    fn, code = _make_impl(h)
    if h.op in _COMPUTE_OPS and not (h.op == "bi" and h.p.get("name") in _NO_PLACE_BI):
        fn = _placed(fn, h)
    sparse_ok = h.op in _SPARSE_OK_OPS or (h.op == "u" and h.p.get("o") in _SPARSE_OK_UNARY) or \
        (h.op == "bi" and h.p.get("name") in _SPARSE_OK_BI)
    lazy_ok = h.op in _LAZY_OK_OPS
    if sparse_ok and lazy_ok:
        return fn, code
    if h.op in _CC_OK_OPS:
        # constant-column views (ops/augmented.py) are handled by these operators themselves
        def is_sp(x, _s=SP.is_special):
            return _s(x) and type(x).__name__ != "ConstCol"
    else:
        is_sp = SP.is_special
    dense = SP.densify
    DS = DevScalar

    if sparse_ok:
        def mat(ctx, a):
            # operators that need Python scalars: device-resident scalars are materialised here
            for x in a:
                if type(x) is DS:
                    return fn(ctx, [y.value() if type(y) is DS else y for y in a])
            return fn(ctx, a)
        return mat, code

    def wrapped(ctx, a):
        for x in a:
            if is_sp(x) or type(x) is DS:
                a = [dense(y) if is_sp(y) else (y.value() if type(y) is DS and not lazy_ok else y) for y in a]
                break
        return fn(ctx, a)
    return wrapped, code


# SYSML_RUNAHEAD_DEVICE=0: run-ahead iterations keep the host placement of small operators
_RA_DEVICE = __import__("os").environ.get("SYSML_RUNAHEAD_DEVICE", "1") != "0"


def _placed(fn, h):
    """CP / GPU execution of one operator by its compiler-chosen exec type (reference:
    hops/Hop.java#findExecTypeByMemEstimate with the GPU operator threshold, re-selected by
    dynamic recompilation when sizes were unknown at compile time -- compiler/cost.py):
      CP   operands in host memory, the operator runs on the CPU (a small op costs a few
           microseconds and its scalar results are available without a device sync);
      GPU  operands in HBM (host operands are copied over), HIP kernels;
      DIST row-partitioned operands, operators of parallel/dist.py (placement untouched).
    A small result computed in HBM (e.g. the D x K output of a fused t(X) %*% f(X %*% V)
    pass) is moved to host memory, where its consumers run."""
    import torch
    from ..ops.backend import backend
    Tensor = torch.Tensor

    keep_dev = bool(h.p.get("keep_dev"))    # read by a vector program (compiler/vecgen.py)

    def run(ctx, a):
        small = backend.small_cells
        if small <= 0 or not backend.on_gpu:
            return fn(ctx, a)
        if backend.defer and _RA_DEVICE:
            # a run-ahead loop iteration (runtime/program.py) is queued on the device behind
            # unread predicates: a host placement would synchronise in the middle of it (the
            # intercept scripts' D x K bookkeeping: 8 reads per CG iteration at icpt = 2), so
            # every operator runs in HBM, host operands (loop invariants) uploaded once
            a = [_upload(x) if (type(x) is Tensor and not x.is_cuda and x.layout == torch.strided) else x
                 for x in a]
            return fn(ctx, a)
        et = h.exec_type
        if keep_dev:
            if et == "CP":
                return fn(ctx, a)
            a = [h2d(x) if (type(x) is Tensor and not x.is_cuda) else x for x in a] if et == "GPU" else a
            return fn(ctx, a)
        if et == "CP":
            a = [d2h(x) if (type(x) is Tensor and x.is_cuda and x.layout == torch.strided) else x for x in a]
            return fn(ctx, a)
        if et == "GPU":
            a = [h2d(x) if (type(x) is Tensor and not x.is_cuda) else x for x in a]
            return demote(fn(ctx, a))
        # not decided (e.g. DIST operands or a block never recompiled): run where the largest
        # operand lives
        dev = None
        mixed = False
        for x in a:
            if type(x) is Tensor:
                d = x.device.type
            elif hasattr(x, "local") and type(getattr(x, "local", None)) is Tensor:
                d = x.local.device.type      # row-partitioned DistMatrix block
            else:
                continue
            if dev is None:
                dev = d
            elif d != dev:
                mixed = True
        if mixed:
            a = [h2d(x) if (type(x) is Tensor and x.device.type != "cuda") else x for x in a]
        return demote(fn(ctx, a))

    ts = transfer_stats

    def h2d(x):
        ts["h2d"] += 1
        ts["h2d_bytes"] += x.numel() * x.element_size()
        return x.to(backend.device, non_blocking=True)

    def _upload(x):
        from ..ops.vprog import _uploads
        ts["h2d"] += 1
        return _uploads.get(x, backend.device)

    def d2h(x):
        ts["d2h"] += 1
        ts["d2h_bytes"] += x.numel() * x.element_size()
        return x.to("cpu")

    def demote(r):
        if type(r) is tuple:                 # multi-output fused operators
            return tuple(demote(x) for x in r)
        if type(r) is Tensor and r.is_cuda and r.numel() < backend.small_cells and r.dtype != torch.bfloat16 \
                and not r.is_sparse and r.layout == torch.strided:
            return d2h(r)
        return r
    return run


class DeferredError:
    """Value of a variable whose (loop-invariant, hoisted) computation failed: the error is
    raised when the loop body first reads it, so a loop that never runs never fails
    (compiler/loops.py LICM)."""
    __slots__ = ("err",)

    def __init__(self, err):
        self.err = err


def _make_impl(h):
    op = h.op
    p = h.p
    if op == "lit":
        v = p["v"]
        return (lambda ctx, a: v), "lit"
    if op == "tread":
        name = p["name"]
        pos = h.pos

        def tread(ctx, a):
            try:
                v = ctx.vars[name]
            except KeyError:
                raise DMLRuntimeError(f"{pos}: Variable '{name}' is not defined" if pos else
                                      f"Variable '{name}' is not defined")
            if type(v) is DeferredError:
                raise v.err
            pool = ctx.pool
            if pool is not None:
                if type(v) is Evicted:
                    v = pool.restore(ctx.vars, name, v)
                pool.touch(ctx.vars, name)
            return v
        return tread, "tread"
    if op == "b":
        o = p["o"]
        f = C.binary
        return (lambda ctx, a: f(o, a[0], a[1])), o
    if op == "u":
        o = p["o"]
        f = C.unary
        return (lambda ctx, a: f(o, a[0])), o
    if op == "agg":
        o, d = p["o"], p["dir"]
        f = C.agg
        code = {"all": "ua", "row": "uar", "col": "uac"}[d] + o
        return (lambda ctx, a: f(o, d, a[0])), code
    if op == "mm":
        tA = p.get("transA", False)
        f = C.mm
        mv = p.get("mvagg")
        if mv:
            # product from simplifyColSums/RowSumsMVMult: when the "vector" turns out to be
            # 1x1 (a scalar-like broadcast against a matrix of more rows / columns), evaluate
            # the original colSums(X * v) / rowSums(X * v)
            def mvf(ctx, a):
                v, X = (a[0], a[1]) if mv == "col" else (a[1], a[0])
                vs, xs = tuple(v.shape), tuple(X.shape)
                n = xs[0] if mv == "col" else xs[1]
                if vs == (1, 1) and n != 1:
                    vv = v if mv == "col" else C.transpose(v)
                    return C.agg("sum", mv, C.binary("*", X, vv))
                return f(a[0], a[1], tA)
            return mvf, ("ba+*T" if tA else "ba+*")
        return (lambda ctx, a: f(a[0], a[1], tA)), ("ba+*T" if tA else "ba+*")
    if op == "tsmm":
        left = p["left"]
        return (lambda ctx, a: C.tsmm(a[0], left)), "tsmm"
    if op == "mmchain":
        t = p["type"]
        return (lambda ctx, a: C.mmchain(t, a[0], a[1], a[2] if len(a) > 2 else None)), "mmchain-" + t
    if op == "smgrad":
        return (lambda ctx, a: C.smgrad(a[0], a[1], a[2], a[3] if len(a) > 3 else None)), "smgrad"
    if op == "smobj":
        return (lambda ctx, a: C.smobj(a[0], a[1], a[2], a[3] if len(a) > 3 else None)), "smobj"
    if op == "wquat":
        from ..ops import quaternary as Q
        return (lambda ctx, a: Q.execute(p, a)), "wquat-" + p["kind"]
    if op == "tak":
        return (lambda ctx, a: C.tak(a[0], a[1])), "tak+*"
    if op == "cell":
        # fused cellwise DAG (compiler/codegen.py): one ops/hip/cell.hip pass on the MI355X;
        # sparse / compressed / constant-column / distributed operands run the original
        # operators one by one (ops/cell.sequential)
        from ..ops import cell as CELL
        prog = p["prog"]
        return (lambda ctx, a: CELL.evaluate(prog, a)), "spoofCell"
    if op == "hcell":
        # horizontal Cell batch (compiler/codegen.batch_cells): n same-program updates, one launch
        from ..ops import cell as CELL
        bprog, bn = p["prog"], p["n"]
        return (lambda ctx, a: CELL.evaluate_batch(bprog, bn, a)), "spoofCellBatch"
    if op == "outer":
        # Outer-product template (compiler/codegen.fuse_outer): sampled at a sparse driver's
        # non-zeros (ops/outer.py)
        from ..ops import outer as OUTR
        oprog = p["prog"]
        return (lambda ctx, a: OUTR.evaluate(oprog, a)), "spoofOP"
    if op == "row":
        # generated Row template (compiler/codegen.fuse_rows): one ops/rowgen.py kernel
        from ..ops import rowgen as ROWG
        rprog = p["prog"]
        return (lambda ctx, a: ROWG.evaluate(rprog, a)), "spoofRA"
    if op == "vprog":
        # Vector template (compiler/vecgen.py): a block's small-matrix + scalar algebra as one
        # single-workgroup kernel, its original operators one by one elsewhere (ops/vprog.py)
        from ..ops import vprog as VP
        vprog_ = p["prog"]
        return (lambda ctx, a: VP.evaluate(vprog_, ctx, a)), "spoofVec"
    if op == "magg":
        # multi-aggregate template (compiler/codegen._multi_agg): a tuple of scalars, one pass
        from ..ops import cell as CELL
        mprog = p["prog"]
        return (lambda ctx, a: CELL.evaluate_multi(mprog, a)), "spoofMA"
    if op == "t":
        return (lambda ctx, a: C.transpose(a[0])), "r'"
    if op == "rix":
        lm = p.get("list", False)
        if p.get("copy"):
            # slice of an update-in-place variable: must not stay a view of its buffer
            def rix_copy(ctx, a):
                r = C.rix(a[0], a[1], a[2], a[3], a[4], lm)
                return r.clone() if type(r) is torch.Tensor else r
            return rix_copy, "rix"
        return (lambda ctx, a: C.rix(a[0], a[1], a[2], a[3], a[4], lm)), "rix"
    if op == "lix":
        lm = p.get("list", False)
        if p.get("inplace"):
            return (lambda ctx, a: C.lix(a[0], a[1], a[2], a[3], a[4], a[5], lm, owned=ctx.owned)), "lix-inplace"
        return (lambda ctx, a: C.lix(a[0], a[1], a[2], a[3], a[4], a[5], lm)), "lix"
    if op == "fout":
        i = p["i"]

        def fout(ctx, a):
            r = a[0]
            if not isinstance(r, tuple):
                if i == 0:
                    return r
                raise DMLRuntimeError("function returned fewer outputs than requested")
            if i >= len(r):
                raise DMLRuntimeError("function returned fewer outputs than requested")
            return r[i]
        return fout, "fout"
    if op == "fcall":
        fkey = p["fkey"]
        given = p["given"]
        from . import program as PR
        return (lambda ctx, a: PR.call_function(ctx, fkey, a, given)), f"fcall {fkey[1]}"
    if op in ("bi", "sink"):
        name = p["name"]
        if name == "exists":
            var = p.get("var")
            return (lambda ctx, a: var in ctx.vars), "exists"
        if name == "_vguard":
            # guard of an if-converted block (compiler/ifconv.py)
            from ..compiler.ifconv import MODE
            from ..ops.vprog import VMAX
            from ..ops.backend import backend as _be
            gvars = p.get("vars", ())
            gdef = p.get("defined", ())
            force = MODE == "force"

            def vguard(ctx, a):
                vs = ctx.vars
                for v in gdef:
                    if v not in vs:
                        return False
                if force:
                    return all(v in vs for v in gvars)
                if not _be.on_gpu:
                    return False
                for v in gvars:
                    x = vs.get(v)
                    if type(x) is not torch.Tensor or x.numel() > VMAX or x.layout is not torch.strided:
                        return False
                return True
            return vguard, "vguard"
        if name == "eval":
            from . import program as PR
            npos = p.get("npos", len(h.inputs))
            named = list(h.named)
            nskey = p["nskey"]
            imports = dict(p["imports"])

            def ev(ctx, a):
                return PR.eval_call(ctx, a[0], list(a[1:npos]), dict(zip(named, a[npos:])), nskey, imports)
            return ev, "eval"
        fn = B.REGISTRY.get(name)
        if fn is None:
            pos = h.pos

            def missing(ctx, a):
                raise DMLRuntimeError(f"{pos}: unknown builtin function '{name}'")
            return missing, name
        npos = p.get("npos", len(h.inputs))
        named = list(h.named)
        if name in ("max_pool", "avg_pool", "max_pool_backward", "avg_pool_backward"):
            pass
        if not named:
            return (lambda ctx, a: fn(ctx, *a)), name
        return (lambda ctx, a: fn(ctx, *a[:npos], **dict(zip(named, a[npos:])))), name
    raise DMLRuntimeError(f"cannot bind instruction for hop {h!r}")
