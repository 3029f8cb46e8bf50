"""Size propagation, memory estimates, execution-type selection and the size-dependent
matrix-multiplication chain optimization (reference: hops/Hop.java refreshSizeInformation
/ computeMemEstimate / findExecTypeByMemEstimate, hops/OptimizerUtils.java,
hops/rewrite/RewriteMatrixMultChainOptimization.java, hops/recompile/Recompiler.java).

* `annotate(cp, input_shapes, config)` walks the program in statement order with the
  known dimensions of every live variable (inputs bound through MLContext / JMLC / the
  bench, or literals), infers the output dimensions of every HOP, attaches a worst-case
  dense memory estimate and picks an execution type:
      CP   scalars and matrices below `gpu_min_cells` (host memory, CPU operators)
      GPU  larger matrices on a GPU backend (HBM-resident, HIP kernels)
      DIST matrices with at least `dist_min_rows` rows in an SPMD run (row-partitioned)
  `-explain hops` prints the dimensions, estimates and exec types.
* Matrix-multiplication chains A1 %*% ... %*% An (n >= 3) whose dimensions are known are
  re-parenthesised by the classic O(n^3) dynamic program over the flop count, and the
  block is re-rewritten so the new shape can become fused operators (for example
  t(X) %*% X %*% v -> t(X) %*% (X %*% v) -> mmchain, never forming t(X) %*% X).
* Blocks whose chains have unknown dimensions at compile time are flagged for dynamic
  recompilation: runtime/program.py re-plans them at first execution from the actual
  operand shapes (`recompile_block`), cached per shape signature.
"""
from __future__ import annotations

from . import hops as H
from .hops import Hop
from .blocks import BasicBlock, IfBlock, WhileBlock, ForBlock

UNK = (-1, -1)
SCALAR = (0, 0)


_ABSENT = object()


def _lv(h):
    return h.value if h.op == "lit" else None


def _known(d):
    return d[0] >= 0 and d[1] >= 0


def _int_or(v, default=-1):
    if isinstance(v, bool) or v is None:
        return default
    if isinstance(v, (int, float)) and v == v and v >= 0:
        return int(v)
    return default


def _sval(h, dims, depth=0):
    """Compile-time value of a scalar hop when it follows from literals and known matrix
    sizes (nrow / ncol / length of a matrix whose dims are known, arithmetic on those) --
    reference: the size-expression evaluation of Hop.computeSizeInformation."""
    if h is None or depth > 8:
        return None
    if h.op == "lit":
        return h.value
    if h.op == "u" and h.p.get("o") in ("nrow", "ncol", "length") and h.inputs:
        d = dims.get(h.inputs[0].id, UNK)
        if _known(d):
            return {"nrow": d[0], "ncol": d[1], "length": d[0] * d[1]}[h.p["o"]]
        return None
    if h.op == "u" and h.p.get("o") in ("cast_int", "cast_double", "cast_scalar") and h.inputs:
        return _sval(h.inputs[0], dims, depth + 1)
    if h.op == "b" and h.p.get("o") in ("+", "-", "*", "/", "%/%") and len(h.inputs) == 2:
        a, b = _sval(h.inputs[0], dims, depth + 1), _sval(h.inputs[1], dims, depth + 1)
        if isinstance(a, (int, float)) and isinstance(b, (int, float)) and not isinstance(a, bool) \
                and not isinstance(b, bool):
            o = h.p["o"]
            if o in ("/", "%/%") and b == 0:
                return None
            return {"+": a + b, "-": a - b, "*": a * b, "/": a / b if o == "/" else a, "%/%": a // b if b else a}[o]
    return None


def infer(h, dims, env):
    """Output (rows, cols) of hop h given input dims; (0, 0) for scalars, -1 unknown."""
    op = h.op
    ins = [dims.get(c.id, UNK) for c in h.inputs]
    if op == "lit" or h.dt == "S":
        return SCALAR
    if op == "tread":
        return env.get(h.p["name"], UNK)
    if op == "b":
        a, b = ins
        if a == SCALAR:
            return b
        if b == SCALAR:
            return a
        if _known(a) and _known(b):
            return (max(a[0], b[0]), max(a[1], b[1]))
        return a if _known(a) else b
    if op == "u":
        o = h.p["o"]
        if o in ("nrow", "ncol", "length", "cast_scalar", "cast_double", "cast_int", "cast_bool"):
            return SCALAR
        if o == "cast_matrix":
            return (1, 1) if ins[0] == SCALAR else ins[0]
        return ins[0]
    if op == "cell":
        mats = [x for x in ins if x != SCALAR]
        if not mats or not all(_known(x) for x in mats):
            d = UNK
        else:
            from ..ops.cell import out_shape
            d = out_shape(h.p["prog"], [None if x == SCALAR else x for x in ins]) or UNK
        agg = h.p["prog"].agg
        if not agg:
            return d
        if agg[1] == "all":
            return SCALAR
        if d == UNK:
            return UNK
        return (d[0], 1) if agg[1] == "row" else (1, d[1])
    if op == "outer":
        prog = h.p["prog"]
        ot = prog.otype
        (m, _), (nn, _) = ins[0], ins[1]
        if ot == "all":
            return SCALAR
        if ot == "cell":
            return (m, nn)
        kb = ins[-1][1]
        return (m, kb) if ot == "left" else (nn, kb)
    if op == "hcell":
        return UNK                       # a tuple of outputs, read through fout hops
    if op == "row":
        from ..ops.rowgen import out_shape
        if h.p["prog"].more:
            return UNK                   # a tuple of outputs, read through fout hops
        if h.p["prog"].otype == "all":
            return SCALAR
        if not all(x == SCALAR or _known(x) for x in ins):
            return UNK
        s = out_shape(h.p["prog"], [None if x == SCALAR else x for x in ins])
        return UNK if s is None else s
    if op == "agg":
        r, c = ins[0]
        d = h.p["dir"]
        return SCALAR if d == "all" else ((r, 1) if d == "row" else (1, c))
    if op == "mm":
        (ra, ca), (rb, cb) = ins
        return (ca if h.p.get("transA") else ra, cb)
    if op == "tsmm":
        r, c = ins[0]
        return (c, c) if h.p.get("left") else (r, r)
    if op == "mmchain":
        return (ins[0][1], ins[1][1])
    if op == "tak":
        return SCALAR
    if op == "t":
        return (ins[0][1], ins[0][0])
    if op == "lix":
        return ins[0]
    if op == "rix":
        r, c = ins[0]
        # a bound is absent (literal None: whole range), a literal, or an expression (unknown)
        rl, ru, cl, cu = ((_ABSENT if (x.op == "lit" and x.value is None) else _lv(x)) for x in h.inputs[1:5])

        def span(lo, hi, n):
            if lo is _ABSENT and hi is _ABSENT:
                return n
            lo_ = 1 if lo is _ABSENT else _int_or(lo)
            hi_ = n if hi is _ABSENT else _int_or(hi)
            return hi_ - lo_ + 1 if lo_ >= 0 and hi_ >= 0 else -1
        lists = h.p.get("list", False)
        return (span(rl, ru, r), c if lists and cl is _ABSENT else span(cl, cu, c))
    if op == "bi":
        return _infer_bi(h, ins, dims)
    return UNK


def _bi_arg(h, i, name):
    npos = h.p.get("npos", len(h.inputs) - len(h.named))
    if i < npos:
        return h.inputs[i]
    if name in h.named:
        return h.inputs[npos + h.named.index(name)]
    return None


def _infer_bi(h, ins, dims=None):
    name = h.p.get("name")
    dims = dims or {}
    if name in ("matrix", "rand"):
        if name == "matrix":
            data = _bi_arg(h, 0, "data")
            r, c = _bi_arg(h, 1, "rows"), _bi_arg(h, 2, "cols")
        else:
            r, c = _bi_arg(h, 99, "rows"), _bi_arg(h, 99, "cols")
        rv = _int_or(_sval(r, dims)) if r is not None else -1
        cv = _int_or(_sval(c, dims)) if c is not None else -1
        return (rv, cv)
    if name == "seq":
        a, b = (_lv(x) for x in h.inputs[:2]) if len(h.inputs) >= 2 else (None, None)
        inc = _lv(h.inputs[2]) if len(h.inputs) > 2 else None
        if isinstance(a, (int, float)) and isinstance(b, (int, float)):
            inc = inc if isinstance(inc, (int, float)) and inc else (1 if b >= a else -1)
            return (int((b - a) / inc) + 1, 1)
        return (-1, 1)
    if name == "_cbind_const":
        r, c = ins[0]
        return (r, c + 1 if c >= 0 else -1)
    if name in ("cbind", "append"):
        if all(_known(d) for d in ins):
            return (ins[0][0], sum(d[1] for d in ins))
        return (ins[0][0] if ins else -1, -1)
    if name == "rbind":
        if all(_known(d) for d in ins):
            return (sum(d[0] for d in ins), ins[0][1])
        return (-1, ins[0][1] if ins else -1)
    if name == "diag":
        r, c = ins[0]
        if c == 1:
            return (r, r)
        return (r, 1) if r >= 0 else UNK
    if name == "solve":
        return (ins[0][1], ins[1][1])
    if name in ("inv", "inverse", "cholesky", "rev", "replace", "lower.tri", "upper.tri", "exp", "abs"):
        return ins[0]
    if name == "_onehot":
        return (_int_or(_lv(h.inputs[1])), _int_or(_lv(h.inputs[2])))
    if name == "outer":
        return (ins[0][0], ins[1][1])
    if name == "_seq_expand":
        return (ins[0][0], _int_or(_lv(h.inputs[1])))
    return UNK


# ----------------------------------------------------------------------------
def mem_estimate(d, bytes_per_cell=8):
    """Worst-case dense size in bytes of a matrix output; None when unknown."""
    if d == SCALAR:
        return 0
    if not _known(d):
        return None
    return d[0] * d[1] * bytes_per_cell


# SYSML_DIST_FORCE=1 (parallel/dist.py init): one-rank SPMD runs plan DIST like N > 1 ranks
_FORCE_DIST = __import__("os").environ.get("SYSML_DIST_FORCE") == "1"


def _world(config):
    w = getattr(config, "_world", None) if config is not None else None
    if w is None:
        from ..parallel import dist as D
        ctx = D.get_context()
        w = ctx.world if ctx is not None else 1
    return w


def exec_type(h, d, in_dims, config):
    """Execution type of a HOP (reference Hop.findExecTypeByMemEstimate): None when a matrix
    operand or the output has unknown dimensions -- decided at run time by dynamic
    recompilation (recompile_exec_types) from the actual shapes."""
    mats = [x for x in in_dims if x != SCALAR]
    if h.op == "sink" or ((h.dt == "S" or d == SCALAR) and not mats):
        return "CP"                          # scalar operations
    if d == SCALAR:
        d = (1, 1)                           # aggregate of matrices: placed by its operands
    if not _known(d) or any(not _known(x) for x in mats):
        return None
    gpu = config is not None and getattr(config, "gpu", False)
    world = _world(config) if config is not None else 1
    if config is not None and (world > 1 or _FORCE_DIST):
        if getattr(config, "dist_min_rows", 0) and d[0] >= config.dist_min_rows:
            return "DIST"
        budget = getattr(config, "gpu_mem_budget", 0)
        if budget and sum(x[0] * x[1] * 8 for x in [d] + list(in_dims) if _known(x)) > budget:
            return "DIST"
    cells = [x[0] * x[1] for x in [d] + list(in_dims) if _known(x)]
    small = getattr(config, "gpu_min_cells", 16384) if config is not None else 16384
    if gpu and max(cells or [0]) >= small:
        return "GPU"
    return "CP"


def physical_op(h, d, in_dims, et, config):
    """Physical operator of a matrix multiplication (reference AggBinaryOp.optFindMMultMethod*):
    DIST: mapmm (row-partitioned left, broadcast right), cpmm (co-partitioned t(X) %*% Y with
    an all-reduce), rmm (both row-partitioned: ring of the right operand's blocks), tsmm /
    mapmmchain (local fused kernel + all-reduce); GPU: MFMA GEMM, or a row-streaming kernel when
    the product is skinny (<= 8 columns) over a tall operand; CP: host GEMM."""
    if et is None or h.op not in ("mm", "tsmm", "mmchain", "smgrad", "smobj"):
        return None
    if h.op == "tsmm":
        return {"DIST": "tsmm+allreduce", "GPU": "mfma-tsmm", "CP": "cp-tsmm"}[et]
    if h.op in ("mmchain", "smgrad", "smobj"):
        return {"DIST": "mapmmchain+allreduce", "GPU": "rowstream-chain", "CP": "cp-chain"}[et]
    a, b = in_dims[0], in_dims[1]
    if et == "DIST":
        rows = getattr(config, "dist_min_rows", 1 << 62)
        if h.p.get("transA"):
            return "cpmm+allreduce"
        return "rmm-ring" if _known(b) and b[0] >= rows else "mapmm"
    if et == "GPU":
        return "rowstream-skinny" if _known(d) and d[1] <= 8 and a[0] >= 2048 else "mfma-gemm"
    return "cp-gemm"


def annotate_dag(roots, env, config=None):
    """Infer dims for a DAG (mutating hop.dim1/dim2, .exec_type, .mem); returns id -> dims."""
    dims = {}
    for h in H.walk(roots):
        d = infer(h, dims, env)
        if d == UNK and h.dim1 >= 0 and h.dim2 >= 0:
            d = (h.dim1, h.dim2)
        dims[h.id] = d
        h.dim1, h.dim2 = d
        ind = [dims.get(c.id, UNK) for c in h.inputs]
        h.exec_type = exec_type(h, d, ind, config)
        h.phys = physical_op(h, d, ind, h.exec_type, config)
    return dims


# ----------------------------------------------------------------------------
# matrix multiplication chains
# ----------------------------------------------------------------------------
def _chain_operands(h, consumers):
    """Flatten a left/right-nested tree of plain mm hops into its operand list."""
    ops = []

    def rec(x, top):
        if x.op == "mm" and not x.p.get("transA") and not x.p.get("mvagg") and (top or consumers.get(x.id, 0) <= 1):
            rec(x.inputs[0], False)
            rec(x.inputs[1], False)
        else:
            ops.append(x)
    rec(h, True)
    return ops


def mmchain_order(dimsv):
    """Classic DP: dimsv = [d0, d1, ..., dn] for n matrices; returns split table."""
    n = len(dimsv) - 1
    cost = [[0.0] * n for _ in range(n)]
    split = [[0] * n for _ in range(n)]
    for ln in range(1, n):
        for i in range(n - ln):
            j = i + ln
            best = None
            for k in range(i, j):
                c = cost[i][k] + cost[k + 1][j] + float(dimsv[i]) * dimsv[k + 1] * dimsv[j + 1]
                if best is None or c < best:
                    best, split[i][j] = c, k
            cost[i][j] = best
    return split, cost[0][n - 1] if n > 1 else 0.0


def _build(ops, split, i, j, pos):
    if i == j:
        return ops[i]
    k = split[i][j]
    return Hop("mm", [_build(ops, split, i, k, pos), _build(ops, split, k + 1, j, pos)], {}, dt="M", pos=pos)


def _tree_cost(h, dims, consumers):
    """Flops of the current parenthesisation of a chain rooted at h."""
    if h.op == "mm" and not h.p.get("transA") and not h.p.get("mvagg") and consumers.get(h.id, 0) <= 1:
        a, b = h.inputs
        (ra, ca), (_, cb) = dims[a.id], dims[b.id]
        return _tree_cost(a, dims, consumers) + _tree_cost(b, dims, consumers) + float(ra) * ca * cb
    return 0.0


def optimize_mm_chains(roots, env, stats):
    """Re-parenthesise mm chains of >= 3 operands with known dims. Returns (roots, changed,
    has_unknown_chain)."""
    dims = annotate_dag(roots, env)
    consumers = {}
    for h in H.walk(roots):
        for c in h.inputs:
            consumers[c.id] = consumers.get(c.id, 0) + 1
    memo = {}
    changed = False
    unknown = False

    def rec(h):
        nonlocal changed, unknown
        r = memo.get(h.id)
        if r is not None:
            return r
        if h.op == "mm" and not h.p.get("transA") and not h.p.get("mvagg"):
            ops = _chain_operands(h, consumers)
            if len(ops) >= 3:
                ods = [dims.get(o.id, UNK) for o in ops]
                if all(_known(d) and d != SCALAR for d in ods):
                    dv = [ods[0][0]] + [d[1] for d in ods]
                    split, best = mmchain_order(dv)
                    if best < _tree_cost(h, dims, consumers) * 0.999:
                        new_ops = [rec(o) for o in ops]
                        nh = _build(new_ops, split, 0, len(ops) - 1, h.pos)
                        memo[h.id] = nh
                        changed = True
                        stats["mmchain_reorder"] = stats.get("mmchain_reorder", 0) + 1
                        return nh
                else:
                    unknown = True
        h.inputs = [rec(c) for c in h.inputs]
        memo[h.id] = h
        return h

    new_roots = [rec(h) for h in roots]
    return new_roots, changed, unknown, memo


def _chain_block(bb, env, stats):
    tops = list(bb.roots) + list(bb.env_out.values())
    _, changed, unknown, memo = optimize_mm_chains(tops, env, stats)
    if changed:
        bb.roots = [memo.get(h.id, h) for h in bb.roots]
        bb.env_out = {k: memo.get(v.id, v) for k, v in bb.env_out.items()}
    return changed, unknown


# ----------------------------------------------------------------------------
# program-level pass
# ----------------------------------------------------------------------------
_SCALAR_TYPES = (bool, int, float, str)


import torch as _torch
_Tensor = _torch.Tensor


def _shape_of(v):
    tv = type(v)
    if tv is _Tensor:
        sh = v.shape
        return (sh[0], sh[1]) if len(sh) == 2 else UNK
    if tv in _SCALAR_TYPES:
        return SCALAR
    if isinstance(v, _SCALAR_TYPES) or getattr(v, "is_dev_scalar", False):
        return SCALAR
    sh = getattr(v, "shape", None)
    if sh is not None and len(sh) == 2:
        return (int(sh[0]), int(sh[1]))
    return UNK


def _deep_copy(roots, env_out):
    import copy
    memo = {}

    def cp_(h):
        r = memo.get(h.id)
        if r is None:
            r = copy.copy(h)
            r.inputs = [cp_(c) for c in h.inputs]
            memo[h.id] = r
        return r
    return [cp_(h) for h in roots], {k: cp_(v) for k, v in env_out.items()}


def _walk_program(cp, env, visit_bb):
    """Size propagation over the program: each basic block is visited with the shapes of the
    variables live into it; loops and branches merge shapes (unknown when they differ).
    Function bodies are visited with their parameters' shapes when every call site agrees on
    them (reference hops/ipa/FunctionCallSizeInfo.java): call sites in the main program outside
    loops, where the argument shapes are exact; otherwise the parameters are unknown and the
    body is planned at run time."""
    from .loops import assigned_in
    sites = {}           # function key -> list of {param: shape} (None: a site we cannot size)

    def record_calls(b, dims, exact):
        for h in H.walk(list(b.roots) + list(b.env_out.values())):
            if h.op != "fcall":
                continue
            k = h.p.get("fkey")
            given = list(h.p.get("given", ()))
            if not exact or len(given) != len(h.inputs):
                sites.setdefault(k, []).append(None)
            else:
                sites.setdefault(k, []).append({n: dims.get(a.id, UNK) for n, a in zip(given, h.inputs)})

    def blocks(bl, env, exact):
        for b in bl:
            if isinstance(b, BasicBlock):
                dims = visit_bb(b, env)
                record_calls(b, dims, exact)
                for k, h in b.env_out.items():
                    env[k] = dims.get(h.id, UNK)
            elif isinstance(b, IfBlock):
                e1, e2 = dict(env), dict(env)
                blocks(b.then_blocks, e1, exact)
                blocks(b.else_blocks, e2, exact)
                for k in set(e1) | set(e2):
                    env[k] = e1.get(k, UNK) if e1.get(k, UNK) == e2.get(k, UNK) else UNK
            elif isinstance(b, (WhileBlock, ForBlock)):
                if isinstance(b, ForBlock):
                    env[b.var] = SCALAR
                body_env = dict(env)
                blocks(b.body, body_env, False)
                for k in assigned_in(b.body):
                    if body_env.get(k, UNK) != env.get(k, UNK):
                        env[k] = UNK
    blocks(cp.blocks, env, True)
    for key, fb in cp.functions.items():
        if fb.body is not None:
            fenv = {p.name: (SCALAR if p.dtype == "SCALAR" else UNK) for p in fb.inputs}
            ss = sites.get(key)
            if ss and all(x is not None for x in ss) and not getattr(fb, "recursive", False):
                for p in fb.inputs:
                    shapes = {x.get(p.name, UNK) for x in ss}
                    if p.dtype != "SCALAR" and len(shapes) == 1:
                        sh = shapes.pop()
                        if _known(sh) and sh != SCALAR:
                            fenv[p.name] = sh
                            if not hasattr(cp, "fcall_sized"):
                                cp.fcall_sized = set()
                            cp.fcall_sized.add((key, p.name))
            blocks(fb.body, fenv, False)


def reorder_chains(cp, inputs=None):
    """Before the HOP rewrites: re-parenthesise mm chains with known dims; flag blocks whose
    chains have unknown dims for dynamic recompilation (keeping their raw DAG)."""
    stats = {}
    env = {k: _shape_of(v) for k, v in (inputs or {}).items()}

    def visit(bb, env):
        changed, unknown = _chain_block(bb, env, stats)
        if unknown:
            bb.recompile = True
            bb._raw = _deep_copy(list(bb.roots), dict(bb.env_out))
            stats["recompile_blocks"] = stats.get("recompile_blocks", 0) + 1
        return annotate_dag(list(bb.roots) + list(bb.env_out.values()), env)

    _walk_program(cp, env, visit)
    cp.chain_stats = stats
    return stats


def _check_dims(roots, dims):
    """Known-dimension validation of unconditional code (reference BinaryExpression /
    AggBinaryOp validate): %*% inner dimensions, cellwise operand shapes."""
    from ..parser.errors import LanguageError
    exact = {}
    ok_bi = ("matrix", "rand", "seq", "cbind", "rbind", "append", "diag")
    for h in H.walk(roots):
        # dims that are certain within this block: literal-sized constructors and exact
        # shape-preserving / shape-computing operators over them (reads of variables from other
        # blocks are not trusted: their shape may depend on control flow)
        ins = [exact.get(c.id, UNK) for c in h.inputs]
        if h.op == "lit" or h.dt == "S":
            d = SCALAR
        elif h.op in ("b", "u", "t", "mm", "agg", "rix") or (h.op == "bi" and h.p.get("name") in ok_bi):
            if h.op == "u" and h.p.get("o", "").startswith("cast"):
                d = UNK
            elif h.op != "bi" and any(x == UNK for x in ins[:2]):
                d = UNK
            else:
                d = infer(h, exact, {})
        else:
            d = UNK
        exact[h.id] = d
    for h in H.walk(roots):
        if h.op not in ("mm", "b") or len(h.inputs) != 2:
            continue
        a, b = (exact.get(c.id, UNK) for c in h.inputs)
        if not (_known(a) and _known(b)) or a == SCALAR or b == SCALAR:
            continue
        if h.op == "mm":
            inner = a[0] if h.p.get("transA") else a[1]
            if inner != b[0]:
                ra, ca = (a[1], a[0]) if h.p.get("transA") else a
                raise LanguageError(f"{h.pos}: matrix multiplication dimension mismatch: "
                                    f"{ra}x{ca} %*% {b[0]}x{b[1]} (inner dimensions must match)")
        else:
            (ra, ca), (rb, cb) = a, b
            ok = (a == b or (ra == rb and (ca == 1 or cb == 1)) or (ca == cb and (ra == 1 or rb == 1))
                  or (ra == 1 and ca == 1) or (rb == 1 and cb == 1) or (ca == 1 and rb == 1)
                  or (ra == 1 and cb == 1))
            if not ok:
                raise LanguageError(f"{h.pos}: mismatch in dimensions for cellwise operator "
                                    f"'{h.p.get('o')}': {ra}x{ca} vs {rb}x{cb}")


def annotate(cp, inputs=None, config=None):
    """After instruction generation: dims, memory estimates and exec types of the final
    (rewritten) HOP DAGs, for -explain and the cost statistics."""
    env = {k: _shape_of(v) for k, v in (inputs or {}).items()}
    counts = {}

    def visit(bb, env):
        dims = annotate_dag(list(bb.roots) + list(bb.env_out.values()), env, config)
        if not getattr(bb, "cond", True):
            _check_dims(list(bb.roots) + list(bb.env_out.values()), dims)
        unknown = False
        for h in H.walk(list(bb.roots) + list(bb.env_out.values())):
            if h.op in ("lit", "tread"):
                continue
            if h.exec_type:
                counts[h.exec_type] = counts.get(h.exec_type, 0) + 1
            elif h.dt == "M":
                unknown = True
        # exec types left open (unknown sizes) are decided when the block runs
        bb.exec_recompile = unknown
        if unknown:
            counts["deferred"] = counts.get("deferred", 0) + 1
        return dims

    _walk_program(cp, env, visit)
    cp.exec_types = counts
    return counts


def recompile_block(bb, vars_, make_impl, config):
    """Dynamic recompilation (reference: Recompiler.recompileHopsDag): re-plan a flagged
    block's mm chains from the actual shapes of its live-in variables.  Plans are cached
    per shape signature; returns True when a re-planned instruction list is in use."""
    from .lops import compile_basic_block
    names = sorted(bb.reads)
    sig = tuple((n, _shape_of(vars_.get(n))) for n in names)
    cache = getattr(bb, "_plans", None)
    if cache is None:
        cache = bb._plans = {}
        bb._orig_plan = (bb.instrs, bb.writes_slots, bb.nslots, getattr(bb, "debug_slots", {}))
    plan = cache.get(sig)
    if plan is None:
        roots, env_out = _deep_copy(*bb._raw)
        tmp = BasicBlock()
        tmp.roots, tmp.env_out = roots, env_out
        tmp.live_out = bb.live_out
        changed, _ = _chain_block(tmp, dict(sig), {})
        if changed:
            compile_basic_block(tmp, make_impl, config)
            plan = (tmp.instrs, tmp.writes_slots, tmp.nslots, getattr(tmp, "debug_slots", {}))
        else:
            plan = bb._orig_plan
        cache[sig] = plan
    bb.instrs, bb.writes_slots, bb.nslots, bb.debug_slots = plan
    return plan is not bb._orig_plan


def recompile_exec_types(bb, vars_, config):
    """Dynamic recompilation of execution types (reference Recompiler.recompileHopsDag +
    Hop.refreshSizeInformation): re-infer the block's sizes from the actual shapes of its
    live-in variables and re-select every operator's exec type / physical operator.  Cached on
    the shape signature; returns True when the plan changed."""
    names = getattr(bb, "_et_names", None)
    if names is None:
        # scalar-typed reads carry no shape: leaving them out of the signature keeps the per-
        # execution check to the block's matrices (it runs once per block execution)
        dts = {}
        for h in H.walk(list(bb.roots) + list(bb.env_out.values())):
            if h.op == "tread":
                dts.setdefault(h.p.get("name"), set()).add(h.dt)
        names = bb._et_names = tuple(n for n in sorted(bb.reads) if dts.get(n) != {"S"})
    get = vars_.get
    sig = tuple(_shape_of(get(n)) for n in names)
    if getattr(bb, "_et_sig", None) == sig:
        return False
    bb._et_sig = sig
    # a function body is entered with a different shape signature per call site (every layer
    # of a network): the annotations of each signature are kept and re-applied
    cache = getattr(bb, "_et_cache", None)
    if cache is None:
        cache = bb._et_cache = {}
    saved = cache.get(sig)
    if saved is not None:
        for h, d1, d2, et, ph in saved:
            h.dim1, h.dim2, h.exec_type, h.phys = d1, d2, et, ph
        return True
    tops = list(bb.roots) + list(bb.env_out.values())
    annotate_dag(tops, dict(zip(names, sig)), config)
    if len(cache) < 256:
        cache[sig] = [(h, h.dim1, h.dim2, h.exec_type, h.phys) for h in H.walk(tops)]
    return True


def runtime_plan(bb, indent=""):
    """-explain recompile_runtime: the block's instructions with their exec types and
    physical operators after dynamic recompilation."""
    lines = []
    for ins in bb.instrs or []:
        h = ins.hop
        et = getattr(h, "exec_type", None) or "?"
        ph = getattr(h, "phys", None)
        dims = f" [{h.dim1}x{h.dim2}]" if h.dt == "M" else ""
        lines.append(f"{indent}{et:4s} {ins.opcode}{dims}" + (f" ({ph})" if ph else ""))
    return "\n".join(lines)
