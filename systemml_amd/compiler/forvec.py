"""For-loop vectorization (reference: hops/rewrite/RewriteForLoopVectorization.java:50, a
StatementBlockRewriteRule).

A for loop with increment 1 whose body is one basic block of a single cell-at-a-time
statement is replaced by the equivalent operation over the whole index range, evaluated
once instead of (b - a + 1) times -- each of those iterations being a separate round of
instruction dispatch, and on the GPU backend a kernel launch or a device round trip:

  for (i in a:b) { s = s + as.scalar(X[i, j]) }   ->  s = s + sum(X[a:b, j])
      (+, *, min, max -> sum, prod, min, max; rows or columns)
  for (i in a:b) { X[i, j] = f(Y[i, k], Z[i, l], s) }  ->  X[a:b, j] = f(Y[a:b, k], Z[a:b, l], s)
      (f cellwise: binary / unary operators, fused cell programs, loop-invariant scalars;
       the reference's vectorizeElementwiseBinary / Unary / IndexedCopy; X may be read at
       the written row or column only)

The replacement runs under `if (b >= a)` (a:b with b < a counts down in DML: the original
loop runs then) and assigns the loop variable its last value, as the loop would.  Anything else -- other
statements in the body, reads of the loop variable outside the index positions, X read at
another index -- keeps the loop.
"""
from __future__ import annotations

from . import hops as H
from .hops import Hop, lit
from .blocks import BasicBlock, IfBlock, WhileBlock, ForBlock, Predicate

_AGG = {"+": "sum", "*": "prod", "min": "min", "max": "max"}
_CELL_U = {"abs", "sqrt", "exp", "log", "round", "floor", "ceil", "sign", "sin", "cos", "tan", "asin", "acos",
           "atan", "sinh", "cosh", "tanh", "sigmoid", "neg", "not"}
_CELL_B = {"+", "-", "*", "/", "^", "%%", "%/%", "==", "!=", "<", "<=", ">", ">=", "&", "|", "min", "max", "xor",
           "log"}


def _is_var(h, name):
    return h.op == "tread" and h.p.get("name") == name


def _uses_var(h, name):
    return any(_is_var(x, name) for x in H.walk([h]))


def _index_leaf(h, iv):
    """('row' | 'col', matrix, other-dim lo, other-dim hi) for rix(M, i, i, c, c) /
    rix(M, r, r, i, i), else None."""
    if h.op != "rix" or h.p.get("list") or len(h.inputs) != 5:
        return None
    M, rl, ru, cl, cu = h.inputs
    if _is_var(rl, iv) and rl is ru and not _uses_var(cl, iv) and not _uses_var(cu, iv):
        return "row", M, cl, cu
    if _is_var(cl, iv) and cl is cu and not _uses_var(rl, iv) and not _uses_var(ru, iv):
        return "col", M, rl, ru
    return None


def _clone_pred(pred):
    memo = {}
    for h in H.walk([pred.root]):
        memo[h.id] = h if h.op in ("lit",) else Hop(h.op, [memo[c.id] for c in h.inputs], dict(h.p),
                                                      named=list(h.named), dt=h.dt, dim1=h.dim1, dim2=h.dim2,
                                                      pos=h.pos)
    return memo[pred.root.id]


def _ranged(kind, M, lo, hi, a, b, pos):
    if kind == "row":
        return Hop("rix", [M, a, b, lo, hi], {}, dt="M", pos=pos)
    return Hop("rix", [M, lo, hi, a, b], {}, dt="M", pos=pos)


def _scalar_agg(bb, iv, a, b):
    """s = s op as.scalar(X[i, j])  ->  s = s op agg(X[a:b, j])."""
    if bb.roots or len(bb.env_out) != 1:
        return None
    (s, h), = bb.env_out.items()
    if h.op != "b" or h.p.get("o") not in _AGG or h.dt != "S" or s == iv:
        return None
    x, y = h.inputs
    if not _is_var(x, s):
        x, y = y, x
    if not _is_var(x, s) or y.op != "u" or y.p.get("o") != "cast_scalar":
        return None
    leaf = _index_leaf(y.inputs[0], iv)
    if leaf is None:
        return None
    kind, M, lo, hi = leaf
    if _uses_var(M, iv) or _uses_var(M, s) or not (lo is hi or (lo.op == "lit" and hi.op == "lit" and lo.value == hi.value)):
        return None
    agg = Hop("agg", [_ranged(kind, M, lo, hi, a, b, h.pos)], {"o": _AGG[h.p["o"]], "dir": "all"}, dt="S", dim1=0,
              dim2=0, pos=h.pos)
    return {s: Hop("b", [x, agg], {"o": h.p["o"]}, dt="S", dim1=0, dim2=0, pos=h.pos)}


def _elementwise(bb, iv, a, b):
    """X[i, j] = f(Y[i, k], ..., s)  ->  X[a:b, j] = f(Y[a:b, k], ..., s)."""
    if bb.roots or len(bb.env_out) != 1:
        return None
    (X, h), = bb.env_out.items()
    if h.op != "lix" or h.p.get("list") or h.p.get("inplace") or len(h.inputs) != 6 or X == iv:
        return None
    tgt, rhs, rl, ru, cl, cu = h.inputs
    if not _is_var(tgt, X):
        return None
    if _is_var(rl, iv) and rl is ru and not _uses_var(cl, iv) and not _uses_var(cu, iv):
        kind, lo, hi = "row", cl, cu
    elif _is_var(cl, iv) and cl is cu and not _uses_var(rl, iv) and not _uses_var(ru, iv):
        kind, lo, hi = "col", rl, ru
    else:
        return None
    if _uses_var(lo, X) or _uses_var(hi, X):
        return None
    memo = {}
    ok = [True]

    def sub(n):
        r = memo.get(n.id)
        if r is not None:
            return r
        leaf = _index_leaf(n, iv)
        if leaf is not None:
            k, M, l2, h2 = leaf
            if k != kind or _uses_var(M, iv) or (_uses_var(M, X) and not _is_var(M, X)):
                ok[0] = False
                return n
            r = _ranged(kind, M, l2, h2, a, b, n.pos)
        elif n.op == "lit":
            r = n
        elif n.op == "tread":
            if n.p.get("name") in (iv, X):
                ok[0] = False
            r = n
        elif n.op == "u" and n.p.get("o") == "cast_scalar" and _index_leaf(n.inputs[0], iv) is not None:
            r = sub(n.inputs[0])           # the cell becomes a column / row of cells
        elif (n.op == "u" and n.p.get("o") in _CELL_U) or (n.op == "b" and n.p.get("o") in _CELL_B) or n.op == "cell":
            kids = [sub(c) for c in n.inputs]
            dt = "M" if any(k.dt == "M" for k in kids) else n.dt
            r = Hop(n.op, kids, dict(n.p), named=list(n.named), dt=dt, pos=n.pos)
        else:
            ok[0] = False
            r = n
        memo[n.id] = r
        return r

    new_rhs = sub(rhs)
    if not ok[0]:
        return None
    if kind == "row":
        nh = Hop("lix", [tgt, new_rhs, a, b, lo, hi], {}, dt="M", pos=h.pos)
    else:
        nh = Hop("lix", [tgt, new_rhs, lo, hi, a, b], {}, dt="M", pos=h.pos)
    return {X: nh}


def _vectorize(fb):
    if fb.parfor or len(fb.body) != 1 or not isinstance(fb.body[0], BasicBlock):
        return None
    if fb.incr is not None and not (fb.incr.is_const and fb.incr.const == 1):
        return None
    bb = fb.body[0]
    iv = fb.var
    a, b = _clone_pred(fb.start), _clone_pred(fb.end)
    env = _scalar_agg(bb, iv, a, b)
    kind = "scalar-aggregate"
    if env is None:
        env = _elementwise(bb, iv, a, b)
        kind = "elementwise"
    if env is None:
        return None
    nb = BasicBlock()
    env[iv] = b
    nb.env_out = env
    nb.reads = {h.p["name"] for h in H.walk(list(env.values())) if h.op == "tread"}
    nb.writes = set(env)
    nb.pos = fb.pos
    ga, gb = _clone_pred(fb.start), _clone_pred(fb.end)
    g = Hop("b", [gb, ga], {"o": ">="}, dt="S", dim1=0, dim2=0, pos=fb.pos)
    reads = set(fb.start.reads) | set(fb.end.reads)
    # a:b with b < a counts down in DML: that (rare) case keeps the loop
    return IfBlock(Predicate(g, reads), [nb], [fb], pos=fb.pos), kind


def run_blocks(blocks, stats):
    out = []
    for b in blocks:
        if isinstance(b, ForBlock):
            r = _vectorize(b)
            if r is not None:
                out.append(r[0])
                stats["for-loop-vectorization"] = stats.get("for-loop-vectorization", 0) + 1
                continue
            b.body = run_blocks(b.body, stats)
        elif isinstance(b, WhileBlock):
            b.body = run_blocks(b.body, stats)
        elif isinstance(b, IfBlock):
            b.then_blocks = run_blocks(b.then_blocks, stats)
            b.else_blocks = run_blocks(b.else_blocks, stats)
        out.append(b)
    return out


def run(cp, config=None):
    """Vectorize the program's eligible for loops (main program and function bodies)."""
    stats = {}
    cp.blocks[:] = run_blocks(cp.blocks, stats)       # in place: the translator holds the list
    for fb in cp.functions.values():
        if fb.body is not None and not fb.external:
            fb.body[:] = run_blocks(fb.body, stats)
    return stats
