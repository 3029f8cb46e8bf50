"""Loop rewrites on statement blocks (reference: hops/rewrite/
RewriteHoistLoopInvariantOperations.java — a StatementBlockRewriteRule).

Loop-invariant code motion: inside a while / for loop, a matrix-valued pure expression
whose inputs are literals or variables the loop never assigns computes the same value in
every iteration.  It is hoisted into a new basic block in front of the loop that assigns
a fresh variable (`_licm<n>`), and the loop body reads that variable instead.  Typical
case: `Pk = P[, 1:K]` inside MultiLogReg's inner CG loop re-slices an N x K matrix on every
Hessian-vector product; hoisted, it is sliced once per outer iteration, and the fused
`t(X) %*% (Q - Pk * rowSums(Q))` operator still sees one shared Pk input.

Only basic blocks directly in the loop body are scanned (not conditionally executed ones),
parfor bodies are left alone, and non-deterministic or side-effecting operators are never
moved.
"""
from __future__ import annotations

import itertools

from . import hops as H
from .hops import Hop
from .blocks import BasicBlock, IfBlock, WhileBlock, ForBlock

_names = itertools.count(1)
_NOT_PURE = {"fcall", "fout", "sink", "lix"}
_NO_HOIST_BI = H.NONDETERMINISTIC | H.SIDE_EFFECT | {"exists", "time", "eval", "list", "read", "print", "toString"}


def assigned_in(blocks):
    """Variables assigned anywhere in a block list (nested blocks included)."""
    out = set()
    for b in blocks:
        if isinstance(b, BasicBlock):
            out |= set(b.writes)
        elif isinstance(b, IfBlock):
            out |= assigned_in(b.then_blocks) | assigned_in(b.else_blocks)
        elif isinstance(b, (WhileBlock, ForBlock)):
            out |= assigned_in(b.body)
            if isinstance(b, ForBlock):
                out.add(b.var)
    return out


def _pure(h):
    if h.op in _NOT_PURE:
        return False
    if h.op in ("bi", "sink") and h.p.get("name") in _NO_HOIST_BI:
        return False
    return True


def _hoist_block(bb: BasicBlock, variant, stats):
    """Returns (new BasicBlock before the loop or None)."""
    inv = {}

    def invariant(h):
        r = inv.get(h.id)
        if r is not None:
            return r
        if h.op == "lit":
            r = True
        elif h.op == "tread":
            r = h.p["name"] not in variant
        else:
            r = _pure(h) and all(invariant(c) for c in h.inputs)
        inv[h.id] = r
        return r

    hoisted = {}          # hop id -> new tread hop
    pre_env = {}

    def worth(h):
        # never a bare transpose: t(X) feeding a variant product is folded into transA /
        # mmchain operators by the HOP rewrites, hoisting it would materialise it
        # nor a constant fill matrix(c, rows, cols): cheap, and rewrites match it by structure
        # (e.g. the outer product v %*% matrix(1, 1, k) that becomes a broadcast)
        if h.op == "bi" and h.p.get("name") in ("matrix", "seq") and all(c.dt == "S" or c.op == "lit"
                                                                        for c in h.inputs):
            return False
        return h.dt == "M" and h.op not in ("lit", "tread", "t")

    def visit(h, seen):
        if h.id in seen:
            return
        seen.add(h.id)
        for c in h.inputs:
            if c.id in hoisted:
                continue
            if invariant(c) and worth(c):
                hoist(c)
            else:
                visit(c, seen)

    def hoist(c):
        name = f"_licm{next(_names)}"
        pre_env[name] = c
        hoisted[c.id] = Hop("tread", p={"name": name}, dt="M", dim1=c.dim1, dim2=c.dim2, pos=c.pos)

    seen = set()
    for v in bb.env_out.values():        # an assigned value that is itself invariant
        if v.id not in hoisted and invariant(v) and worth(v):
            hoist(v)
    tops = [h for h in list(bb.roots) + list(bb.env_out.values()) if h.id not in hoisted]
    for h in tops:
        visit(h, seen)
    if not hoisted:
        return None
    # rewire the body DAG to the new transient reads
    done = set()

    def rewire(h):
        if h.id in done:
            return
        done.add(h.id)
        h.inputs = [hoisted.get(c.id, c) for c in h.inputs]
        for c in h.inputs:
            if c.op != "tread" or c.p["name"] not in pre_env:
                rewire(c)

    for h in tops:
        rewire(h)
    bb.env_out = {k: (hoisted.get(v.id, v)) for k, v in bb.env_out.items()}
    bb.reads |= set(pre_env)
    pre = BasicBlock()
    pre.pos = bb.pos
    pre.env_out = pre_env
    pre.writes = set(pre_env)
    reads = set()
    for h in H.walk(list(pre_env.values())):
        if h.op == "tread":
            reads.add(h.p["name"])
    pre.reads = reads
    stats["hoisted"] = stats.get("hoisted", 0) + len(pre_env)
    return pre


def hoist_loop_invariants(blocks, stats=None):
    """Apply LICM to a block list in place (recursively); returns the stats dict."""
    stats = {} if stats is None else stats
    i = 0
    while i < len(blocks):
        b = blocks[i]
        if isinstance(b, IfBlock):
            hoist_loop_invariants(b.then_blocks, stats)
            hoist_loop_invariants(b.else_blocks, stats)
        elif isinstance(b, (WhileBlock, ForBlock)):
            hoist_loop_invariants(b.body, stats)       # inner loops first
            if not (isinstance(b, ForBlock) and b.parfor):
                variant = assigned_in(b.body)
                if isinstance(b, ForBlock):
                    variant.add(b.var)
                pres = []
                for bb in b.body:
                    if isinstance(bb, BasicBlock):
                        pre = _hoist_block(bb, variant, stats)
                        if pre is not None:
                            pres.append(pre)
                if pres:
                    blocks[i:i] = pres
                    i += len(pres)
        i += 1
    return stats


def hoist_program(cp):
    stats = hoist_loop_invariants(cp.blocks)
    for fb in cp.functions.values():
        if fb.body is not None:
            hoist_loop_invariants(fb.body, stats)
    return stats
