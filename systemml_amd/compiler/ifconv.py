"""If-conversion of small branches (a statement-block rewrite; no reference counterpart --
the reference executes every IfProgramBlock as control flow, runtime/controlprogram/
IfProgramBlock.java, which on a GPU costs one device round trip for the predicate).

Inside a solver loop, a branch on a freshly computed scalar splits the iteration into
blocks and puts a device synchronisation in the middle of it -- truncated CG's
`if (sum(S_try ^ 2) <= delta2) {...} else {...}` (MultiLogReg.dml:216) between the
Hessian-vector product and the state update.  When both branches are pure and cheap
(cellwise operators, aggregates and scalar algebra: no prints, calls, products or
indexing), the IfBlock becomes straight-line code: both branches are evaluated and every
variable they assign takes `_sel(pred, then value, else value)` (a variable assigned on one
side keeps its previous value on the other; one dead after the if is dropped).  The result
is merged with the neighbouring basic blocks, so a CG iteration becomes ONE block whose
update tail the Vector template (compiler/vecgen.py) compiles into one kernel, with one
synchronisation for the loop predicate.

Evaluating both branches is only cheap for small state, which is only known at run time,
so the converted block is guarded: `if (_vguard(state vars)) {converted} else {original
blocks}`.  The guard holds on a GPU backend when every matrix the branches assign currently
holds at most VMAX cells (ops/vprog.py); CPU runs and big matrices take the original
control flow.  SYSML_IFCONV=0 disables the rewrite, =force makes the guard always true.

Evaluating the branch not taken can fail where the original program does not: a shape
mismatch valid only under the predicate (`if (nrow(A) == nrow(B)) {C = A + B}`), or a read of
a variable defined on one path only.  The converted block is pure (branches are cheap
expressions; neighbours with prints, writes, calls or random draws are not merged) and a
basic block assigns its variables only once all its instructions succeeded, so the runtime
answers any error of the converted block by running the original blocks instead
(runtime/program.py): the error, if any, is then the original program's.
"""
from __future__ import annotations

import os

from . import hops as H
from .hops import Hop
from .blocks import BasicBlock, IfBlock, WhileBlock, ForBlock, Predicate

MODE = os.environ.get("SYSML_IFCONV", "1")
_PURE_BI = {"ifelse", "_sel", "matrix"}
_OPS = {"lit", "tread", "b", "u", "agg", "tak"}


def _cheap(roots):
    for h in H.walk(roots):
        if h.op in _OPS:
            if h.op == "agg" and h.p.get("dir") != "all":
                return False
            continue
        if h.op == "bi" and h.p.get("name") in _PURE_BI and not (h.p.get("name") == "matrix" and h.named
                                                                   and "data" in h.named):
            continue
        return False
    return True


def _clone(roots, subst, treads):
    """Copy of the DAG under `roots`; reads of variables in `subst` become those hops, other
    reads one shared tread per name (`treads`)."""
    memo = {}
    for h in H.walk(roots):
        if h.op == "tread":
            n = h.p["name"]
            if n in subst:
                memo[h.id] = subst[n]
                continue
            t = treads.get(n)
            if t is None:
                t = treads[n] = Hop("tread", p=dict(h.p), dt=h.dt, dim1=h.dim1, dim2=h.dim2, pos=h.pos)
            memo[h.id] = t
        elif h.op == "lit":
            memo[h.id] = h
        else:
            memo[h.id] = Hop(h.op, [memo[c.id] for c in h.inputs], dict(h.p), named=list(h.named), dt=h.dt,
                             dim1=h.dim1, dim2=h.dim2, pos=h.pos)
    return memo


class _Seq:
    """A straight-line block under construction: env (var -> hop), roots, reads."""

    def __init__(self):
        self.env = {}
        self.roots = []
        self.reads = set()
        self.treads = {}
        self.pos = None

    def add_block(self, bb):
        memo = _clone(list(bb.roots) + list(bb.env_out.values()), self.env, self.treads)
        self.reads |= {n for n in bb.reads if n not in self.env}
        self.roots += [memo[h.id] for h in bb.roots]
        for k, h in bb.env_out.items():
            self.env[k] = memo[h.id]
        self.pos = self.pos or bb.pos

    def block(self):
        bb = BasicBlock()
        bb.roots = self.roots
        bb.env_out = dict(self.env)
        bb.reads = set(self.reads)
        bb.writes = set(self.env)
        bb.pos = self.pos
        return bb


def _pure(bb):
    """No side effects and no random draws: a neighbour merged into a converted block may be
    executed twice (the converted block, then the original blocks when it raises)."""
    for h in H.walk(list(bb.roots) + list(bb.env_out.values())):
        if h.op in ("sink", "fcall") or (h.op == "bi" and h.p.get("name") in (H.SIDE_EFFECT | H.NONDETERMINISTIC)):
            return False
        # an update-in-place left index changes its target buffer before a later error would
        # send execution to the original blocks, which then see the changed data
        if h.op == "lix" and h.p.get("inplace"):
            return False
    return True


def _tail_live(blocks):
    if not blocks:
        return None
    b = blocks[-1]
    if isinstance(b, BasicBlock):
        return b.live_out
    if isinstance(b, IfBlock):
        r = _tail_live(b.then_blocks)
        return r if r is not None else _tail_live(b.else_blocks)
    return None


def _branch(blocks, live_after):
    """One converted BasicBlock for a branch's block list, or None."""
    seq = _Seq()
    for b in blocks:
        if isinstance(b, BasicBlock):
            if not _cheap(list(b.roots) + list(b.env_out.values())) or b.roots:
                return None
            seq.add_block(b)
        elif isinstance(b, IfBlock):
            c = _convert(b, _tail_live(b.then_blocks) or _tail_live(b.else_blocks) or live_after)
            if c is None:
                return None
            seq.add_block(c[0])
        else:
            return None
    return seq.block()


def _convert(ib, live_after):
    """(converted BasicBlock, assigned matrix-or-unknown vars) of an IfBlock, or None."""
    if live_after is None or not _cheap([ib.pred.root]):
        return None
    T = _branch(ib.then_blocks, live_after)
    E = _branch(ib.else_blocks, live_after)
    if T is None or E is None:
        return None
    treads = {}
    pm = _clone([ib.pred.root], {}, treads)
    c = pm[ib.pred.root.id]
    tm = _clone(list(T.env_out.values()), {}, treads)
    em = _clone(list(E.env_out.values()), {}, treads)
    seq = _Seq()
    seq.treads = treads
    seq.reads = set(ib.pred.reads) | T.reads | E.reads
    state, onesided = [], []
    for v in sorted(T.writes | E.writes):
        if v not in live_after:
            continue
        if v in T.env_out and v in E.env_out:
            tv, ev = tm[T.env_out[v].id], em[E.env_out[v].id]
        else:
            old = treads.get(v)
            if old is None:
                src = T.env_out.get(v) or E.env_out.get(v)
                old = treads[v] = Hop("tread", p={"name": v}, dt=src.dt, pos=ib.pos)
            seq.reads.add(v)
            onesided.append(v)
            tv = tm[T.env_out[v].id] if v in T.env_out else old
            ev = em[E.env_out[v].id] if v in E.env_out else old
        dt = tv.dt if tv.dt == ev.dt else "U"
        if tv is ev:
            seq.env[v] = tv
        else:
            seq.env[v] = Hop("bi", [c, tv, ev], {"name": "_sel", "npos": 3}, dt=dt, pos=ib.pos)
        if dt != "S":
            state.append(v)
    seq.pos = ib.pos
    return seq.block(), (state, onesided)


def _guard(state, pos):
    """state = (matrix vars whose size decides, vars assigned on one side only: they keep their
    previous value on the other, so they must be defined)."""
    mats, onesided = state
    h = Hop("bi", [], {"name": "_vguard", "vars": tuple(mats), "defined": tuple(onesided)}, dt="S", pos=pos)
    return Predicate(h, set())


def _scan(blocks, stats):
    """Convert the outermost convertible if-blocks of a block list; nested lists of loops and
    of branches that stay control flow are scanned in turn."""
    for b in blocks:
        if isinstance(b, WhileBlock):
            b.body = _scan(b.body, stats)
        elif isinstance(b, ForBlock) and not b.parfor:
            b.body = _scan(b.body, stats)
    res = []
    k = 0
    while k < len(blocks):
        b = blocks[k]
        if isinstance(b, IfBlock) and not getattr(b, "vguard", False):
            live_after = _tail_live(b.then_blocks)
            if live_after is None:
                live_after = _tail_live(b.else_blocks)
            c = _convert(b, live_after) if live_after is not None else None
            if c is not None:
                conv, state = c
                orig = [b]
                seq = _Seq()
                prev = res[-1] if res and isinstance(res[-1], BasicBlock) and not getattr(res[-1], "licm_pre", False) \
                    and _pure(res[-1]) else None
                if prev is not None:
                    res.pop()
                    orig.insert(0, prev)
                    seq.add_block(prev)
                seq.add_block(conv)
                nxt = blocks[k + 1] if k + 1 < len(blocks) and isinstance(blocks[k + 1], BasicBlock) \
                    and _pure(blocks[k + 1]) else None
                if nxt is not None:
                    orig.append(nxt)
                    seq.add_block(nxt)
                    k += 1
                merged = seq.block()
                g = IfBlock(_guard(state, b.pos), [merged], orig, pos=b.pos)
                g.vguard = True
                res.append(g)
                stats["if-converted"] = stats.get("if-converted", 0) + 1
                k += 1
                continue
        if isinstance(b, IfBlock) and not getattr(b, "vguard", False):
            b.then_blocks = _scan(b.then_blocks, stats)
            b.else_blocks = _scan(b.else_blocks, stats)
        res.append(b)
        k += 1
    return res


def run(cp, config=None):
    """Convert the program's small pure if-blocks (main program and function bodies);
    liveness must be current (BasicBlock.live_out) and is recomputed by the caller."""
    if MODE == "0" or (config is not None and not (getattr(config, "rewrites", True)
                                                   and getattr(config, "fusion", True))):
        return {}
    stats = {}
    cp.blocks = _scan(cp.blocks, stats)
    for fb in cp.functions.values():
        if fb.body is not None and not fb.external:
            fb.body = _scan(fb.body, stats)
    return stats
