"""Splitting basic blocks after data-dependent operators (reference: hops/rewrite/
RewriteSplitDagDataDependentOperators.java:67, a StatementBlockRewriteRule).

The output size of removeEmpty, of table / ctable without explicit dimensions and of eval
is known only once the operator has run.  Operators of the same basic block that consume
such a result are planned with unknown sizes -- exec type, physical operator and memory
estimate are guesses until dynamic recompilation, and recompilation happens per block.  The
block is therefore cut right after the operator: a first block computes it into a fresh
variable (`_sdag<n>`), the second block reads that variable and is recompiled when it
starts, with the exact size in hand (runtime/program.py -> compiler/cost.py).

A cut is skipped when it would repeat work or change results: the operator's inputs share a
computed (non-leaf) hop with the rest of the block, or its input DAG contains random
generators / side effects; and, as the reference's PMM flag, a table(seq(1, n), y) consumed
only as the left operand of %*% stays whole so the product remains a row gather.
"""
from __future__ import annotations

import itertools

from . import hops as H
from .hops import Hop
from .blocks import BasicBlock, IfBlock, WhileBlock, ForBlock

_names = itertools.count(1)
_BAD = H.NONDETERMINISTIC | H.SIDE_EFFECT


def _is_candidate(h):
    if h.op != "bi" or h.dt != "M":
        return False
    name = h.p.get("name")
    if name == "removeEmpty":
        return True
    if name in ("table", "ctable"):
        npos = h.p.get("npos", len(h.inputs) - len(h.named))
        return npos < 4 and not h.named           # output dimensions not given
    return name == "eval"


def _consumers(roots):
    cons = {}
    for h in H.walk(roots):
        for c in h.inputs:
            cons.setdefault(c.id, []).append(h)
    return cons


def _split(bb, stats):
    roots = list(bb.roots) + list(bb.env_out.values())
    cons = _consumers(roots)
    cands = []
    for h in H.walk(roots):
        if not _is_candidate(h):
            continue
        users = cons.get(h.id, [])
        if not users:
            continue                                    # only written to a variable: no consumer to re-plan
        if h.p.get("name") in ("table", "ctable") and all(u.op == "mm" and u.inputs[0] is h for u in users):
            continue                                    # permutation-matrix product (row gather)
        sub = H.walk([h])
        if any(x.op in ("fcall", "sink") or (x.op == "bi" and x.p.get("name") in _BAD) for x in sub):
            continue
        inside = {x.id for x in sub}
        shared = any(x.op not in ("lit", "tread") and x is not h and
                     any(u.id not in inside for u in cons.get(x.id, [])) for x in sub)
        if shared or any(c is not h and c.id in inside for c in cands):
            continue
        cands.append(h)
    if not cands:
        return None
    first = BasicBlock()
    first.pos = bb.pos
    repl = {}
    for h in cands:
        v = f"_sdag{next(_names)}"
        first.env_out[v] = h
        repl[h.id] = Hop("tread", p={"name": v}, dt="M", pos=h.pos)
    first.reads = {x.p["name"] for x in H.walk(list(first.env_out.values())) if x.op == "tread"}
    first.writes = set(first.env_out)
    # the rest of the block reads the cut variables instead
    memo = {}
    for x in H.walk(roots):
        if x.id in repl:
            memo[x.id] = repl[x.id]
            continue
        ins = [memo.get(c.id, c) for c in x.inputs]
        if any(a is not b for a, b in zip(ins, x.inputs)):
            x.inputs = ins                              # in place: identities of sinks / writes stay
        memo[x.id] = x
    bb.env_out = {k: memo.get(h.id, h) for k, h in bb.env_out.items()}
    bb.roots = [memo.get(h.id, h) for h in bb.roots]
    bb.reads = (set(bb.reads) - first.writes) | set(first.writes) | {
        x.p["name"] for x in H.walk(list(bb.roots) + list(bb.env_out.values())) if x.op == "tread"}
    stats["split-dag"] = stats.get("split-dag", 0) + len(cands)
    return [first, bb]


def run_blocks(blocks, stats):
    out = []
    for b in blocks:
        if isinstance(b, BasicBlock):
            r = _split(b, stats)
            out.extend(r if r is not None else [b])
            continue
        if isinstance(b, (WhileBlock, ForBlock)):
            b.body[:] = run_blocks(b.body, stats)
        elif isinstance(b, IfBlock):
            b.then_blocks[:] = run_blocks(b.then_blocks, stats)
            b.else_blocks[:] = run_blocks(b.else_blocks, stats)
        out.append(b)
    return out


def run(cp, config=None):
    stats = {}
    cp.blocks[:] = run_blocks(cp.blocks, stats)
    for fb in cp.functions.values():
        if fb.body is not None and not fb.external:
            fb.body[:] = run_blocks(fb.body, stats)
    return stats
