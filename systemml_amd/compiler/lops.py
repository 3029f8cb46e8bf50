"""Linearise HOP DAGs into flat instruction lists (the role of the LOP layer,
reference: lops/compile/Dag.java + hops/Hop.constructLops).

Each basic block becomes a list of ``Instr`` executing over a per-block slot
array.  Emission order follows statement order of the side-effecting roots
(prints, writes, stop, function calls) so observable behaviour matches the
reference, with every pure hop emitted lazily at its first use (post-order).
After its last use a slot is cleared so large intermediates are released from
HBM as early as possible (the reference's rmvar/cpvar bookkeeping).
"""
from __future__ import annotations

import threading

from .hops import walk
from .blocks import BasicBlock, IfBlock, WhileBlock, ForBlock, Predicate
from . import rewrites as RW


class Instr:
    __slots__ = ("fn", "ins", "out", "hop", "free", "opcode")

    def __init__(self, fn, ins, out, hop, opcode):
        self.fn = fn
        self.ins = ins
        self.out = out
        self.hop = hop
        self.free = ()
        self.opcode = opcode

    def __repr__(self):
        return f"{self.opcode} {list(self.ins)} -> {self.out}"


def _linearize(roots, tail_writes, make_impl):
    """roots: ordered hops to evaluate; tail_writes: list of (name, hop)."""
    order = []
    seen = set()
    for r in roots:
        for h in walk([r]):
            if h.id not in seen:
                seen.add(h.id)
                order.append(h)
    for _, h in tail_writes:
        for x in walk([h]):
            if x.id not in seen:
                seen.add(x.id)
                order.append(x)
    order = _launch_first(order)
    slot_of = {}
    instrs = []
    for i, h in enumerate(order):
        slot_of[h.id] = i
        fn, opcode = make_impl(h)
        instrs.append(Instr(fn, tuple(slot_of[c.id] for c in h.inputs), i, h, opcode))
    # last-use analysis (tail writes use slots at the very end)
    last = {}
    for idx, ins in enumerate(instrs):
        for s in ins.ins:
            last[s] = idx
    keep = {slot_of[h.id] for _, h in tail_writes}
    frees = {}
    for s, idx in last.items():
        if s in keep:
            continue
        frees.setdefault(idx, []).append(s)
    for idx, ins in enumerate(instrs):
        f = frees.get(idx)
        if f:
            ins.free = tuple(s for s in f if s != ins.out)
    writes = [(name, slot_of[h.id]) for name, h in tail_writes]
    return instrs, writes, len(order)


_HEAVY = {"mm", "tsmm", "mmchain", "smgrad", "smobj", "row", "wquat", "outer"}
_SIDE = {"sink", "fcall", "fout"}


def _launch_first(order):
    """Issue the block's big device operators (products, fused row / chain kernels) as early
    as their inputs allow, ahead of unrelated host scalar work: the GPU starts on the long
    kernel while the host interprets the rest of the block (e.g. a solver loop's counter
    updates and convergence bookkeeping).  Operators that depend on a side effect (calls,
    prints, random generators) keep their statement order."""
    if not any(h.op in _HEAVY for h in order):
        return order
    from .hops import NONDETERMINISTIC
    pos = {h.id: i for i, h in enumerate(order)}
    tainted = set()
    for h in order:
        if h.op in _SIDE or (h.op == "bi" and h.p.get("name") in NONDETERMINISTIC) or \
                any(c.id in tainted for c in h.inputs):
            tainted.add(h.id)
    out, done = [], set()

    def emit(h):
        stack = [(h, False)]
        while stack:
            x, ready = stack.pop()
            if x.id in done:
                continue
            if ready:
                done.add(x.id)
                out.append(x)
                continue
            stack.append((x, True))
            for c in sorted(x.inputs, key=lambda c: -pos.get(c.id, 0)):
                if c.id not in done:
                    stack.append((c, False))

    for h in order:
        if h.op in _HEAVY and h.id not in tainted:
            emit(h)
    for h in order:
        if h.id not in done:
            done.add(h.id)
            out.append(h)
    return out


_TLS = threading.local()    # .rw: rewrite counters of the program this thread compiles


def compile_basic_block(bb: BasicBlock, make_impl, config=None):
    st = RW.rewrite_block(bb, config)
    acc = getattr(_TLS, "rw", None)
    if acc is not None:
        for k, v in st.items():
            acc[k] = acc.get(k, 0) + v
    live = bb.live_out
    tail = []
    for name, h in bb.env_out.items():
        if live is None or name in live:
            if h.op == "tread" and h.p["name"] == name:
                continue     # x = x: nothing to write
            tail.append((name, h))
    bb.instrs, bb.writes_slots, bb.nslots = _linearize(bb.roots, tail, make_impl)
    # variable -> slot of its last assignment in this block (debugger symbol table)
    out_of = {ins.hop.id: ins.out for ins in bb.instrs}
    bb.debug_slots = {name: out_of[h.id] for name, h in bb.env_out.items() if h.id in out_of}


def compile_predicate(pred: Predicate, make_impl, config=None):
    RW.rewrite_pred(pred, config)
    instrs, _, n = _linearize([pred.root], [], make_impl)
    pred.instrs = instrs
    pred.nslots = n
    pred.out = n - 1


def compile_blocks(blocks, make_impl, config=None):
    for b in blocks:
        if isinstance(b, BasicBlock):
            compile_basic_block(b, make_impl, config)
        elif isinstance(b, IfBlock):
            compile_predicate(b.pred, make_impl, config)
            compile_blocks(b.then_blocks, make_impl, config)
            compile_blocks(b.else_blocks, make_impl, config)
        elif isinstance(b, WhileBlock):
            compile_predicate(b.pred, make_impl, config)
            compile_blocks(b.body, make_impl, config)
        elif isinstance(b, ForBlock):
            compile_predicate(b.start, make_impl, config)
            compile_predicate(b.end, make_impl, config)
            if b.incr is not None:
                compile_predicate(b.incr, make_impl, config)
            compile_blocks(b.body, make_impl, config)


def compile_program(cp, make_impl, config=None):
    prev = getattr(_TLS, "rw", None)
    _TLS.rw = acc = {}
    try:
        compile_blocks(cp.blocks, make_impl, config)
        for fb in cp.functions.values():
            if fb.body is not None:
                compile_blocks(fb.body, make_impl, config)
            for p in fb.default_preds.values():
                compile_predicate(p, make_impl, config)
        cp.rewrite_stats = acc           # -stats "rewrite <rule>" counters
    finally:
        _TLS.rw = prev
    return cp
