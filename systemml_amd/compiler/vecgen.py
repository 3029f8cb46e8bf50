"""Vector template: the small-matrix + scalar algebra of a basic block as one generated
single-workgroup kernel (ops/vprog.py).

Reference analogue: hops/codegen/SpoofCompiler with the Cell / MAgg templates fuses
cellwise operators and full aggregates of one size class; it never crosses an aggregate
into the scalar algebra that consumes it, so an iterative solver's update step stays a
chain of small operators and CP scalar instructions.  On the MI355X each of those is a
launch plus, for every scalar, a device round trip; this template instead takes

  * cellwise binary / unary operators and selects over matrices (and scalars),
  * full aggregates (sum, sumsq, min, max, mean) and sum(A * B [* C]) (`tak`),
  * the scalar operators that depend on those aggregates,

of one "epoch" of the DAG -- operators separated by no other (non-template) operator --
into one VProgram.  Grouping by epoch (the number of non-template operators on the longest
path from the block's inputs) keeps every group convex: no path leaves a group through
another operator and comes back.  Scalar operators that depend only on the block's inputs
stay host scalar instructions.  Operators with a known dimension above the program's cell
limit (the big data matrix and anything N-row) never join; unknown sizes are decided at
run time, where a program outside the kernel's scope runs its original operators.
"""
from __future__ import annotations

from . import hops as H
from .hops import Hop
from ..ops.cell import BIN_CODES, UN_CODES
from ..ops.vprog import VMAX, VProgram

_AGG = ("sum", "sumsq", "min", "max", "mean")
_SCALAR_BIN_OK = set(BIN_CODES) - {"%%", "%/%"}


_DNN = {"conv2d", "conv2d_backward_data", "conv2d_backward_filter", "max_pool", "avg_pool", "max_pool_backward",
        "avg_pool_backward", "bias_add", "bias_multiply", "relu_backward"}


def _big(h, act=frozenset()):
    d1, d2 = h.dim1, h.dim2
    return (d1 > VMAX) or (d2 > VMAX) or (d1 >= 0 and d2 >= 0 and d1 * d2 > VMAX) or h.id in act


def _activations(order):
    """Ids of the block's DL activations / gradients: the values of DNN builtins and the
    cellwise operators over them.  Their sizes are only known at run time, but they are never
    single-workgroup vectors, so they stay with the Cell template (which fuses them with their
    neighbours) instead of joining a vector program whose run-time guard would send them to
    the one-region fallback."""
    act = set()
    for h in order:
        if h.dt != "M":
            continue
        if h.op == "bi" and h.p.get("name") in _DNN:
            act.add(h.id)
        elif h.op in ("b", "u") and any(c.id in act and c.dt == "M" for c in h.inputs):
            act.add(h.id)
    return frozenset(act)


def _stringy(h, memo):
    """Statically string-valued scalar (a string literal or a concatenation with one)."""
    r = memo.get(h.id)
    if r is not None:
        return r
    if h.op == "lit":
        r = isinstance(h.value, str)
    elif h.op == "b" and h.p.get("o") == "+":
        r = any(_stringy(c, memo) for c in h.inputs)
    elif h.op == "bi" and h.p.get("name") in ("toString", "append"):
        r = True
    else:
        r = False
    memo[h.id] = r
    return r


def _kind(h, smemo):
    """('m' | 's' | 'r', op) when h can join a vector program, else None."""
    act = smemo.get("__act", frozenset())
    if h.dt not in ("M", "S") or _big(h, act):
        return None
    op = h.op
    if op == "b" and len(h.inputs) == 2:
        o = h.p.get("o")
        if any(c.dt not in ("M", "S") for c in h.inputs) or _stringy(h, smemo):
            return None
        if h.dt == "M":
            return ("m", o) if o in BIN_CODES else None
        return ("s", o) if o in _SCALAR_BIN_OK else None
    if op == "u" and len(h.inputs) == 1:
        o = h.p.get("o")
        if o not in UN_CODES or h.inputs[0].dt != h.dt:
            return None
        return ("m" if h.dt == "M" else "s", o)
    if op == "agg" and len(h.inputs) == 1 and h.p.get("dir") == "all" and h.p.get("o") in _AGG \
            and h.inputs[0].dt == "M" and not _big(h.inputs[0], act):
        return ("r", h.p["o"])
    if op == "tak" and len(h.inputs) in (2, 3) and all(c.dt == "M" and not _big(c, act) for c in h.inputs):
        return ("r", "dot" if len(h.inputs) == 2 else "dot3")
    if op == "bi" and h.p.get("name") in ("ifelse", "_sel") and len(h.inputs) == 3 and not h.named:
        if any(c.dt not in ("M", "S") for c in h.inputs):
            return None
        if h.dt == "S" and h.inputs[0].dt == "M":
            return None
        return ("m" if h.dt == "M" else "s", "sel")
    return None


_names = iter(range(1 << 62))


def fuse_vectors(bb):
    """Replace the vector regions of a basic block by `vprog` hops; returns the number of
    fused operators."""
    live = getattr(bb, "live_out", None)
    tops = list(bb.roots) + [h for k, h in bb.env_out.items() if live is None or k in live]
    order = H.walk(tops)
    smemo = {"__act": _activations(order)}
    kinds = {h.id: _kind(h, smemo) for h in order}
    # epochs
    ep = {}
    for h in order:
        e = 0
        for c in h.inputs:
            bump = 0 if (kinds.get(c.id) is not None or c.op in ("lit", "tread")) else 1
            e = max(e, ep[c.id] + bump)
        ep[h.id] = e
    # device-dependence: matrix operators and aggregates, and scalar operators reading one
    dev = {}
    for h in order:
        k = kinds.get(h.id)
        if k is None:
            continue
        if k[0] in ("m", "r"):
            dev[h.id] = True
        else:
            dev[h.id] = any(dev.get(c.id, False) and ep[c.id] == ep[h.id] for c in h.inputs)
    consumers = {}
    for h in order:
        for c in h.inputs:
            consumers.setdefault(c.id, []).append(h)
    outset = {h.id for h in bb.roots} | {h.id for k, h in bb.env_out.items() if live is None or k in live}
    # sinking: an operator read only by template operators of one later epoch joins that
    # epoch's program (e.g. `lambda * V` of the block inputs, consumed after the big product)
    for h in reversed(order):
        if not dev.get(h.id) or h.id in outset:
            continue
        us = consumers.get(h.id, [])
        es = {ep[u.id] for u in us}
        if us and all(dev.get(u.id) for u in us) and len(es) == 1:
            e2 = es.pop()
            if e2 > ep[h.id]:
                ep[h.id] = e2
    groups = {}
    for h in order:
        if dev.get(h.id):
            groups.setdefault(ep[h.id], []).append(h)
    if not groups:
        return 0
    nfused = 0
    repl = {}
    for e, hs in groups.items():
        if not any(kinds[h.id][0] in ("m", "r") for h in hs):
            continue
        ids = {h.id for h in hs}
        outs = [h for h in hs if h.id in outset or any(u.id not in ids for u in consumers.get(h.id, []))]
        if not outs or len(hs) < 2:
            continue
        leaves, lpos = [], {}
        for h in hs:
            for c in h.inputs:
                if c.id not in ids and c.id not in lpos:
                    lpos[c.id] = len(leaves)
                    leaves.append(c)
        if any(c.dt not in ("M", "S") for c in leaves):
            continue
        for c in leaves:
            if c.dt == "M" and c.op not in ("lit", "tread"):
                c.p["keep_dev"] = True       # the program reads it from HBM: no host demotion
        n = len(leaves)
        vid = dict((c.id, k) for k, c in enumerate(leaves))
        instrs = []
        for h in hs:
            kind, o = kinds[h.id]
            vid[h.id] = n + len(instrs)
            instrs.append((kind, o, [vid[c.id] for c in h.inputs]))
        # fallback DAG: a clone of the region over placeholder reads of its operands
        names = [f"__vp{next(_names)}" for _ in leaves]
        memo = {}
        for c, nm in zip(leaves, names):
            memo[c.id] = Hop("tread", p={"name": nm}, dt=c.dt, dim1=c.dim1, dim2=c.dim2, pos=c.pos)
        for h in hs:
            memo[h.id] = Hop(h.op, [memo[c.id] for c in h.inputs], dict(h.p), named=list(h.named), dt=h.dt,
                             dim1=h.dim1, dim2=h.dim2, pos=h.pos)
        vp = VProgram([c.dt for c in leaves], instrs, [vid[h.id] for h in outs],
                      fallback_dag=(names, [memo[h.id] for h in outs]))
        V = Hop("vprog", list(leaves), {"prog": vp, "o": vp.describe()}, dt="U", pos=hs[-1].pos)
        lines = sorted({getattr(h.pos, "line", None) for h in hs} - {None})
        V.p["lines"] = lines
        for i, h in enumerate(outs):
            repl[h.id] = Hop("fout", [V], {"i": i}, dt=h.dt, dim1=h.dim1, dim2=h.dim2, pos=h.pos)
        nfused += len(hs)
    if not repl:
        return 0
    # rewire every consumer outside the regions (region-internal hops are unreachable now)
    seen = set()

    def sub(h):
        r = repl.get(h.id)
        if r is not None:
            return r
        if h.id in seen:
            return h
        seen.add(h.id)
        h.inputs = [sub(c) for c in h.inputs]
        return h

    for r in repl.values():
        V = r.inputs[0]
        if V.id not in seen:
            seen.add(V.id)
            V.inputs = [sub(c) for c in V.inputs]
    bb.roots = [sub(h) for h in bb.roots]
    bb.env_out = {k: sub(v) for k, v in bb.env_out.items()}
    return nfused
