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
        # licm_def: the hoisted expression, so fused-template matchers in the body can see
        # through the transient read (rewrites.fuse_softmax_grad)
        hoisted[c.id] = Hop("tread", p={"name": name, "licm_def": c}, dt="M", dim1=c.dim1, dim2=c.dim2, pos=c.pos)

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
    pre.licm_pre = True          # runtime defers its errors to the first read (zero-trip loops)
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
    # temporaries numbered per program: a recompilation of the same script names them alike
    # (runtime/graphloop.py finds a loop's captured graph by the names its body reads)
    global _names
    _names = itertools.count(1)
    stats = hoist_loop_invariants(cp.blocks)
    for fb in cp.functions.values():
        if fb.body is not None:
            hoist_loop_invariants(fb.body, stats)
    return stats


# ----------------------------------------------------------------------------
# update-in-place (reference: hops/rewrite/RewriteMarkLoopVariablesUpdateInPlace.java)
# ----------------------------------------------------------------------------
_SHAPE = ("nrow", "ncol", "length")
_FRESH = ("agg", "tak", "mm", "tsmm", "mmchain")


def _dag(bb):
    """All hops of a basic block and their consumers: id -> [(consumer hop | 'ENV:<name>', input index)]."""
    tops = list(bb.roots) + list(bb.env_out.values())
    hops = H.walk(tops)
    cons = {}
    for h in hops:
        for i, c in enumerate(h.inputs):
            cons.setdefault(c.id, []).append((h, i))
    for name, h in bb.env_out.items():
        cons.setdefault(h.id, []).append(("ENV:" + name, -1))
    for r in bb.roots:
        cons.setdefault(r.id, []).append(("ROOT", -1))
    return hops, cons


def _closure(hs):
    out = {}
    for h in H.walk(hs):
        out[h.id] = h
    return out


def _bb_update_in_place_ok(bb, v):
    """True when, in this block, matrix variable v is only (a) the target of a left-indexing
    chain whose final result is v's new value, (b) an input of nrow/ncol/length, or (c) read
    inside the index/value inputs of that chain and nowhere else -- so modifying v's buffer in
    place can neither be observed through another reference nor race an unordered read."""
    if v not in bb.reads and v not in bb.writes:
        return True
    hops, cons = _dag(bb)
    final = bb.env_out.get(v)
    chain = []
    if final is not None and not (final.op == "tread" and final.p.get("name") == v):
        h = final
        while h.op == "lix":
            chain.append(h)
            h = h.inputs[0]
        if not (h.op == "tread" and h.p.get("name") == v) or not chain:
            return False
    elif final is not None:
        return True
    chain_ids = {h.id for h in chain}
    # hops allowed to consume (values derived from) v: inside the non-target inputs of the chain
    inner = _closure([x for lx in chain for x in lx.inputs[1:]])
    treads = [h for h in hops if h.op == "tread" and h.p.get("name") == v]
    sources = treads + chain[:-1] if chain else treads
    if not chain:
        # v only read in this block: by operators that produce a fresh value (never a view
        # or the same buffer), so no reference to v's buffer survives the block
        for t in treads:
            for c, i in cons.get(t.id, []):
                if isinstance(c, str) or not (c.op in _FRESH or (c.op == "u" and c.p.get("o") in _SHAPE)):
                    return False
        return True
    for s in sources:
        for c, i in cons.get(s.id, []):
            if isinstance(c, str):
                return False                      # aliased into another variable / root
            if c.id in chain_ids and i == 0:
                continue                          # next left-indexing of the chain
            if c.op == "u" and c.p.get("o") in _SHAPE:
                continue
            if c.id in inner:
                continue
            return False
    # everything computed inside the chain's inputs FROM v must be consumed only there (no
    # escaping views); values that do not depend on v cannot alias its buffer
    src_ids = {s.id for s in sources}
    dep = {}

    def from_v(h):
        r = dep.get(h.id)
        if r is None:
            r = dep[h.id] = h.id in src_ids or any(from_v(c) for c in h.inputs)
        return r
    for hid, h in inner.items():
        if h.op in ("tread", "lit") or h.dt == "S" or not from_v(h):
            continue                              # scalars hold no view of v's buffer
        for c, i in cons.get(hid, []):
            if isinstance(c, str) or not (c.id in inner or c.id in chain_ids):
                return False
    for h in inner.values():
        if h.op == "rix" and h.inputs[0].id in {s.id for s in sources}:
            h.p["copy"] = True                    # a view of v must not alias the updated buffer
    return True


def _uip_ok(blocks, v):
    """Predicates only produce scalars (evaluated before the blocks they guard), so reads
    there are safe; nested loops that touch v must have marked it themselves."""
    for b in blocks:
        if isinstance(b, BasicBlock):
            if not _bb_update_in_place_ok(b, v):
                return False
        elif isinstance(b, IfBlock):
            if not (_uip_ok(b.then_blocks, v) and _uip_ok(b.else_blocks, v)):
                return False
        elif isinstance(b, (WhileBlock, ForBlock)):
            if v in assigned_in(b.body):
                if v not in getattr(b, "inplace_vars", ()):
                    return False
            elif not _uip_ok(b.body, v):
                return False
    return True


def _reads_in(blocks, v):
    for b in blocks:
        if isinstance(b, BasicBlock):
            if v in b.reads:
                return True
        elif isinstance(b, IfBlock):
            if v in b.pred.reads or _reads_in(b.then_blocks, v) or _reads_in(b.else_blocks, v):
                return True
        elif isinstance(b, WhileBlock):
            if v in b.pred.reads or _reads_in(b.body, v):
                return True
        elif isinstance(b, ForBlock):
            preds = [b.start, b.end] + ([b.incr] if b.incr is not None else [])
            if any(v in p.reads for p in preds) or _reads_in(b.body, v):
                return True
    return False


def _in_parfor(blocks, v):
    """True when `v` is assigned inside a parfor nested in `blocks`."""
    for b in blocks:
        if isinstance(b, IfBlock):
            if _in_parfor(b.then_blocks, v) or _in_parfor(b.else_blocks, v):
                return True
        elif isinstance(b, (WhileBlock, ForBlock)):
            if isinstance(b, ForBlock) and b.parfor and v in assigned_in(b.body):
                return True
            if _in_parfor(b.body, v):
                return True
    return False


def _lix_in(blocks, v, out):
    for b in blocks:
        if isinstance(b, BasicBlock):
            h = b.env_out.get(v)
            while h is not None and h.op == "lix":
                out.append(h)
                h = h.inputs[0]
        elif isinstance(b, IfBlock):
            _lix_in(b.then_blocks, v, out)
            _lix_in(b.else_blocks, v, out)
        elif isinstance(b, (WhileBlock, ForBlock)):
            _lix_in(b.body, v, out)
    return out


def mark_update_in_place(blocks, stats=None):
    """Mark loop variables that are only modified by left indexing (and otherwise only queried
    for their shape) as update-in-place: the runtime then copies the matrix once on loop entry
    and applies every `X[i, ] = ...` to that private buffer instead of cloning the whole matrix
    per assignment (O(rows) instead of O(rows^2) bytes for a row-by-row loop).  parfor bodies
    are excluded (workers share the pre-loop value)."""
    stats = {} if stats is None else stats
    for b in blocks:
        if isinstance(b, IfBlock):
            mark_update_in_place(b.then_blocks, stats)
            mark_update_in_place(b.else_blocks, stats)
        elif isinstance(b, (WhileBlock, ForBlock)):
            mark_update_in_place(b.body, stats)           # inner loops first
            b.inplace_vars = []
            if isinstance(b, ForBlock) and b.parfor:
                _mark_parfor_inplace(b, stats)
                continue
            cand = sorted(assigned_in(b.body) - ({b.var} if isinstance(b, ForBlock) else set()))
            for v in cand:
                lixes = _lix_in(b.body, v, [])
                # a variable left-indexed inside a nested parfor stays copy-on-write: the
                # workers share the pre-loop buffer and merge by comparing against it
                if _in_parfor(b.body, v):
                    continue
                if lixes and all(h.dt == "M" for h in lixes) and _uip_ok(b.body, v):
                    b.inplace_vars.append(v)
                    for h in lixes:
                        h.p["inplace"] = True
                    stats["update-in-place"] = stats.get("update-in-place", 0) + 1
    return stats


def _mark_parfor_inplace(b, stats):
    """In-place result indexing of a parfor (reference OptimizerRuleBased.
    rewriteSetInPlaceResultIndexing, :1642, and rewriteRemoveUnnecessaryCompareMatrix, :2021):
    a variable the body modifies only by left indexing -- and otherwise reads at most for its
    shape -- has disjoint per-iteration writes once the dependency analysis accepted the loop
    (compiler/parfor_deps.py).  Its writes are marked in place; at run time all workers then
    update ONE private copy of the pre-loop matrix and no result merge with a compare matrix
    is needed (runtime/parfor.py).  `check=0` switches the analysis off, and with it this."""
    chk = b.params.get("check")
    if chk is not None and str(chk) in ("0", "0.0", "False", "false", "FALSE"):
        b.parfor_inplace = []
        return
    acc = set(getattr(b, "accumulators", ()))
    out = []
    for v in sorted(assigned_in(b.body) - {b.var} - acc):
        lixes = _lix_in(b.body, v, [])
        if lixes and all(h.dt == "M" for h in lixes) and _uip_ok(b.body, v):
            out.append(v)
            for h in lixes:
                h.p["inplace"] = True
            stats["parfor-inplace-result"] = stats.get("parfor-inplace-result", 0) + 1
    b.parfor_inplace = out


def mark_program(cp):
    stats = mark_update_in_place(cp.blocks)
    for fb in cp.functions.values():
        if fb.body is not None:
            mark_update_in_place(fb.body, stats)
    return stats
