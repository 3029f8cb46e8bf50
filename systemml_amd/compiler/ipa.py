"""Inter-procedural analysis (reference: hops/ipa/InterProceduralAnalysis.java with
FunctionCallGraph.java, IPAPassRemoveUnusedFunctions.java, IPAPassInlineFunctions.java,
IPAPassPropagateReplaceLiterals.java and the recursion flags of FunctionCallGraph).

Runs on the translated program (HOP DAGs per basic block, before rewrites and
instruction generation):

  1. function call graph over main program + function bodies (fcall hops, literal
     `eval("name")` targets); functions on a cycle are flagged recursive;
  2. unused-function removal (unreachable from the main program; skipped when the
     program has an `eval` with a computed function name);
  3. inlining of small side-effect-free functions: a body that is a single basic block
     without function calls or side effects, called with all its parameters, is copied
     into the caller's DAG (parameters bound to the argument HOPs, declared scalar types
     enforced by casts) — the caller's rewrites then see through the call (e.g. fused
     operators across nn layer boundaries), and the call frame disappears;
  4. literal propagation: a scalar parameter that every call site passes as the same
     literal (and the body never reassigns) is replaced by that literal in the body;
  5. constant binary operations (IPAPassRemoveConstantBinaryOps): products with a main-program
     matrix of ones become products with the literal 1.
Static size propagation into function bodies (FunctionCallSizeInfo) is part of the program
walk of compiler/cost.py.
"""
from __future__ import annotations

from . import hops as H
from .hops import Hop, lit
from .blocks import BasicBlock, IfBlock, WhileBlock, ForBlock

INLINE_MAX_OPS = 24      # reference: InterProceduralAnalysis.INLINING_MAX_NUM_OPS (10)


# ----------------------------------------------------------------------------
# traversal helpers
# ----------------------------------------------------------------------------
def _block_dags(blocks):
    """Yield (owner, roots) for every HOP DAG in a block list (basic blocks and predicates)."""
    for b in blocks:
        if isinstance(b, BasicBlock):
            yield b, list(b.roots) + list(b.env_out.values())
        elif isinstance(b, IfBlock):
            yield b.pred, [b.pred.root]
            yield from _block_dags(b.then_blocks)
            yield from _block_dags(b.else_blocks)
        elif isinstance(b, WhileBlock):
            yield b.pred, [b.pred.root]
            yield from _block_dags(b.body)
        elif isinstance(b, ForBlock):
            for p in (b.start, b.end, b.incr):
                if p is not None:
                    yield p, [p.root]
            yield from _block_dags(b.body)


def _calls(blocks):
    """(fcall hops, literal eval targets, has dynamic eval) in a block list."""
    calls, evals, dyn = [], set(), False
    for _, roots in _block_dags(blocks):
        for h in H.walk(roots):
            if h.op == "fcall":
                calls.append(h)
            elif h.op == "bi" and h.p.get("name") == "eval":
                f = h.inputs[0] if h.inputs else None
                if f is not None and f.op == "lit" and isinstance(f.value, str):
                    evals.add(f.value.split("::")[-1])
                else:
                    dyn = True
    return calls, evals, dyn


# ----------------------------------------------------------------------------
def call_graph(cp):
    """{caller: set(callee fkeys)} with caller None = main program; plus dynamic-eval flag."""
    graph = {}
    dynamic = False
    by_name = {}
    for k in cp.functions:
        by_name.setdefault(k[1], []).append(k)
    units = [(None, cp.blocks)] + [(k, fb.body) for k, fb in cp.functions.items() if fb.body is not None]
    for key, blocks in units:
        calls, evals, dyn = _calls(blocks)
        dynamic |= dyn
        edges = {h.p["fkey"] for h in calls}
        for name in evals:
            edges |= set(by_name.get(name, []))
        graph[key] = edges
    for k, fb in cp.functions.items():
        for p in fb.default_preds.values():
            for h in H.walk([p.root]):
                if h.op == "fcall":
                    graph.setdefault(k, set()).add(h.p["fkey"])
    return graph, dynamic


def _reachable(graph, start=None):
    seen, stack = set(), [start]
    while stack:
        u = stack.pop()
        for v in graph.get(u, ()):
            if v not in seen:
                seen.add(v)
                stack.append(v)
    return seen


def flag_recursive(cp, graph):
    for k, fb in cp.functions.items():
        fb.recursive = k in _reachable(graph, k)


# ----------------------------------------------------------------------------
# inlining
# ----------------------------------------------------------------------------
def _inlineable(fb):
    if fb.external or fb.recursive or fb.body is None or len(fb.body) != 1:
        return False
    bb = fb.body[0]
    if not isinstance(bb, BasicBlock) or bb.roots:
        return False           # side effects (print/write/stop) or nested calls are roots
    outs = [o.name for o in fb.outputs]
    if any(o not in bb.env_out for o in outs):
        return False
    params = {p.name for p in fb.inputs}
    nops = 0
    for h in H.walk([bb.env_out[o] for o in outs]):
        if h.op == "tread" and h.p["name"] not in params:
            return False       # reads a variable that is neither parameter nor local
        if h.op in ("fcall", "fout", "sink") or (h.op == "bi" and h.p.get("name") in ("eval", "exists")):
            return False
        if h.op not in ("lit", "tread"):
            nops += 1
    fb._inline_ops = nops
    return True


def _cast(h, vtype):
    if h.dt != "S":
        return h
    if vtype == "DOUBLE":
        if h.op == "lit" and isinstance(h.value, (int, float)) and not isinstance(h.value, bool):
            return lit(float(h.value), h.pos)
        return Hop("u", [h], {"o": "cast_double"}, dt="S", pos=h.pos)
    if vtype == "BOOLEAN" and not (h.op == "lit" and isinstance(h.value, bool)):
        return Hop("u", [h], {"o": "cast_bool"}, dt="S", pos=h.pos)
    return h


def _copy_dag(outs, binding):
    """Deep copy of a function body DAG with parameter reads bound to argument HOPs."""
    memo = {}

    def cp_(h):
        r = memo.get(h.id)
        if r is not None:
            return r
        if h.op == "tread" and h.p["name"] in binding:
            r = binding[h.p["name"]]
        else:
            r = Hop(h.op, [cp_(c) for c in h.inputs], dict(h.p), list(h.named), h.dt, h.dim1, h.dim2, h.pos)
        memo[h.id] = r
        return r
    return [cp_(o) for o in outs]


def inline_functions(cp, graph, stats, rounds=4):
    """Inline bottom-up: a function whose body calls a small function becomes inlineable itself
    once that call is inlined (nn layers calling util::channel_sums), so candidates are
    recomputed until a round inlines nothing."""
    ncalls = {}
    for edges in graph.values():
        for k in edges:
            ncalls[k] = ncalls.get(k, 0) + 1
    for _ in range(rounds):
        candidates = {k: fb for k, fb in cp.functions.items() if _inlineable(fb)}
        if not candidates:
            return
        before = stats.get("inlined", 0)
        units = [cp.blocks] + [fb.body for fb in cp.functions.values() if fb.body is not None]
        for blocks in units:
            for owner, _ in list(_block_dags(blocks)):
                if not isinstance(owner, BasicBlock):
                    continue
                _inline_in_block(owner, candidates, ncalls, stats)
        if stats.get("inlined", 0) == before:
            return


def _inline_in_block(bb, candidates, ncalls, stats):
    repl = {}
    keep_roots = []
    for r in bb.roots:
        fkey = r.p.get("fkey") if r.op == "fcall" else None
        fb = candidates.get(fkey) if fkey else None
        if fb is None or (fb._inline_ops > INLINE_MAX_OPS and ncalls.get(fkey, 0) > 1):
            keep_roots.append(r)
            continue
        given = list(r.p["given"])
        params = {p.name: p for p in fb.inputs}
        if set(given) != set(params):
            keep_roots.append(r)          # defaults needed: keep the call
            continue
        binding = {}
        for name, arg in zip(given, r.inputs):
            p = params[name]
            binding[name] = _cast(arg, p.vtype) if p.dtype == "SCALAR" else arg
        body = fb.body[0]
        outs = _copy_dag([body.env_out[o.name] for o in fb.outputs], binding)
        outs = [_cast(h, o.vtype) if o.dtype == "SCALAR" else h for h, o in zip(outs, fb.outputs)]
        repl[r.id] = outs
        stats["inlined"] = stats.get("inlined", 0) + 1
    if not repl:
        return
    bb.roots = keep_roots
    memo = {}

    def sub(h):
        if h.op == "fout" and h.inputs and h.inputs[0].id in repl:
            # the inlined body may itself consume outputs of other calls inlined here
            return sub(repl[h.inputs[0].id][h.p["i"]])
        r = memo.get(h.id)
        if r is not None:
            return r
        memo[h.id] = h
        h.inputs = [sub(c) for c in h.inputs]
        return h

    bb.roots = [sub(h) for h in bb.roots]
    bb.env_out = {k: sub(v) for k, v in bb.env_out.items()}


# ----------------------------------------------------------------------------
# literal propagation into functions
# ----------------------------------------------------------------------------
def _assigned(blocks):
    from .loops import assigned_in
    return assigned_in(blocks)


def literal_params(cp):
    """{function key: {scalar parameter: literal}} for the parameters every call site passes as
    the same literal and the body never reassigns."""
    sites = {}
    units = [cp.blocks] + [fb.body for fb in cp.functions.values() if fb.body is not None]
    for blocks in units:
        calls, _, _ = _calls(blocks)
        for h in calls:
            sites.setdefault(h.p["fkey"], []).append(h)
    out = {}
    for k, fb in cp.functions.items():
        if fb.body is None or fb.external or k not in sites:
            continue
        assigned = _assigned(fb.body)
        consts = {}
        for p in fb.inputs:
            if p.dtype != "SCALAR" or p.name in assigned:
                continue
            vals = []
            for h in sites[k]:
                given = list(h.p["given"])
                if p.name not in given:
                    vals = None
                    break
                a = h.inputs[given.index(p.name)]
                if a.op != "lit":
                    vals = None
                    break
                vals.append(a.value)
            if vals and all(type(v) is type(vals[0]) and v == vals[0] for v in vals):
                v = vals[0]
                if p.vtype == "DOUBLE" and isinstance(v, int) and not isinstance(v, bool):
                    v = float(v)
                consts[p.name] = v
        if consts:
            out[k] = consts
    return out


def propagate_literals(cp, stats):
    for k, consts in literal_params(cp).items():
        fb = cp.functions[k]
        for owner, roots in _block_dags(fb.body):
            for h in H.walk(roots):
                h.inputs = [lit(consts[c.p["name"]], c.pos) if (c.op == "tread" and c.p["name"] in consts) else c
                            for c in h.inputs]
            if isinstance(owner, BasicBlock):
                owner.env_out = {n: (lit(consts[v.p["name"]], v.pos) if v.op == "tread" and v.p["name"] in consts
                                     else v) for n, v in owner.env_out.items()}
            elif owner.root.op == "tread" and owner.root.p["name"] in consts:
                owner.root = lit(consts[owner.root.p["name"]])
                owner.is_const, owner.const = True, owner.root.value
        stats["literals"] = stats.get("literals", 0) + len(consts)


def _is_ones(h):
    """matrix(1, rows=.., cols=..): a constant datagen of ones."""
    if h.op != "bi" or h.p.get("name") != "matrix" or not h.inputs:
        return False
    d = h.inputs[0]
    return d.op == "lit" and isinstance(d.value, (int, float)) and not isinstance(d.value, bool) and d.value == 1


def _ones_shape(h):
    """(rows, cols) hops of a matrix(1, rows=.., cols=..) datagen."""
    named = dict(zip(h.named, h.inputs[len(h.inputs) - len(h.named):]))
    return named.get("rows"), named.get("cols")


def _broadcasts_into(ones, x):
    """True if `x * ones` has x's shape: ones is x's shape, an x-length column or an x-width row
    -- never an outer-vector product (n x 1 times 1 x k) or a ones matrix larger than x
    (reference IPAPassRemoveConstantBinaryOps.java:139-143 skips isOuterVectorOperator).  Shapes
    are matched structurally (rows=nrow(X) / cols=ncol(X) of the same variable, or 1), else by
    known dimensions."""
    r, c, xr, xc = ones.dim1, ones.dim2, x.dim1, x.dim2
    if min(r, c, xr, xc) > 0:
        return (r, c) in ((xr, xc), (xr, 1), (1, xc))
    if x.op != "tread":
        return False
    rh, ch = _ones_shape(ones)

    def fits(d, which):
        if d is None:
            return False
        if d.op == "lit" and d.value == 1:
            return True
        return d.op == "u" and d.p.get("o") == which and d.inputs and d.inputs[0].op == "tread" \
            and d.inputs[0].p.get("name") == x.p.get("name")
    return fits(rh, "nrow") and fits(ch, "ncol")


def _shape_vars(ones):
    """Variables the ones matrix's shape expressions read (reassigning one invalidates it)."""
    return {h.p["name"] for h in H.walk([i for i in _ones_shape(ones) if i is not None]) if h.op == "tread"}


def remove_constant_binary_ops(cp, stats):
    """IPAPassRemoveConstantBinaryOps (reference hops/ipa/IPAPassRemoveConstantBinaryOps.java):
    a main-program variable assigned matrix(1, ...) in a basic block and not reassigned later
    makes every later `M * ones` (and `ones * M`, M a matrix) a `M * 1`, which the algebraic
    rewrites then drop -- e.g. the all-ones weight vectors scripts default to."""
    from .loops import assigned_in
    ones = {}
    n = [0]

    def rewrite(blocks):
        for owner, roots in _block_dags(blocks):
            for h in H.walk(roots):
                if h.op == "b" and h.p.get("o") == "*" and len(h.inputs) == 2:
                    # like the reference, only the RIGHT operand is replaced, and only when the
                    # product keeps the left operand's shape: the ones matrix must broadcast INTO
                    # X (same shape, X's column or X's row) -- never an outer-vector product
                    # (n x 1 times 1 x k) or a ones matrix larger than X
                    x, y = h.inputs
                    if y.op == "tread" and y.p.get("name") in ones and x.dt == "M" \
                            and _broadcasts_into(ones[y.p["name"]], x):
                        h.inputs = [x, lit(1)]
                        n[0] += 1

    for b in cp.blocks:
        upd = b.writes if isinstance(b, BasicBlock) else assigned_in([b])
        for v in upd:
            ones.pop(v, None)
            for k in [k for k, o in ones.items() if v in _shape_vars(o)]:
                ones.pop(k)
        if ones:
            rewrite([b])
        if isinstance(b, BasicBlock):
            for v, h in b.env_out.items():
                if _is_ones(h) and not (_shape_vars(h) & set(b.writes)):
                    ones[v] = h
    if n[0]:
        stats["constant-binary-ops"] = n[0]


# ----------------------------------------------------------------------------
def run(cp, config=None):
    """Apply the IPA passes in place; returns a stats dict (also kept as cp.ipa_stats)."""
    stats = {}
    graph, dynamic = call_graph(cp)
    flag_recursive(cp, graph)
    if not dynamic:
        used = _reachable(graph, None)
        for k in list(cp.functions):
            if k not in used and not cp.functions[k].external:
                del cp.functions[k]
                stats["removed"] = stats.get("removed", 0) + 1
    if config is None or getattr(config, "inline_functions", True):
        inline_functions(cp, graph, stats)
    propagate_literals(cp, stats)
    remove_constant_binary_ops(cp, stats)
    cp.ipa_stats = stats
    return stats
