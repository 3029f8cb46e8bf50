"""Operator fusion for cellwise DAGs: the Cell template of the reference's code generator
(reference: hops/codegen/SpoofCompiler.java#optimize, template/TemplateCell.java for the
candidate exploration, opt/PlanSelectionFuseCostBased for the materialisation points, and
cplan/CNodeCell for the generated operator).

Candidates are the cellwise binary / unary operators over matrices (the operator set of
ops/cell.py).  Fusion plans follow the reference's materialisation rules:
  * an operator is fused into its consumer only if that consumer is its ONLY consumer in the
    basic block and the value is not a block output (variable written or statement root) --
    a shared intermediate is materialised once instead of being recomputed per consumer;
  * a fused DAG may end in a full / row / column aggregate (sum, sumsq, mean, min, max) whose
    input it is the only consumer of (the reference's Cell template with
    CellType.FULL_AGG / ROW_AGG / COL_AGG);
  * a plan is bounded by the kernel's limits (<= 8 distinct inputs, <= 40 operators, <= 16
    live registers); a candidate that would exceed them is cut and its input materialised;
  * single operators are not fused (nothing to save), except as the body of an aggregate.
Each plan replaces its root hop (in place, so consumers need no rewiring) by a `cell` hop
whose inputs are the plan's leaves and whose `prog` is the register program that ops/cell.py
runs -- one HIP kernel launch on the MI355X, the original operators one by one elsewhere.

Everything the hand-written templates already cover (mmchain, smgrad, wquat, tak, sumsq,
softmax-gradient row template) is matched earlier by compiler/rewrites.py; this pass runs
last and only sees what is left.
"""
from __future__ import annotations

from .hops import walk
from ..ops.cell import BIN_CODES, UN_CODES, AGG_CODES, MAXIN, MAXOPS, NR, CellProgram, MultiAggProgram
from .hops import Hop

AGG_DIRS = ("all", "row", "col")


def _is_sq(h):
    b = h.inputs[1]
    return h.p.get("o") == "^" and b.op == "lit" and not isinstance(b.value, bool) and b.value == 2


def _cellwise(h):
    if h.dt != "M":
        return False
    if h.op == "b":
        return h.p.get("o") in BIN_CODES and len(h.inputs) == 2
    if h.op == "u":
        return h.p.get("o") in UN_CODES and len(h.inputs) == 1
    return False


def _operands(h):
    """Inputs the fused instruction reads (x ^ 2 reads only x)."""
    return [h.inputs[0]] if (h.op == "b" and _is_sq(h)) else list(h.inputs)


def _merge_leaves(a, b):
    out = list(a)
    for x in b:
        if all(x is not y for y in out):
            out.append(x)
    return out


def _regalloc(ops, leaves):
    """Linear-scan register assignment; None if more than NR registers would be live."""
    op_ids = {h.id for h in ops}

    def key(c):
        return ("op" if c.id in op_ids else "in", c.id)

    last = {}
    for k, h in enumerate(ops):
        for c in _operands(h):
            last[key(c)] = k
    reg = {("in", leaf.id): i for i, leaf in enumerate(leaves)}
    free = list(range(len(leaves), NR))
    code = []
    for k, h in enumerate(ops):
        srcs = [reg[key(c)] for c in _operands(h)]
        for c in _operands(h):
            kc = key(c)
            if last.get(kc) == k and kc in reg:
                free.append(reg.pop(kc))
        free.sort()
        if not free:
            return None
        d = free.pop(0)
        reg[("op", h.id)] = d
        if h.op == "b" and _is_sq(h):
            code.append(("u", "sq", d, srcs[0], 0))
        elif h.op == "b":
            code.append(("b", h.p["o"], d, srcs[0], srcs[1]))
        else:
            code.append(("u", h.p["o"], d, srcs[0], 0))
    return code, reg[("op", ops[-1].id)]


def fuse_cells(bb):
    """Fuse the cellwise sub-DAGs of a basic block; returns the number of fused operators."""
    live = getattr(bb, "live_out", None)
    order = walk(list(bb.roots) + list(bb.env_out.values()))
    # block outputs are materialised: statement roots and the variables read after the block
    outs = list(bb.roots) + [h for k, h in bb.env_out.items() if live is None or k in live]
    ncons = {}
    for h in order:
        for c in h.inputs:
            ncons[c.id] = ncons.get(c.id, 0) + 1
    for h in outs:
        ncons[h.id] = ncons.get(h.id, 0) + 1
    groups = {}                                       # hop id -> (ops in topological order, leaves)
    absorbed = set()
    for h in order:
        if not _cellwise(h):
            continue
        ops, leaves = [], []
        for c in _operands(h):
            g = groups.get(c.id)
            if g is not None and ncons.get(c.id, 0) == 1 and c.id not in absorbed:
                nl = _merge_leaves(leaves, g[1])
                if len(ops) + len(g[0]) + 1 <= MAXOPS and len(nl) <= MAXIN:
                    ops += g[0]
                    leaves = nl
                    absorbed.add(c.id)
                    continue
            leaves = _merge_leaves(leaves, [c])
        if len(leaves) > MAXIN:
            continue
        ops.append(h)
        groups[h.id] = (ops, leaves)
    plans = []
    for h in order:
        if h.op == "agg" and h.p.get("o") in AGG_CODES and h.p.get("dir") in AGG_DIRS and len(h.inputs) == 1:
            c = h.inputs[0]
            g = groups.get(c.id)
            if g is not None and ncons.get(c.id, 0) == 1 and c.id not in absorbed:
                absorbed.add(c.id)
                plans.append((h, g[0], g[1], (h.p["o"], h.p["dir"])))
    for h in order:
        g = groups.get(h.id)
        if g is not None and h.id not in absorbed and len(g[0]) >= 2:
            plans.append((h, g[0], g[1], None))
    n = 0
    built = []
    for root, ops, leaves, agg in plans:
        ra = _regalloc(ops, leaves)
        if ra is None:
            continue
        code, out = ra
        built.append((root, ops, leaves, CellProgram(code, len(leaves), out, agg)))
    grouped = _multi_agg(built)
    for root, ops, leaves, prog in built:
        if root.id in grouped:
            n += len(ops)
            continue
        root.op = "cell"
        root.inputs = list(leaves)
        root.named = []
        lines = sorted({getattr(o.pos, "line", None) for o in ops + [root]} - {None})
        root.p = {"o": prog.describe(), "prog": prog, "lines": lines}   # debugger: fused source lines
        n += len(ops)
    return n


MAGG_MAX = 4


def _multi_agg(built):
    """MAgg template (reference: template/TemplateMultiAgg.java and the multi-aggregate
    merge of PlanSelectionFuseCostBased): full aggregates of fused cell programs that read a
    common matrix input are combined -- up to MAGG_MAX per group and MAXIN distinct inputs --
    into one `magg` hop evaluated in a single pass (ops/cell.evaluate_multi); each original
    aggregate hop becomes output i of it.  Aggregates that depend on each other are never
    grouped.  Returns the ids of the replaced roots."""
    cands = [b for b in built if b[3].agg and b[3].agg[1] == "all"]
    if len(cands) < 2:
        return set()
    reach = {}
    for root, _, leaves, _ in cands:
        reach[root.id] = {h.id for h in walk(list(leaves))}
    groups = []
    for c in cands:
        root, _, leaves, _ = c
        mats = {h.id for h in leaves if h.dt == "M"}
        placed = False
        for g in groups:
            if len(g) >= MAGG_MAX:
                continue
            gm = {h.id for x in g for h in x[2] if h.dt == "M"}
            if not (mats & gm):
                continue
            union = {h.id for x in g for h in x[2]} | {h.id for h in leaves}
            if len(union) > MAXIN:
                continue
            if any(root.id in reach[x[0].id] or x[0].id in reach[root.id] for x in g):
                continue
            g.append(c)
            placed = True
            break
        if not placed:
            groups.append([c])
    done = set()
    for g in groups:
        if len(g) < 2:
            continue
        union = []
        for _, _, leaves, _ in g:
            for h in leaves:
                if all(h is not u for u in union):
                    union.append(h)
        idx = {h.id: i for i, h in enumerate(union)}
        m = MultiAggProgram([x[3] for x in g], [[idx[h.id] for h in x[2]] for x in g], len(union))
        mh = Hop("magg", list(union), {"o": m.describe(), "prog": m}, dt="U", pos=g[0][0].pos)
        for i, (root, ops, leaves, prog) in enumerate(g):
            lines = sorted({getattr(o.pos, "line", None) for o in ops + [root]} - {None})
            root.op = "fout"
            root.inputs = [mh]
            root.named = []
            root.p = {"i": i, "lines": lines}
            done.add(root.id)
    return done
