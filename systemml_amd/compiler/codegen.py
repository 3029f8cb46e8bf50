"""Operator fusion for cellwise DAGs: the Cell template of the reference's code generator
(reference: hops/codegen/SpoofCompiler.java#optimize, template/TemplateCell.java for the
candidate exploration, opt/PlanSelectionFuseCostBased for the materialisation points, and
cplan/CNodeCell for the generated operator).

Candidates are the cellwise binary / unary operators over matrices (the operator set of
ops/cell.py).  Fusion plans follow the reference's materialisation rules:
  * an operator is fused into its consumer if that consumer is its ONLY consumer in the basic
    block and the value is not a block output (variable written or statement root);
  * a shared intermediate (several consumers, not a block output) is a materialisation point:
    the cost-based plan selection (`_select_plan`, the reference's PlanSelectionFuseCostBasedV2)
    prices every combination of "materialise once" / "recompute inside each consumer" by HBM
    reads + writes and operator cost and takes the cheapest;
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


_BIAS = {"bias_add": "bias+", "bias_multiply": "bias*"}


def _is_bias(h):
    """bias_add / bias_multiply (per-channel broadcast of a C x 1 vector over an N x (C*H*W)
    operand): cellwise operators of the Cell template with a CHAN-mode second operand."""
    return h.op == "bi" and h.p.get("name") in _BIAS and len(h.inputs) == 2 and not h.named


def _cellwise(h):
    if h.dt != "M":
        return False
    if _is_bias(h):
        return True
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
        if _is_bias(h):
            code.append(("b", _BIAS[h.p["name"]], d, srcs[0], srcs[1]))
        elif h.op == "b" and _is_sq(h):
            code.append(("u", "sq", d, srcs[0], 0))
        elif h.op == "b":
            code.append(("b", h.p["o"], d, srcs[0], srcs[1]))
        else:
            code.append(("u", h.p["o"], d, srcs[0], 0))
    return code, reg[("op", ops[-1].id)]


def _group(order, ncons, inline):
    """Cell-template grouping for one materialisation plan: every cellwise hop gets the fused
    DAG (ops in topological order, leaves) ending in it.  An operand's DAG is absorbed when the
    hop is its only consumer, or when the plan recomputes that shared intermediate inside
    each consumer (`inline`).  Returns (groups, times each hop was absorbed)."""
    groups = {}                                       # hop id -> (ops in topological order, leaves)
    absorbed = {}
    for h in order:
        if not _cellwise(h):
            continue
        ops, leaves, took = [], [], []
        for ci, c in enumerate(_operands(h)):
            g = groups.get(c.id)
            if _is_bias(h) and ci == 1:
                g = None                      # the per-channel operand is read by the kernel as is
            if g is not None and ((ncons.get(c.id, 0) == 1 and c.id not in absorbed) or c.id in inline):
                extra = [o for o in g[0] if all(o is not x for x in ops)]
                nl = _merge_leaves(leaves, g[1])
                if len(ops) + len(extra) + 1 <= MAXOPS and len(nl) <= MAXIN:
                    ops += extra
                    leaves = nl
                    absorbed[c.id] = absorbed.get(c.id, 0) + 1
                    took.append(c.id)
                    continue
            leaves = _merge_leaves(leaves, [c])
        if len(leaves) > MAXIN:
            # a later operand overflowed the input limit: the absorbed operands stay
            # materialised (their own plans) and h reads them
            for cid in took:
                absorbed[cid] -= 1
                if not absorbed[cid]:
                    del absorbed[cid]
            ops, leaves = [], _merge_leaves([], _operands(h))
            if len(leaves) > MAXIN:
                continue
        ops.append(h)
        groups[h.id] = (ops, leaves)
    aggs = []                                         # (aggregate hop, fused DAG it absorbs)
    for h in order:
        if _is_cell_agg(h):
            c = h.inputs[0]
            g = groups.get(c.id)
            if g is not None and ((ncons.get(c.id, 0) == 1 and c.id not in absorbed) or c.id in inline):
                absorbed[c.id] = absorbed.get(c.id, 0) + 1
                aggs.append((h, g))
    return groups, absorbed, aggs


def _is_cell_agg(h):
    return h.op == "agg" and h.p.get("o") in AGG_CODES and h.p.get("dir") in AGG_DIRS and len(h.inputs) == 1


_HEAVY_OPS = {"exp", "log", "sqrt", "^", "sigmoid", "tanh", "sin", "cos", "tan", "asin", "acos", "atan",
              "sinh", "cosh", "%%", "%/%", "/"}


def _cells(h, memo):
    """Estimated cell count of a hop's value (0 for scalars; unknown matrices 1e6, cellwise
    hops the largest of their operands)."""
    r = memo.get(h.id)
    if r is None:
        if h.dt != "M":
            r = 0.0
        elif h.dim1 >= 0 and h.dim2 >= 0:
            r = float(h.dim1 * h.dim2)
        elif h.op == "agg" and h.p.get("dir") in ("row", "col"):
            r = 1e3                                   # a row / column aggregate: a vector
        elif _cellwise(h):
            r = max((_cells(c, memo) for c in _operands(h)), default=0.0) or 1e6
        else:
            r = 1e6
        memo[h.id] = r
    return r


def _plan_cost(order, groups, absorbed, aggs, ncons, memo):
    """HBM + compute cost of a Cell-template plan, in cell-reads: every materialised fused DAG
    reads its leaves and writes its root once; its operators cost a fraction of a read per
    cell (transcendentals more).  The reference's PlanSelectionFuseCostBasedV2 prices plans
    the same way (memory traffic + compute of each fused operator)."""
    cost = 0.0
    for h in order:
        g = groups.get(h.id)
        if g is None or absorbed.get(h.id, 0) >= ncons.get(h.id, 0):
            continue
        ops, leaves = g
        n = _cells(h, memo)
        cost += n + sum(_cells(c, memo) for c in leaves)
        cost += sum((0.25 if o.p.get("o") in _HEAVY_OPS else 0.05) * n for o in ops)
    fused = set()
    for h, (ops, leaves) in aggs:                     # fused aggregates: read the leaves once
        n = _cells(h.inputs[0], memo)
        cost += sum(_cells(c, memo) for c in leaves)
        cost += sum((0.25 if o.p.get("o") in _HEAVY_OPS else 0.05) * n for o in ops)
        fused.add(h.id)
    for h in order:                                   # plain aggregates read their materialised input
        if h.id not in fused and _is_cell_agg(h) and h.inputs[0].id in groups:
            cost += _cells(h.inputs[0], memo)
    return cost


ENUM_MAX = 8          # exhaustive plan enumeration up to this many materialisation points


def _select_plan(order, ncons, outs):
    """Materialisation-point selection (reference: opt/PlanSelectionFuseCostBasedV2): the
    shared cellwise intermediates that are no block output are the interesting points; each is
    either materialised once or recomputed inside every consumer.  Up to ENUM_MAX points every
    combination is costed, beyond that a greedy pass flips one point at a time; recomputing a
    point must save >= 5 % of a pass over it to be taken.  Returns (inline set, stats)."""
    out_ids = {h.id for h in outs}
    cons = {}
    for h in order:
        for c in h.inputs:
            cons.setdefault(c.id, []).append(h)
    base_groups, _, _ = _group(order, ncons, frozenset())
    points = [h.id for h in order if h.id in base_groups and ncons.get(h.id, 0) > 1 and h.id not in out_ids
              and any(_cellwise(u) or _is_cell_agg(u) for u in cons.get(h.id, ()))]
    if not points:
        return frozenset(), None
    memo = {}

    def cost(inl):
        g, a, ag = _group(order, ncons, inl)
        return _plan_cost(order, g, a, ag, ncons, memo)
    size = {h.id: _cells(h, memo) for h in order if h.id in set(points)}
    best_cost = cost(frozenset())
    best = frozenset()
    evaluated = 1
    # a plan must save at least 5 % of one pass over the values it stops materialising
    if len(points) <= ENUM_MAX:
        for mask in range(1, 1 << len(points)):
            inl = frozenset(p for i, p in enumerate(points) if mask >> i & 1)
            c = cost(inl)
            evaluated += 1
            if c < best_cost - 0.05 * sum(size[p] for p in inl - best):
                best, best_cost = inl, c
    else:
        # many points (e.g. a whole network's layers inlined into one block): each flip is
        # priced on its neighbourhood only -- the point's fused DAG and the downstream
        # cellwise / aggregate consumers it could be recomputed in, with their fused DAGs
        for p in points:
            region = {o.id for o in base_groups[p][0]}
            stack = [p]
            while stack:
                u = stack.pop()
                for v in cons.get(u, ()):
                    if v.id in region or not (_cellwise(v) or _is_cell_agg(v)):
                        continue
                    region.add(v.id)
                    g = base_groups.get(v.id)
                    if g is not None:
                        region.update(o.id for o in g[0])
                    if len(region) < 256:
                        stack.append(v.id)
            sub = [h for h in order if h.id in region]
            g0, a0, ag0 = _group(sub, ncons, best)
            g1, a1, ag1 = _group(sub, ncons, best | {p})
            evaluated += 1
            if _plan_cost(sub, g1, a1, ag1, ncons, memo) < _plan_cost(sub, g0, a0, ag0, ncons, memo) - 0.05 * size[p]:
                best = frozenset(best | {p})
    return best, {"points": len(points), "plans": evaluated, "inlined": len(best)}


def fuse_cells(bb, single=False, stats=None):
    """Fuse the cellwise sub-DAGs of a basic block; returns the number of fused operators.
    single: also single operators and aggregates of a plain input become generated kernels
    (GPU plans: the reference's SystemML.cu matrix_matrix_cellwise_op / reduce_* kernels, here
    generated per operator and operand signature instead of ATen's).  Shared intermediates are
    materialised or recomputed per consumer as the cost-based plan selection decides."""
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
    inline, st = _select_plan(order, ncons, outs)
    if st is not None and stats is not None:
        for k, v in st.items():
            stats[f"cell-plan-{k}"] = stats.get(f"cell-plan-{k}", 0) + v
    groups, absorbed, aggs = _group(order, ncons, inline)
    plans = [(h, g[0], g[1], (h.p["o"], h.p["dir"])) for h, g in aggs]
    fused_aggs = {h.id for h, _ in aggs}
    if single:
        for h in order:
            if _is_cell_agg(h) and h.id not in fused_aggs and h.inputs[0].dt == "M" and h.dt in ("M", "S"):
                # aggregate of a plain or materialised input
                plans.append((h, [], [h.inputs[0]], (h.p["o"], h.p["dir"])))
    for h in order:
        g = groups.get(h.id)
        if g is not None and absorbed.get(h.id, 0) < ncons.get(h.id, 0) and len(g[0]) >= (1 if single else 2):
            plans.append((h, g[0], g[1], None))
    n = 0
    built = []
    planned = set()
    for root, ops, leaves, agg in plans:
        if not ops:
            built.append((root, ops, leaves, CellProgram((), 1, 0, agg)))
            continue
        ra = _regalloc(ops, leaves)
        if ra is None:
            # more live values than registers: the DAG's operators become one-operator
            # programs (on the GPU: generated kernels, not the unfused fallback)
            if single:
                for o in ops:
                    if o.id in planned or (o is root and agg is None):
                        continue
                    planned.add(o.id)
                    lv = _merge_leaves([], _operands(o))
                    r1 = _regalloc([o], lv)
                    if r1 is not None:
                        built.append((o, [o], lv, CellProgram(r1[0], len(lv), r1[1], None)))
                if agg is not None:
                    built.append((root, [], [root.inputs[0]], CellProgram((), 1, 0, agg)))
                elif root.id not in planned:
                    lv = _merge_leaves([], _operands(root))
                    r1 = _regalloc([root], lv)
                    if r1 is not None:
                        built.append((root, [root], lv, CellProgram(r1[0], len(lv), r1[1], None)))
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

# ----------------------------------------------------------------------------- Row template
ROW_AGG_OPS = ("sum", "sumsq", "mean", "min", "max")


ROW_MAXW = 16       # widest side matrix of a Row-template product (ops/rowgen.MAXW)
ROW_MERGE = __import__("os").environ.get("SYSML_ROW_MERGE", "1") != "0"   # multi-output Row programs


def _narrow(h):
    """A side operand of a row product: a D x 1 vector or a D x K matrix with K <= ROW_MAXW
    (unknown widths are admitted; the kernel re-checks the actual shapes)."""
    return h.dim2 == -1 or 1 <= h.dim2 <= ROW_MAXW


def _const_col(h):
    """The scalar c of a constant column matrix(c, rows=n, cols=1), else None."""
    if h.op == "bi" and h.p.get("name") == "matrix" and len(h.inputs) == 3 and h.inputs[0].dt == "S" \
            and h.inputs[2].op == "lit" and h.inputs[2].value == 1 and h.p.get("npos", 1) == 1:
        return h.inputs[0]
    return None


def _wcols_k(h):
    """k of a leading-column slice X[, 1:k]: an int for a literal bound, the bound's hop for a
    scalar expression (the kernel is specialised on its value at run time), else None."""
    if h.op != "rix" or len(h.inputs) != 5:
        return None
    _, rl, ru, cl, cu = h.inputs
    none = lambda z: z.op == "lit" and z.value is None                      # noqa: E731
    if not (none(rl) and none(ru) and cl.op == "lit" and cl.value == 1):
        return None
    if cu.op == "lit":
        if isinstance(cu.value, (int, float)) and not isinstance(cu.value, bool) and 1 <= cu.value <= ROW_MAXW:
            return int(cu.value)
        return None
    return cu if cu.dt == "S" else None


def _row_body_kind(h):
    """Role of h inside a Row-template region: 'cell' | 'ragg' | 'dot' | 'cbindc' | 'wcols' |
    None (not fusable).  'cbindc' (a constant column appended) and 'wcols' (leading columns)
    apply to the narrow per-row vectors of products with side matrices only -- the region
    admits them when their input is a region product (_form_row_region)."""
    if h.dt != "M" or _is_bias(h):
        return None
    if _cellwise(h):
        return "cell"
    if h.op == "agg" and h.p.get("dir") == "row" and h.p.get("o") in ROW_AGG_OPS and len(h.inputs) == 1:
        return "ragg"
    if h.op == "mm" and not h.p.get("transA") and not h.p.get("mvagg") and len(h.inputs) == 2 \
            and _narrow(h.inputs[1]) and h.inputs[0].dim2 != 1:
        return "dot"
    if h.op == "bi" and h.p.get("name") == "cbind" and len(h.inputs) == 2 and _const_col(h.inputs[1]) is not None:
        return "cbindc"
    if _wcols_k(h) is not None:
        return "wcols"
    return None


def _row_root_kind(h):
    """Output type when h ends a Row-template region ('col' | 'all' | 'tmv'), else None."""
    if h.dt == "M" and h.op == "agg" and len(h.inputs) == 1:
        if h.p.get("dir") == "col" and h.p.get("o") in ("sum", "sumsq", "mean"):
            return "col"
    if h.op == "agg" and h.p.get("dir") == "all" and h.p.get("o") in ROW_AGG_OPS and len(h.inputs) == 1 \
            and h.inputs[0].dt == "M":
        return "all"
    if h.dt == "M" and h.op == "mm" and h.p.get("transA") and not h.p.get("mvagg") and len(h.inputs) == 2 \
            and _narrow(h.inputs[1]):
        return "tmv"
    return None


def _body_inputs(h, kind):
    """Inputs of a region hop that may join the region (a dot's side vector never does)."""
    if kind in ("dot", "cbindc", "wcols"):
        return [h.inputs[0]]
    return _operands(h) if kind == "cell" else list(h.inputs)


def _narrow_source(x, kinds):
    """x is (derived from) a region product with a side matrix: a K-wide per-row vector."""
    k = kinds.get(x.id)
    if k in ("dot", "cbindc", "wcols"):
        return True
    return k == "cell" and any(_narrow_source(c, kinds) for c in _operands(x) if c.id in kinds)


def _size_class(h, memo):
    """Structural size class of a hop's value for the materialisation cost model: 1.0 for a
    full N x D matrix, 1e-3 for a per-row N x 1 vector (row aggregates, matrix-vector
    products) or a small side vector, 0 for scalars.  Known dimensions decide where present;
    an unknown matrix is priced as a full one (the conservative choice: recomputation that
    would have to read it is never free)."""
    r = memo.get(h.id)
    if r is not None:
        return r
    if h.dt == "S" or h.op == "lit":
        r = 0.0
    elif h.dim1 >= 0 and h.dim2 >= 0:
        # narrow matrices (N x K, K <= ROW_MAXW: per-row vectors of products with side
        # matrices) are priced by their width like K per-row scalars
        r = 0.0 if h.dim1 * h.dim2 <= 1 else (1.0 if (h.dim1 > 1 and h.dim2 > ROW_MAXW) else 1e-3 * max(h.dim2, 1))
    else:
        k = _row_body_kind(h)
        if k in ("ragg", "dot"):
            r = 1e-3
        elif k == "cell":
            r = max((_size_class(c, memo) for c in _operands(h)), default=0.0)
        else:
            r = 1.0
    memo[h.id] = r
    return r


def _recompute_cost(c, region, leafset, memo, depth=0):
    """HBM cost (in full-matrix units) of evaluating hop c inside a region instead of reading
    its materialised value: the inputs it needs that the region does not already read; fusable
    inputs are themselves priced as min(read, recompute)."""
    kind = _row_body_kind(c)
    tot = 0.0
    for i, x in enumerate(c.inputs):
        if x.id in region or x.id in leafset or x.dt == "S" or x.op == "lit":
            continue
        if kind == "dot" and i == 1:
            tot += 1e-3                          # the D x 1 side vector
            continue
        if kind == "cell" and c.op == "b" and _is_sq(c) and i == 1:
            continue
        sx = _size_class(x, memo)
        if depth < 4 and _row_body_kind(x) is not None:
            sx = min(sx, _recompute_cost(x, region, leafset, memo, depth + 1))
        tot += sx
    return tot


def _consumers(order):
    cons = {}
    for h in order:
        for c in h.inputs:
            cons.setdefault(c.id, []).append(h)
    return cons


def fuse_rows(bb, costed=True):
    """Row template (reference: hops/codegen/template/TemplateRow.java, cplan/CNodeRow.java):
    regions of cellwise operators, row aggregates and matrix-vector products over the rows of
    a tall matrix, ending in a row / cellwise value, a column aggregate, a full aggregate or
    t(.) %*% a per-row scalar, become ONE generated kernel (ops/rowgen.py).

    Region growth, from the last operator of the block backwards:
      * closure -- an operator whose consumers are ALL in the region (and which is not a block
        output) joins it: the value never leaves registers;
      * cost-based recomputation (reference: the materialisation-point enumeration of
        hops/codegen/opt/PlanSelectionFuseCostBasedV2.java) -- a shared operator joins a region
        as a private recomputed copy when that costs no more HBM traffic than reading its
        materialised value (`_recompute_cost` <= its size class): e.g. X %*% v used by three
        row regions that all stream X anyway is recomputed in each, and the separate pass over
        X that would have materialised it disappears once no consumer is left.
    A region is only formed when the Cell template cannot do its work in one pass: it must
    contain a row aggregate or matrix-vector product whose result is used again inside the
    region, or end in a column / full aggregate or t(.) %*% over such a result.  Returns the
    number of fused operators."""
    from ..ops.rowgen import RowProgram, MAXIN as RMAXIN, MAXOPS as RMAXOPS
    live = getattr(bb, "live_out", None)
    allroots = list(bb.roots) + list(bb.env_out.values())
    outs = {h.id for h in bb.roots} | {h.id for k, h in bb.env_out.items() if live is None or k in live}
    tried = set()
    n = 0
    memo = {}
    while True:
        order = walk(allroots)
        pos = {h.id: i for i, h in enumerate(order)}
        consumers = _consumers(order)
        formed = False
        for root in reversed(order):
            if root.id in tried:
                continue
            tried.add(root.id)
            r = _form_row_region(root, consumers, outs, pos, memo, costed, RowProgram, RMAXIN, RMAXOPS)
            if r:
                n += r
                formed = True
                break                          # the DAG changed: recompute order and consumers
        if not formed:
            return n


def _row_key(h):
    """The matrix a Row-template hop streams: its first product's row operand, else its first
    matrix input that is not narrow (rows of the program)."""
    prog = h.p["prog"]
    for kind, _, a, _ in prog.ops:
        if kind == "dot" and a < prog.n_in:
            return h.inputs[a]
    for x in h.inputs:
        if x.dt == "M" and not (0 < x.dim2 <= ROW_MAXW):
            return x
    return None


def merge_row_programs(bb):
    """Multi-output Row template (reference: the multi-aggregate / multi-output CPlans of
    hops/codegen): Row-template hops of a block that stream the same matrix and do not depend
    on each other become ONE program with several outputs, its operators de-duplicated (a
    product X %*% B recomputed by several regions is computed once), so the kernel reads the
    rows once for all of them.  The original hops become fout views of the merged one.
    Returns the number of hops merged away."""
    from ..ops.rowgen import RowProgram, MAXIN as RMAXIN, MAXOPS as RMAXOPS, MAXOUT as RMAXOUT
    allroots = list(bb.roots) + list(bb.env_out.values())
    order = walk(allroots)
    rows = [h for h in order if h.op == "row" and not h.p["prog"].more]
    groups = {}
    for h in rows:
        k = _row_key(h)
        if k is not None:
            groups.setdefault(k.id, []).append(h)
    merged = 0
    if not ROW_MERGE:
        return 0
    for grp in groups.values():
        while len(grp) > 1:
            taken = [grp[0]]
            for h in grp[1:]:
                if len(taken) >= RMAXOUT:
                    break
                # independent of every taken hop, both ways
                if any(_reaches(h, t) or _reaches(t, h) for t in taken):
                    continue
                taken.append(h)
            grp = [h for h in grp if h not in taken]
            if len(taken) < 2:
                continue
            r = _merge(taken, RowProgram, RMAXIN, RMAXOPS)
            if r is None:
                continue
            prog, leaves = r
            M = Hop("row", leaves, {"o": prog.describe(), "prog": prog,
                                    "lines": sorted({ln for t in taken for ln in t.p.get("lines", ())})},
                    dt="U", pos=taken[0].pos)
            for i, t in enumerate(taken):
                t.op = "fout"
                t.inputs = [M]
                t.named = []
                t.p = {"i": i}
            merged += len(taken) - 1
    return merged


def _reaches(a, b):
    """b is (transitively) an input of a."""
    seen = set()
    stack = list(a.inputs)
    while stack:
        x = stack.pop()
        if x is b:
            return True
        if x.id in seen:
            continue
        seen.add(x.id)
        stack.extend(x.inputs)
    return False


def _merge(hops, RowProgram, RMAXIN, RMAXOPS):
    leaves = []

    def leaf(x):
        for i, y in enumerate(leaves):
            if y is x:
                return i
        leaves.append(x)
        return len(leaves) - 1
    maps = []
    for h in hops:
        maps.append([leaf(x) for x in h.inputs])
    nin = len(leaves)
    if nin > RMAXIN:
        return None
    ops, seen, outs = [], {}, []
    for h, m in zip(hops, maps):
        prog = h.p["prog"]
        loc = list(m)
        for kind, o, a, b in prog.ops:
            a2 = loc[a]
            b2 = loc[b] if kind in ("b", "dot", "cbindc", "wcolsv") else b
            key = (kind, o, a2, b2)
            j = seen.get(key)
            if j is None:
                ops.append(key)
                j = seen[key] = nin + len(ops) - 1
            loc.append(j)
        for node, ot, oagg, extra in prog.outputs():
            outs.append((loc[node], ot, oagg, loc[extra] if extra is not None else None))
    if len(ops) > RMAXOPS:
        return None
    p0 = outs[0]
    parts = tuple((h.p["prog"], tuple(m)) for h, m in zip(hops, maps))
    return RowProgram(nin, ops, p0[0], p0[1], p0[2], p0[3], more=outs[1:], parts=parts), leaves


def _form_row_region(root, consumers, outs, pos, memo, costed, RowProgram, RMAXIN, RMAXOPS):
    rk = _row_root_kind(root)
    bk = _row_body_kind(root)
    if rk is None and bk is None:
        return 0
    region = {root.id}
    kinds = {}
    if rk is None:
        kinds[root.id] = bk
        starts = _body_inputs(root, bk)
    else:
        starts = list(root.inputs) if rk == "tmv" else [root.inputs[0]]
    members = [root]
    dup = set()
    leafset = {c.id for c in starts}
    frontier = list(starts)
    changed = True
    while changed:
        changed = False
        for c in list(frontier):
            if c.id in region:
                continue
            ck = _row_body_kind(c)
            if ck is None:
                continue
            if ck in ("cbindc", "wcols") and c.inputs[0].id not in region and \
                    _row_body_kind(c.inputs[0]) not in ("dot", "cell", "cbindc", "wcols"):
                continue             # a plain matrix's column slice / append stays outside
            # closure: every consumer is in the region and none of them is a recomputed copy
            # (a copied operator stays alive outside the region and still reads c)
            closed = c.id not in outs and all(p.id in region and p.id not in dup for p in consumers.get(c.id, ()))
            if not closed:
                if not costed:
                    continue
                # ties go to recomputation: equal reads, and the materialising write disappears
                # once every consumer recomputes
                if _recompute_cost(c, region, leafset, memo) > _size_class(c, memo) + 1e-2:
                    continue
                dup.add(c.id)
            region.add(c.id)
            kinds[c.id] = ck
            members.append(c)
            leafset.discard(c.id)
            for x in _body_inputs(c, ck) + ([c.inputs[1]] if ck == "dot" else []):
                if x.id not in region:
                    leafset.add(x.id)
            frontier.extend(_body_inputs(c, ck))
            changed = True
    body = sorted((h for h in members if h.id in kinds), key=lambda h: pos[h.id])
    reds = [h for h in body if kinds[h.id] in ("ragg", "dot")]
    if not reds:
        return 0
    internal = any(any(p.id in kinds for p in consumers.get(r.id, ())) for r in reds)
    if not (internal or (rk is not None and len(body) >= 2)):
        return 0                 # a lone product / row aggregate: the plain operator is as good
    if rk == "tmv" and kinds.get(root.inputs[0].id) is None and kinds.get(root.inputs[1].id) is None:
        return 0
    # leaves: inputs of region hops outside the region, side vectors of dots included
    leaves = []

    def leaf(x):
        for i, y in enumerate(leaves):
            if y is x:
                return i
        leaves.append(x)
        return len(leaves) - 1
    for h in body:
        k = kinds[h.id]
        if k in ("cbindc", "wcols") and h.inputs[0].id not in kinds:
            return 0                 # applies to region products only
        if k == "cbindc":
            leaf(_const_col(h.inputs[1]))
            continue
        if k == "wcols":
            kb = _wcols_k(h)
            if not isinstance(kb, int):
                leaf(kb)
            continue
        for c in h.inputs:
            if c.id not in kinds and not (k == "cell" and h.op == "b" and _is_sq(h) and c is h.inputs[1]):
                leaf(c)
    if rk is not None:
        for c in (root.inputs if rk == "tmv" else root.inputs[:1]):
            if c.id not in kinds:
                leaf(c)
    if len(leaves) > RMAXIN or len(body) > RMAXOPS:
        return 0
    # a constant-column view cbind(X, c) (ops/augmented.ConstCol) is no dense row operand: the
    # generated kernel cannot read it, and a region over it would run operator by operator
    # (materialising its squares); its products stay the view's own passes
    if any(x.op == "bi" and x.p.get("name") == "_cbind_const" for x in leaves):
        return 0
    # a few very long rows (e.g. N x (C*H*W) activations of a small batch): one row per lane
    # group leaves the chip idle -- the unfused operators parallelise within rows instead
    for x in leaves:
        if x.dt == "M" and 0 < x.dim1 < 512 and x.dim2 > 1 and x.dim1 * x.dim2 >= (1 << 20):
            return 0
    nin = len(leaves)
    idx = {}
    ops = []

    def ref(x):
        return idx[x.id] if x.id in idx else leaf(x)
    for h in body:
        k = kinds[h.id]
        if k == "cell":
            if h.op == "b" and _is_sq(h):
                ops.append(("u", "sq", ref(h.inputs[0]), 0))
            elif h.op == "b":
                ops.append(("b", h.p["o"], ref(h.inputs[0]), ref(h.inputs[1])))
            else:
                ops.append(("u", h.p["o"], ref(h.inputs[0]), 0))
        elif k == "ragg":
            ops.append(("ragg", h.p["o"], ref(h.inputs[0]), 0))
        elif k == "cbindc":
            ops.append(("cbindc", None, ref(h.inputs[0]), ref(_const_col(h.inputs[1]))))
        elif k == "wcols":
            kb = _wcols_k(h)
            ops.append(("wcols", None, ref(h.inputs[0]), kb) if isinstance(kb, int)
                       else ("wcolsv", None, ref(h.inputs[0]), ref(kb)))
        else:
            ops.append(("dot", None, ref(h.inputs[0]), ref(h.inputs[1])))
        idx[h.id] = nin + len(ops) - 1
    if rk is None:
        prog = RowProgram(nin, ops, idx[root.id], "row" if bk == "ragg" else "vec")
    elif rk == "tmv":
        prog = RowProgram(nin, ops, ref(root.inputs[0]), "tmv", extra=ref(root.inputs[1]))
    else:
        prog = RowProgram(nin, ops, ref(root.inputs[0]), rk, oagg=root.p["o"])
    if len(leaves) != nin:
        return 0
    lines = sorted({getattr(o.pos, "line", None) for o in members} - {None})
    root.op = "row"
    root.inputs = list(leaves)
    root.named = []
    root.p = {"o": prog.describe(), "prog": prog, "lines": lines}
    return len(body)


# ----------------------------------------------------------------------------- Outer template
_SAFE_UN = {"abs", "sqrt", "sign", "neg", "round", "floor", "ceil", "sin", "tan", "asin", "atan", "sinh", "tanh"}


def _lit0(h):
    return h.op == "lit" and not isinstance(h.value, bool) and h.value == 0


def _zero_where(h, W, ids):
    """True when h's value is 0 wherever W's is (structural proof over the region `ids`)."""
    if h is W:
        return True
    if h.id not in ids:
        return False
    if h.op == "b":
        a, b = h.inputs
        o = h.p.get("o")
        if _is_sq(h):
            return _zero_where(a, W, ids)
        if o == "*":
            return _zero_where(a, W, ids) or _zero_where(b, W, ids)
        if o == "/":
            return _zero_where(a, W, ids)
        if o in ("+", "-"):
            return _zero_where(a, W, ids) and _zero_where(b, W, ids)
        if o == "!=":
            return (_zero_where(a, W, ids) and _lit0(b)) or (_zero_where(b, W, ids) and _lit0(a))
        if o == "^":
            return b.op == "lit" and not isinstance(b.value, bool) and isinstance(b.value, (int, float)) \
                and b.value > 0 and _zero_where(a, W, ids)
        return False
    if h.op == "u":
        return h.p.get("o") in _SAFE_UN and _zero_where(h.inputs[0], W, ids)
    return False


def _outer_root(h):
    """(output type, body hop, B) when h can end an Outer-template region."""
    if _cellwise(h):
        return "cell", h, None
    if h.op == "agg" and h.p.get("dir") == "all" and h.p.get("o") == "sum" and len(h.inputs) == 1 \
            and _cellwise(h.inputs[0]):
        return "all", h.inputs[0], None
    if h.op == "mm" and not h.p.get("mvagg") and len(h.inputs) == 2 and _cellwise(h.inputs[0]):
        return ("right" if h.p.get("transA") else "left"), h.inputs[0], h.inputs[1]
    return None


def fuse_outer(bb):
    """Outer-product template (reference: hops/codegen/template/TemplateOuterProduct.java):
    a cellwise DAG over U %*% t(V) that is zero wherever a driver matrix W is zero (proved
    structurally: W * g, g / ..., (W != 0), sums of such terms, f(0)=0 unaries) -- optionally
    summed, or multiplied by a matrix from the left (f %*% B) or the right (t(f) %*% B) --
    becomes one `outer` operator (ops/outer.py): with a sparse W the product is sampled at W's
    non-zeros only.  The region grows by closure (single-consumer cellwise operators), and
    U %*% t(V) must have no consumer outside it.  Returns the number of fused operators."""
    from ..ops.outer import OuterProgram
    from .rewrites import _uv
    live = getattr(bb, "live_out", None)
    allroots = list(bb.roots) + list(bb.env_out.values())
    outs = {h.id for h in bb.roots} | {h.id for k, h in bb.env_out.items() if live is None or k in live}
    order = walk(allroots)
    pos = {h.id: i for i, h in enumerate(order)}
    consumers = _consumers(order)
    absorbed = set()
    n = 0
    for root in reversed(order):
        if root.id in absorbed:
            continue
        r = _outer_root(root)
        if r is None:
            continue
        otype, top, B = r
        if top is not root and (top.id in outs or len(consumers.get(top.id, ())) != 1):
            continue
        region = {root.id, top.id}
        members = [top] if top is root else [root, top]
        frontier = list(_operands(top))
        uvs = []
        changed = True
        while changed:
            changed = False
            for c in list(frontier):
                if c.id in region:
                    continue
                if _uv(c) is not None and c.dt == "M":
                    # the low-rank product is always recomputed inside the region (sampled at
                    # the driver's non-zeros it costs less than reading a materialised m x n
                    # value); other consumers keep their own copy
                    region.add(c.id)
                    uvs.append(c)
                    changed = True
                    continue
                if c.id in absorbed or c.id in outs:
                    continue
                if not all(p.id in region for p in consumers.get(c.id, ())):
                    continue
                if not _cellwise(c) or _is_bias(c):
                    continue
                region.add(c.id)
                members.append(c)
                frontier.extend(_operands(c))
                changed = True
        if len(uvs) != 1 or _is_bias(top):
            continue
        uvh = uvs[0]
        U, V = _uv(uvh)
        ops = sorted((h for h in members if h.id in region and _cellwise(h)), key=lambda h: pos[h.id])
        leaves = []
        for h in ops:
            for c in _operands(h):
                if c.id not in region or c is uvh:
                    if all(c is not y for y in leaves):
                        leaves.append(c)
        if len(leaves) > MAXIN or len(ops) > MAXOPS:
            continue
        ids = {h.id for h in ops}
        W = next((x for x in leaves if x is not uvh and x.dt != "S" and x.op != "lit" and x is not U and x is not V
                  and _zero_where(top, x, ids)), None)
        if W is None:
            continue
        ra = _regalloc(ops, leaves)
        if ra is None:
            continue
        code, out = ra
        cprog = CellProgram(code, len(leaves), out)
        ui = next(i for i, x in enumerate(leaves) if x is uvh)
        wi = next(i for i, x in enumerate(leaves) if x is W)
        prog = OuterProgram(cprog, ui, wi, otype)
        ins = [U, V] + [x for x in leaves if x is not uvh] + ([B] if B is not None else [])
        lines = sorted({getattr(o.pos, "line", None) for o in ops + [root, uvh]} - {None})
        for h in ops + [root]:
            absorbed.add(h.id)
        root.op = "outer"
        root.inputs = ins
        root.named = []
        root.p = {"o": prog.describe(), "prog": prog, "lines": lines}
        n += len(ops) + 1
    return n


def _multi_agg(built):
    """MAgg template (reference: template/TemplateMultiAgg.java and the multi-aggregate
    merge of PlanSelectionFuseCostBased): full aggregates of fused cell programs that read a
    common matrix input are combined -- up to MAGG_MAX per group and MAXIN distinct inputs --
    into one `magg` hop evaluated in a single pass (ops/cell.evaluate_multi); each original
    aggregate hop becomes output i of it.  Aggregates that depend on each other are never
    grouped.  Returns the ids of the replaced roots."""
    done = set()
    # full aggregates (no per-channel operands), and column sums (per-channel operands
    # allowed: the batch-norm statistics of a convolution output) -- never mixed in one group
    alls = [b for b in built if b[3].agg and b[3].agg[1] == "all" and
            not any(o in ("bias+", "bias*") for _, o, _, _, _ in b[3].ops)]
    cols = [b for b in built if b[3].agg and b[3].agg[1] == "col" and b[3].agg[0] in ("sum", "sumsq", "mean")]
    for cands in (alls, cols):
        done |= _multi_agg_group(cands)
    return done


def _multi_agg_group(cands):
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


# ------------------------------------------------------------------ horizontal Cell batches
BATCH_MIN = 3      # smallest group of same-program Cell hops made one launch
BATCH_MAX_CELLS = 1 << 22   # largest member output batched


def batch_cells(bb):
    """Horizontal fusion of the Cell template: unaggregated Cell hops of a block that run the
    SAME program on different, independent operands -- the per-parameter optimizer updates of a
    network (`v = mu * v - lr * dW`, `W = W + v` once per weight) -- become one `hcell` hop whose
    kernel covers all of their cells in one launch (ops/cell.evaluate_batch: a per-operand table
    and a block -> operand map), instead of one launch per parameter.  Members must be
    independent (no member an ancestor of another), their matrix inputs of the output's shape
    and the rest scalars.  The original hops become fout views.  Returns the number of hops
    batched.  (Reference analogue: the multi-threaded per-parameter updates of the CP backend;
    on a GPU every tiny launch costs a few microseconds of device time.)"""
    allroots = list(bb.roots) + list(bb.env_out.values())
    order = walk(allroots)
    cand = []
    for h in order:
        if h.op != "cell":
            continue
        prog = h.p.get("prog")
        # small operands only (weights, per-channel vectors): batching delays every member to
        # the last one's inputs, which for activations would stretch their lifetimes
        if prog is None or prog.agg or h.dim1 <= 0 or h.dim2 <= 0 or h.dim1 * h.dim2 > BATCH_MAX_CELLS:
            continue
        kinds = []
        for x in h.inputs:
            if x.dt == "S":
                kinds.append("s")
            elif x.dt == "M" and ((x.dim1 == h.dim1 and x.dim2 == h.dim2) or x.dim1 < 0 or x.dim2 < 0):
                kinds.append("m")               # unknown dims: checked per operand set at run time
            else:
                kinds = None
                break
        if kinds is None or "m" not in kinds:
            continue
        cand.append((h, (prog.key(), tuple(kinds))))
    if len(cand) < BATCH_MIN:
        return 0
    groups = {}
    for h, k in cand:
        groups.setdefault(k, []).append(h)
    groups = {k: v for k, v in groups.items() if len(v) >= BATCH_MIN}
    if not groups:
        return 0
    n = 0
    for key in list(groups):
        # ancestor sets over this group's hops, as bitsets, in topological order -- recomputed
        # per group, since a batch made for an earlier group adds dependences (its hop reads
        # all of its members' inputs)
        order = walk(list(bb.roots) + list(bb.env_out.values()))
        members = [h for h in order if h.op == "cell" and h.id in {m.id for m in groups[key]}]
        bit = {h.id: 1 << i for i, h in enumerate(members)}
        anc = {}
        for h in order:
            a = 0
            for x in h.inputs:
                a |= anc.get(x.id, 0) | bit.get(x.id, 0)
            anc[h.id] = a
        rest = members
        while len(rest) >= BATCH_MIN:
            # greedy antichains in both topological directions, the larger one is taken (a member
            # that feeds all the others -- an early `a + b` ahead of the update sweep -- blocks the
            # forward sweep, the backward one skips it)
            fwd, mask = [], 0
            for h in rest:                      # forward: only earlier members can be ancestors
                if not anc[h.id] & mask:
                    fwd.append(h)
                    mask |= bit[h.id]
            bwd, under = [], 0
            for h in reversed(rest):            # backward: skip ancestors of the members taken
                if not bit[h.id] & under:
                    bwd.append(h)
                    under |= anc[h.id]
            taken = fwd if len(fwd) >= len(bwd) else bwd[::-1]
            ids = {t.id for t in taken}
            rest = [h for h in rest if h.id not in ids]
            if len(taken) < BATCH_MIN:
                break
            prog = taken[0].p["prog"]
            leaves = [x for t in taken for x in t.inputs]
            M = Hop("hcell", leaves, {"o": "batch[" + prog.describe() + f"]x{len(taken)}", "prog": prog,
                                      "n": len(taken), "lines": sorted({ln for t in taken
                                                                       for ln in t.p.get("lines", ())})},
                    dt="U", pos=taken[0].pos)
            for i, t in enumerate(taken):
                t.op = "fout"
                t.inputs = [M]
                t.named = []
                t.p = {"i": i}
            n += len(taken)
            # the taken hops are fouts of M now: later batches of this group must not read them
            # through M's inputs (rest are independent of taken by construction, but M reads all
            # taken inputs, so recompute reachability before the next batch)
            break
    return n
