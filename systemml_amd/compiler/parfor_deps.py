"""Loop dependency analysis of parfor bodies (reference: parser/ParForStatementBlock.java
#validate: candidate determination, the constant self-check for output dependencies and the
pairwise write/read checks; `check=0` skips the analysis).

A parfor may only write variables that existed before the loop through left-indexing whose
subscript depends on the iteration variable, so that every iteration writes its own cells;
anything else makes the result depend on the iteration order.  The analysis is conservative
(no false negatives, possibly false positives -- the reference gives the same guarantee):

  * candidates: variables written in the body (also inside nested control flow) that are
    defined before the loop or read after it (later statements, enclosing loop bodies) --
    variables only used inside the body are iteration-private;
  * output dependency: a plain (non-indexed) assignment to a candidate -- every iteration
    overwrites the same object -- or a left-indexed write whose row and column subscripts
    are both loop-invariant (reference: runConstantCheck);
  * data / anti dependency: a candidate read in the body without indexing (the whole object
    sees other iterations' writes), or read through a subscript that differs from the
    subscript it is written through (the reference resolves some of these pairs with GCD /
    Banerjee tests over linear subscripts; here only identical subscripts are proven
    independent).
A subscript "depends on the iteration variable" when it references it directly or through a
body variable computed from it (transitive closure over the body's assignments).
"""
from __future__ import annotations

from ..parser import ast as A
from ..parser.errors import LanguageError


def _expr_vars(e, out):
    """Variable names an expression reads (Indexed counts its base variable)."""
    if e is None:
        return out
    if isinstance(e, A.Ident):
        out.add(e.name)
    elif isinstance(e, A.Indexed):
        out.add(e.name)
        for r in (e.rows, e.cols):
            if r is not None:
                _expr_vars(r.lower, out)
                _expr_vars(r.upper, out)
    elif isinstance(e, A.BinOp):
        _expr_vars(e.left, out)
        _expr_vars(e.right, out)
    elif isinstance(e, A.UnOp):
        _expr_vars(e.operand, out)
    elif isinstance(e, A.Call):
        for a in e.args:
            _expr_vars(a.value, out)
    elif isinstance(e, A.ExprList):
        for x in e.items:
            _expr_vars(x, out)
    return out


def _sub_key(e):
    """Canonical text of a subscript (IndexRange or None) for identity comparison."""
    if e is None:
        return None
    return (_ekey(e.lower), _ekey(e.upper), bool(e.is_range))


def _ekey(e):
    if e is None:
        return None
    if isinstance(e, A.Literal):
        return ("lit", e.value)
    if isinstance(e, A.Ident):
        return ("id", e.name)
    if isinstance(e, A.BinOp):
        return ("b", e.op, _ekey(e.left), _ekey(e.right))
    if isinstance(e, A.UnOp):
        return ("u", e.op, _ekey(e.operand))
    if isinstance(e, A.Call):
        return ("c", e.namespace, e.name, tuple((a.name, _ekey(a.value)) for a in e.args))
    if isinstance(e, A.Indexed):
        return ("ix", e.name, _sub_key(e.rows), _sub_key(e.cols))
    return ("?", id(e))


class _Body:
    """Writes and reads of a parfor body (recursively through nested control flow)."""

    def __init__(self):
        self.plain_writes = {}     # var -> first statement position
        self.ix_writes = {}        # var -> [(rows, cols, pos)]
        self.reads_whole = {}      # var -> pos (reads without subscript)
        self.reads_ix = {}         # var -> [(rows, cols, pos)]
        self.defs = []             # (var, vars of the defining expression) for dependence closure
        self.inner_loop_vars = set()

    def read(self, e, pos):
        if e is None:
            return
        if isinstance(e, A.Ident):
            self.reads_whole.setdefault(e.name, pos)
        elif isinstance(e, A.Indexed):
            self.reads_ix.setdefault(e.name, []).append((e.rows, e.cols, pos))
            for r in (e.rows, e.cols):
                if r is not None:
                    self.read(r.lower, pos)
                    self.read(r.upper, pos)
        elif isinstance(e, A.BinOp):
            self.read(e.left, pos)
            self.read(e.right, pos)
        elif isinstance(e, A.UnOp):
            self.read(e.operand, pos)
        elif isinstance(e, A.Call):
            for a in e.args:
                self.read(a.value, pos)
        elif isinstance(e, A.ExprList):
            for x in e.items:
                self.read(x, pos)

    def stmts(self, body):
        for st in body:
            pos = getattr(st, "pos", None)
            if isinstance(st, A.Assign):
                self.read(st.value, pos)
                t = st.target
                if isinstance(t, A.Indexed):
                    for r in (t.rows, t.cols):
                        if r is not None:
                            self.read(r.lower, pos)
                            self.read(r.upper, pos)
                    self.ix_writes.setdefault(t.name, []).append((t.rows, t.cols, pos, st.accumulate))
                    if st.accumulate:
                        self.reads_ix.setdefault(t.name, []).append((t.rows, t.cols, pos))
                else:
                    if st.accumulate:
                        self.reads_whole.setdefault(t.name, pos)
                    self.plain_writes.setdefault(t.name, pos)
                    self.defs.append((t.name, _expr_vars(st.value, set())))
            elif isinstance(st, A.MultiAssign):
                self.read(st.value, pos)
                srcs = _expr_vars(st.value, set())
                for t in st.targets:
                    self.plain_writes.setdefault(t.name, pos)
                    self.defs.append((t.name, srcs))
            elif isinstance(st, A.ExprStmt):
                self.read(st.call, pos)
            elif isinstance(st, A.If):
                self.read(st.pred, pos)
                self.stmts(st.then_body)
                self.stmts(st.else_body)
            elif isinstance(st, A.While):
                self.read(st.pred, pos)
                self.stmts(st.body)
            elif isinstance(st, A.For):
                for e in (st.start, st.end, st.incr):
                    self.read(e, pos)
                self.inner_loop_vars.add(st.var)
                self.defs.append((st.var, _expr_vars(st.start, set()) | _expr_vars(st.end, set())))
                self.stmts(st.body)


def check_parfor(st: A.For, defined_before):
    """Raise LanguageError on loop-carried dependencies of parfor statement `st`; variables in
    `defined_before` exist at loop entry.  `check=0` disables the analysis."""
    chk = st.params.get("check")
    if isinstance(chk, A.Literal) and str(chk.value) in ("0", "False", "false", "FALSE"):
        return
    body = _Body()
    body.stmts(st.body)
    # variables whose value depends on the iteration variable (fixpoint over the body's defs;
    # nested loop variables vary within an iteration and count as iteration-dependent)
    dep = {st.var} | body.inner_loop_vars
    changed = True
    while changed:
        changed = False
        for v, srcs in body.defs:
            if v not in dep and srcs & dep:
                dep.add(v)
                changed = True

    def varies(r):
        if r is None:
            return False
        return bool((_expr_vars(r.lower, set()) | _expr_vars(r.upper, set())) & dep)

    cands = (set(body.plain_writes) | set(body.ix_writes)) & set(defined_before)
    cands.discard(st.var)
    bad = []
    for c in sorted(cands):
        why = None
        if c in body.plain_writes:
            why = "output dependency (every iteration assigns the whole variable)"
        else:
            writes = body.ix_writes[c]
            if any(not varies(r) and not varies(cc) and not acc for r, cc, _, acc in writes):
                why = "output dependency (left-indexing with a loop-invariant subscript)"
            elif c in body.reads_whole:
                why = "data dependency (read without subscript while written per iteration)"
            else:
                wkeys = {(_sub_key(r), _sub_key(cc)) for r, cc, _, _ in writes}
                for r, cc, _ in body.reads_ix.get(c, []):
                    if (_sub_key(r), _sub_key(cc)) not in wkeys:
                        why = "data/anti dependency (read through a different subscript than written)"
                        break
        if why:
            bad.append(f"{c} [{why}]")
    if bad:
        raise LanguageError(f"{st.pos}: PARFOR loop dependency analysis: inter-iteration (loop-carried) "
                            f"dependencies detected for variable(s): {', '.join(bad)}. Please, ensure "
                            f"independence of iterations (or set check=0).")


def _exposed(stmts, killed=()):
    """(upward-exposed reads, definitely-assigned variables) of a statement list: variables
    read before every path through the list has assigned them (a left-indexed write reads
    the cells it keeps)."""
    killed = set(killed)
    exp = set()

    def rd(e):
        exp.update(_expr_vars(e, set()) - killed)

    for st in stmts:
        if isinstance(st, A.Assign):
            rd(st.value)
            t = st.target
            if isinstance(t, A.Indexed):
                for r in (t.rows, t.cols):
                    if r is not None:
                        rd(r.lower)
                        rd(r.upper)
                if t.name not in killed:
                    exp.add(t.name)
            else:
                if st.accumulate and t.name not in killed:
                    exp.add(t.name)
                killed.add(t.name)
        elif isinstance(st, A.MultiAssign):
            rd(st.value)
            killed.update(t.name for t in st.targets)
        elif isinstance(st, A.ExprStmt):
            rd(st.call)
        elif isinstance(st, A.If):
            rd(st.pred)
            e1, k1 = _exposed(st.then_body, killed)
            e2, k2 = _exposed(st.else_body, killed)
            exp |= e1 | e2
            killed |= (k1 & k2)
        elif isinstance(st, A.While):
            rd(st.pred)
            exp |= _exposed(st.body, killed)[0]
        elif isinstance(st, A.For):
            for e in (st.start, st.end, st.incr):
                rd(e)
            exp |= _exposed(st.body, killed | {st.var})[0]
    return exp, killed


def _assigned(st):
    b = _Body()
    b.stmts([st])
    out = set(b.plain_writes) | set(b.ix_writes)
    if isinstance(st, A.For):
        out.add(st.var)
    return out


def _has_parfor(st, memo):
    k = id(st)
    r = memo.get(k)
    if r is None:
        if isinstance(st, A.For) and st.parfor:
            r = True
        elif isinstance(st, A.If):
            r = any(_has_parfor(x, memo) for x in st.then_body) or any(_has_parfor(x, memo) for x in st.else_body)
        elif isinstance(st, (A.For, A.While)):
            r = any(_has_parfor(x, memo) for x in st.body)
        else:
            r = False
        memo[k] = r
    return r


def check_program(prog: A.Program):
    """Run the analysis on every parfor of the program and its functions (before translation).
    Only statement subtrees that contain a parfor are walked (the read-after sets are
    computed there alone), so programs without parfor pay one linear scan."""
    memo = {}

    def walk(stmts, defined, after, loop=False):
        defined = set(defined)
        for k, st in enumerate(stmts):
            if _has_parfor(st, memo):
                # upward-exposed reads that follow statement k: the rest of the list, what
                # follows the list, and in a loop body the statements before k (next iteration)
                e1, k1 = _exposed(stmts[k + 1:])
                later = e1 | (after - k1)
                if loop:
                    later |= _exposed(stmts[:k], k1)[0]
                if isinstance(st, A.If):
                    walk(st.then_body, defined, later)
                    walk(st.else_body, defined, later)
                elif isinstance(st, (A.For, A.While)):
                    if isinstance(st, A.For) and st.parfor:
                        check_parfor(st, defined | later)
                    inner_after = later | (_expr_vars(st.pred, set()) if isinstance(st, A.While) else set())
                    walk(st.body, defined | ({st.var} if isinstance(st, A.For) else set()), inner_after, loop=True)
            defined |= _assigned(st)

    walk(prog.statements, set(), set())
    fns = list(prog.functions.values())
    for ns in (prog.namespaces or {}).values():
        fns.extend(ns.values())
    for fd in fns:
        if not getattr(fd, "external", False) and any(_has_parfor(x, memo) for x in fd.body):
            walk(fd.body, {p.name for p in fd.inputs}, {p.name for p in fd.outputs})
