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
    overwrites the same object -- or a left-indexed write that is not proven to address
    distinct cells per iteration (reference: runConstantCheck over LinearFunction).  A write
    is proven distinct when its row or column subscript is a linear function a*i + b of the
    parfor variable i with a != 0 (directly or through body variables defined once as linear
    functions of i; b may involve loop-invariant variables), or a range lo:hi with
    lo = a*i + b1, hi = a*i + b2 whose width b2 - b1 is provably smaller than the step a
    (e.g. (i-1)*bs+1 : i*bs).  Nested loop variables, data-dependent or non-linear
    subscripts (ceil(i/2), i*i, as.scalar(...) of iteration data) prove nothing;
  * data / anti dependency: a candidate read in the body without indexing (the whole object
    sees other iterations' writes), or read through a subscript that differs from the
    subscript it is written through (the reference resolves some of these pairs with GCD /
    Banerjee tests over linear subscripts; here only identical subscripts are proven
    independent).
A subscript "depends on the iteration variable" when it references it directly or through a
body variable computed from it (transitive closure over the body's assignments).  Symbolic
coefficients (a loop-invariant block size) are taken as non-zero, as the reference does.
"""
from __future__ import annotations

import math

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
        self.acc_writes = {}       # var -> pos of plain `var += ...` updates
        self.defs = []             # (var, vars of the defining expression) for dependence closure
        self.def_exprs = {}        # var -> [defining expressions] (None: not an expression def)
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
            if e.name in ("nrow", "ncol", "length") and len(e.args) == 1 and isinstance(e.args[0].value, A.Ident):
                return                 # shape queries read no cells (iterations never change shapes)
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
                elif st.accumulate:
                    self.acc_writes.setdefault(t.name, pos)
                    self.defs.append((t.name, _expr_vars(st.value, set()) | {t.name}))
                    self.def_exprs.setdefault(t.name, []).append(None)
                else:
                    self.plain_writes.setdefault(t.name, pos)
                    self.defs.append((t.name, _expr_vars(st.value, set())))
                    self.def_exprs.setdefault(t.name, []).append(None if st.accumulate else st.value)
            elif isinstance(st, A.MultiAssign):
                self.read(st.value, pos)
                srcs = _expr_vars(st.value, set())
                for t in st.targets:
                    self.plain_writes.setdefault(t.name, pos)
                    self.defs.append((t.name, srcs))
                    self.def_exprs.setdefault(t.name, []).append(None)
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
                self.def_exprs.setdefault(st.var, []).append(None)
                self.defs.append((st.var, _expr_vars(st.start, set()) | _expr_vars(st.end, set())))
                self.stmts(st.body)


# --- linear subscript forms ---------------------------------------------------------------
# A polynomial over loop-invariant symbols is a dict monomial -> number (a monomial is a
# sorted tuple of symbol keys; () is the constant term).  A subscript's linear form in the
# parfor variable is (coef, const), both polynomials.

def _padd(a, b, sign=1.0):
    out = dict(a)
    for k, v in b.items():
        out[k] = out.get(k, 0.0) + sign * v
    return {k: v for k, v in out.items() if v != 0}


def _pmul(a, b):
    out = {}
    for ka, va in a.items():
        for kb, vb in b.items():
            k = tuple(sorted(ka + kb))
            out[k] = out.get(k, 0.0) + va * vb
    return {k: v for k, v in out.items() if v != 0}


def _pconst(p):
    """The number a polynomial equals, or None when it has symbolic terms."""
    if not p:
        return 0.0
    if set(p) == {()}:
        return p[()]
    return None


_SCALAR_CALLS = {"nrow", "ncol", "length", "as.scalar", "as.integer", "as.double", "as.logical",
                 "sum", "mean", "avg", "prod", "var", "sd", "trace", "castAsScalar", "floor", "ceil",
                 "ceiling", "round", "abs", "sqrt", "exp", "log"}


def _is_scalar(e, scalars):
    """Whether expression `e` is scalar-valued (literals, scalar variables, shape queries /
    full aggregates / scalar casts, arithmetic over those)."""
    if isinstance(e, (A.Literal, A.CmdParam)):
        return True
    if isinstance(e, A.Ident):
        return e.name in scalars
    if isinstance(e, A.UnOp):
        return _is_scalar(e.operand, scalars)
    if isinstance(e, A.BinOp):
        return _is_scalar(e.left, scalars) and _is_scalar(e.right, scalars)
    if isinstance(e, A.Call) and e.namespace in (None, ".builtinNS"):
        if e.name in ("nrow", "ncol", "length", "as.scalar", "castAsScalar", "sum", "mean", "avg",
                      "prod", "var", "sd", "trace"):
            return True
        if e.name in _SCALAR_CALLS or e.name in ("min", "max"):
            return all(_is_scalar(x.value, scalars) for x in e.args)
    return False


def _integral(p):
    return all(float(v).is_integer() for v in p.values())


class _Linear:
    """Linear forms a*i + b of subscript expressions in the parfor variable i, and the
    pairwise disjointness tests over them (reference: ParForStatementBlock's LinearFunction,
    runConstantCheck, GCD and Banerjee tests)."""

    def __init__(self, st, body, dep, scalars):
        self.var, self.body, self.dep, self.scalars = st.var, body, dep, scalars
        self.active = set()
        self.bounds = None                     # numeric (first, last) iteration value
        try:
            f, t = float(st.start.value), float(st.end.value)
            inc = 1.0 if st.incr is None else float(st.incr.value)
            if inc > 0 and t >= f:
                self.bounds = (f, f + inc * math.floor((t - f) / inc))
        except (AttributeError, TypeError, ValueError):
            pass

    def form(self, e):
        if e is None:
            return None
        if isinstance(e, A.Literal):
            try:
                return {}, _padd({}, {(): float(e.value)})
            except (TypeError, ValueError):
                return None
        names = _expr_vars(e, set())
        if not (names & self.dep):
            if not _is_scalar(e, self.scalars):
                return None                     # e.g. a matrix-valued factor
            return {}, {(("e", _ekey(e)),): 1.0}   # loop-invariant scalar: an opaque symbol
        if isinstance(e, A.Ident):
            if e.name == self.var:
                return {(): 1.0}, {}
            defs = self.body.def_exprs.get(e.name, [])
            if len(defs) != 1 or defs[0] is None or e.name in self.body.inner_loop_vars \
                    or e.name in self.active:
                return None
            self.active.add(e.name)
            try:
                return self.form(defs[0])
            finally:
                self.active.discard(e.name)
        if isinstance(e, A.UnOp) and e.op in ("-", "+"):
            f = self.form(e.operand)
            if f is None or e.op == "+":
                return f
            return _padd({}, f[0], -1.0), _padd({}, f[1], -1.0)
        if isinstance(e, A.BinOp) and e.op in ("+", "-", "*", "/"):
            l, r = self.form(e.left), self.form(e.right)
            if l is None or r is None:
                return None
            if e.op in ("+", "-"):
                sg = 1.0 if e.op == "+" else -1.0
                return _padd(l[0], r[0], sg), _padd(l[1], r[1], sg)
            if e.op == "*":
                if not l[0]:
                    return _pmul(l[1], r[0]), _pmul(l[1], r[1])
                if not r[0]:
                    return _pmul(r[1], l[0]), _pmul(r[1], l[1])
                return None
            d = _pconst(r[1])
            if r[0] or not d:
                return None
            return _pmul(l[0], {(): 1.0 / d}), _pmul(l[1], {(): 1.0 / d})
        return None

    def _resolve(self, e):
        """The defining expression of a body variable assigned once (else e itself)."""
        seen = set()
        while isinstance(e, A.Ident) and e.name not in seen:
            seen.add(e.name)
            defs = self.body.def_exprs.get(e.name, [])
            if len(defs) != 1 or defs[0] is None or e.name in self.body.inner_loop_vars:
                break
            e = defs[0]
        return e

    def interval(self, r):
        """(a, lo, hi): the subscript addresses [a*i + lo, a*i + hi]; None = unknown / all."""
        if r is None or r.lower is None:
            return None
        lo = self.form(r.lower)
        low = self._resolve(r.lower)
        if lo is None and isinstance(low, A.Call) and low.name == "max" and r.is_range:
            # a lower bound max(a, ...) addresses a subset of [a, hi]
            for a in low.args:
                f = self.form(a.value)
                if f is not None and f[0]:
                    lo = f
                    break
        if lo is None or not all(_integral(x) for x in lo):
            return None
        if not r.is_range or r.upper is None:
            return lo[0], lo[1], lo[1]
        # an upper bound min(a, b, ...) addresses a subset of [lo, a]: any argument with lo's
        # step gives a sound (wider) interval, e.g. beg:min(N, beg + bs - 1)
        up = self._resolve(r.upper)
        ups = [r.upper]
        if isinstance(up, A.Call) and up.name == "min" and up.namespace in (None, ".builtinNS"):
            ups = [a.value for a in up.args]
        for u in ups:
            hi = self.form(u)
            if hi is not None and not _padd(hi[0], lo[0], -1.0) and _integral(hi[1]):
                return lo[0], lo[1], hi[1]
        return None

    def _span(self, iv):
        """Numeric [min, max] of the cells an interval addresses over the whole loop."""
        if self.bounds is None:
            return None
        a, lo, hi = (_pconst(x) for x in iv)
        if a is None or lo is None or hi is None:
            return None
        ends = [a * self.bounds[0], a * self.bounds[1]]
        return min(ends) + lo, max(ends) + hi

    def disjoint(self, r1, r2):
        """True when subscript r1 in iteration i1 and r2 in iteration i2 address disjoint
        index sets for every i1 != i2 (r1 is r2 for the self-check of one write)."""
        v1, v2 = self.interval(r1), self.interval(r2)
        if v1 is None or v2 is None:
            return False
        # Banerjee-style bounds test: the index ranges over the whole loop never meet
        s1, s2 = self._span(v1), self._span(v2)
        if s1 is not None and s2 is not None and (s1[1] < s2[0] or s2[1] < s1[0]):
            return True
        (a1, l1, u1), (a2, l2, u2) = v1, v2
        if a1 and not _padd(a1, a2, -1.0):
            # same non-zero step a: a*(i1 - i2) shifts one interval past the other for |i1 - i2| >= 1
            c = _pconst(a1)
            step = {(): abs(c)} if c is not None else a1
            g1 = _pconst(_padd(_padd(step, l1), u2, -1.0))
            g2 = _pconst(_padd(_padd(step, l2), u1, -1.0))
            if g1 is not None and g2 is not None and g1 > 0 and g2 > 0:
                return True
        # GCD test on two single indices a1*i1 + b1 = a2*i2 + b2
        c1, c2 = _pconst(a1), _pconst(a2)
        b = _pconst(_padd(l2, l1, -1.0))
        if l1 == u1 and l2 == u2 and c1 is not None and c2 is not None and b is not None and (c1 or c2):
            g = math.gcd(int(c1), int(c2))
            if b % g != 0:
                return True
        return False

    def disjoint_cells(self, w1, w2):
        """Two (rows, cols) subscripts never address a common cell from different iterations."""
        return self.disjoint(w1[0], w2[0]) or (w1[1] is not None and w2[1] is not None
                                                and self.disjoint(w1[1], w2[1]))


def accumulators(body, scalars=frozenset()):
    """Matrix variables only updated through plain `+=` in the body and not otherwise used
    there: parfor accumulators (reference parfor_accumulator tests), merged as the sum of
    every worker's increments.  A scalar `s += ...` stays an output dependency, as in the
    reference (ParForStatementBlock.rCheckCandidates accumulates matrices only)."""
    out = set()
    for v in body.acc_writes:
        if v in scalars:
            continue
        if v not in body.plain_writes and v not in body.reads_whole and v not in body.ix_writes \
                and v not in body.reads_ix:
            out.add(v)
    return out


def loop_accumulators(st: A.For, scalars=frozenset()):
    """Accumulator variables (`v += ...` only) of a parfor statement."""
    body = _Body()
    body.stmts(st.body)
    return sorted(accumulators(body, scalars))


def check_parfor(st: A.For, defined_before, scalars=frozenset()):
    """Raise LanguageError on loop-carried dependencies of parfor statement `st`; variables in
    `defined_before` exist at loop entry, `scalars` are known scalar variables.  `check=0`
    disables the analysis.  Records the loop's accumulator variables on `st.accumulators`."""
    body = _Body()
    body.stmts(st.body)
    st.accumulators = sorted(accumulators(body, scalars))
    chk = st.params.get("check")
    if isinstance(chk, A.Literal) and str(chk.value) in ("0", "False", "false", "FALSE"):
        return
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

    lin = _Linear(st, body, dep, set(scalars) | {st.var})
    cands = (set(body.plain_writes) | set(body.ix_writes) | set(body.acc_writes)) & set(defined_before)
    cands -= set(st.accumulators)
    cands.discard(st.var)
    bad = []
    for c in sorted(cands):
        why = None
        if c in body.plain_writes or c in body.acc_writes:
            why = "output dependency (every iteration assigns the whole variable)"
        elif c in body.reads_whole:
            why = "data dependency (read without subscript while written per iteration)"
        else:
            writes = [(r, cc) for r, cc, _, acc in body.ix_writes[c]]
            if any(not lin.disjoint_cells(w, w) for w in writes):
                why = ("output dependency (left-indexing not proven to address distinct cells per "
                       "iteration: no subscript linear in the loop variable)")
            elif any(not lin.disjoint_cells(w1, w2) for k, w1 in enumerate(writes) for w2 in writes[k + 1:]):
                why = "output dependency (two left-indexing writes may address the same cells)"
            else:
                wkeys = {(_sub_key(r), _sub_key(cc)) for r, cc in writes}
                for r, cc, _ in body.reads_ix.get(c, []):
                    rd = (r, cc)
                    if (_sub_key(r), _sub_key(cc)) in wkeys and len(wkeys) == 1:
                        continue
                    if not all(lin.disjoint_cells(rd, w) for w in writes):
                        why = "data/anti dependency (a read may address cells other iterations write)"
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
    out = set(b.plain_writes) | set(b.ix_writes) | set(b.acc_writes)
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

    def walk(stmts, defined, after, loop=False, scalars=frozenset()):
        defined = set(defined)
        scalars = set(scalars)
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
                        check_parfor(st, defined | later, scalars)
                    inner_after = later | (_expr_vars(st.pred, set()) if isinstance(st, A.While) else set())
                    walk(st.body, defined | ({st.var} if isinstance(st, A.For) else set()), inner_after, loop=True,
                         scalars=scalars | ({st.var} if isinstance(st, A.For) else set()))
            if isinstance(st, A.Assign) and isinstance(st.target, A.Ident):
                if not st.accumulate and _is_scalar(st.value, scalars):
                    scalars.add(st.target.name)
                elif not (st.accumulate and st.target.name in scalars and _is_scalar(st.value, scalars)):
                    scalars.discard(st.target.name)
            else:
                for v in _assigned(st):
                    scalars.discard(v)
                if isinstance(st, A.For):
                    scalars.add(st.var)
            defined |= _assigned(st)

    walk(prog.statements, set(), set())
    fns = list(prog.functions.values())
    for ns in (prog.namespaces or {}).values():
        fns.extend(ns.values())
    for fd in fns:
        if not getattr(fd, "external", False) and any(_has_parfor(x, memo) for x in fd.body):
            walk(fd.body, {p.name for p in fd.inputs}, {p.name for p in fd.outputs},
                 scalars={p.name for p in fd.inputs if str(getattr(p, "dtype", "")).lower().startswith("scalar")
                          or str(getattr(p, "dtype", "")).lower() in ("int", "integer", "double", "boolean")})
