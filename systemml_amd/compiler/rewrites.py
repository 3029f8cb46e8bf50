"""Static HOP rewrites (reference: hops/rewrite/RewriteConstantFolding.java,
RewriteAlgebraicSimplificationStatic.java, RewriteAlgebraicSimplificationDynamic.java,
RewriteCommonSubexpressionElimination.java and the fused-operator selection of
hops/AggBinaryOp.java (MMTSJ / MapMultChain) and hops/codegen row templates).

Rules implemented (applied bottom-up until fixpoint per node):
  * constant folding of scalar binary / unary ops
  * t(t(X)) -> X ; X*1, 1*X, X/1, X+0, 0+X, X-0, X^1 -> X
  * sum(X^2) -> sumsq(X); rowSums(X^2) / colSums(X^2) -> row/col sumsq
  * sum(X*Y) -> tak(X,Y)  (ternary aggregate, no materialised product)
  * sum(t(X)) -> sum(X)
  * t(X) %*% Y -> mm(X, Y, transA)      (no materialised transpose)
  * t(X) %*% X -> tsmm(X, LEFT),  X %*% t(X) -> tsmm(X, RIGHT)
  * t(X)%*%(X%*%v)        -> mmchain XtXv
    t(X)%*%(w*(X%*%v))    -> mmchain XtwXv
    t(X)%*%((X%*%v)-y)    -> mmchain XtXvy
    t(X)%*%(Q - P*rowSums(Q)), Q = P*(X%*%V)  -> mmchain XtPSXv (multinomial-logreg
        Hessian-vector product; a codegen "Row template" instance)
  * A op (v %*% matrix(1,1,k)) -> A op v  (unnecessary outer product → broadcast)
  * common subexpression elimination (hash consing)
"""
from __future__ import annotations

from ..runtime import scalars as S
from ..parser.errors import DMLRuntimeError
from .hops import Hop, lit
from . import hops as H

CELLWISE = {"+", "-", "*", "/", "^", "%%", "%/%", "==", "!=", "<", "<=", ">", ">=", "&", "|",
            "min", "max", "xor"}


def _is_lit(h, v=None):
    if h.op != "lit":
        return False
    if v is None:
        return True
    x = h.value
    return isinstance(x, (int, float)) and not isinstance(x, bool) and x == v


def _is_ones_matrix(h, rows1=None, cols1=None):
    """matrix(1, rows=.., cols=..) datagen with literal fill 1."""
    if h.op != "bi" or h.p.get("name") != "matrix":
        return False
    if not h.inputs or not _is_lit(h.inputs[0], 1):
        return False
    args = _bi_args(h)
    r = args.get("rows")
    c = args.get("cols")
    if rows1 and not (r is not None and _is_lit(r, 1)):
        return False
    if cols1 and not (c is not None and _is_lit(c, 1)):
        return False
    return True


def _bi_args(h):
    npos = h.p.get("npos", len(h.inputs) - len(h.named))
    names = ["data", "rows", "cols"] if h.p.get("name") == "matrix" else []
    out = {}
    for i in range(npos):
        if i < len(names):
            out[names[i]] = h.inputs[i]
    for j, n in enumerate(h.named):
        out[n] = h.inputs[npos + j]
    return out


_NOT_CMP = {"==": "!=", "!=": "==", "<": ">=", ">=": "<", ">": "<=", "<=": ">"}


def _num_lit(h):
    return h.op == "lit" and isinstance(h.value, (int, float)) and not isinstance(h.value, bool)


def _full_range(src, lo, hi, dimop):
    """Index range [lo, hi] covering the whole dimension: empty (None) bounds, or 1 .. nrow/ncol(src)."""
    if lo.op == "lit" and lo.value is None and hi.op == "lit" and hi.value is None:
        return True
    return _is_lit(lo, 1) and hi.op == "u" and hi.p["o"] == dimop and hi.inputs[0] is src


def _vec_kind(h):
    """'col' / 'row' when h is a column / row vector by construction, else None."""
    if h.op == "agg" and h.p.get("dir") == "row":
        return "col"
    if h.op == "agg" and h.p.get("dir") == "col":
        return "row"
    if h.op == "t":
        k = _vec_kind(h.inputs[0])
        return {"col": "row", "row": "col"}.get(k)
    if _is_ones_matrix(h) or (h.op == "bi" and h.p.get("name") in ("matrix", "rand")):
        args = _bi_args(h) if h.p.get("name") == "matrix" else {}
        if h.p.get("name") == "rand":
            npos = h.p.get("npos", len(h.inputs) - len(h.named))
            args = {n: h.inputs[npos + j] for j, n in enumerate(h.named)}
        if set(args) & {"data", "rows", "cols"} and args.get("cols") is not None and _is_lit(args["cols"], 1):
            return "col"
        if args.get("rows") is not None and _is_lit(args["rows"], 1):
            return "row"
    return None


def _equal_size(A, B):
    """dims(A) == dims(B): the same hop, or both sizes known and equal (HopRewriteUtils
    .isEqualSize)."""
    if A is B:
        return True
    return min(A.dim1, A.dim2, B.dim1, B.dim2) > 0 and (A.dim1, A.dim2) == (B.dim1, B.dim2)


def _smaller(h, x):
    """Known sizes with cells(h) < cells(x) (HopRewriteUtils.compareSize < 0)."""
    return min(h.dim1, h.dim2, x.dim1, x.dim2) > 0 and h.dim1 * h.dim2 < x.dim1 * x.dim2


def _seq_args(h):
    if h.op != "bi" or h.p.get("name") != "seq" or h.named:
        return None
    a = h.inputs[:h.p.get("npos", len(h.inputs))]
    return a if len(a) in (2, 3) else None


def _basic_1n_seq(h):
    """n when h is seq(1, n[, 1]) (HopRewriteUtils.isBasic1NSequence), else None."""
    a = _seq_args(h)
    if a is None or not _is_lit(a[0], 1) or (len(a) == 3 and not _is_lit(a[2], 1)):
        return None
    return a[1]


def _basic_n1_seq(h):
    """n when h is seq(n, 1, -1) (isBasicN1Sequence), else None."""
    a = _seq_args(h)
    if a is None or len(a) != 3 or not _is_lit(a[1], 1) or not _is_lit(a[2], -1):
        return None
    return a[0]


def _same_hop_value(a, b):
    """a and b denote the same scalar: one hop, equal literals, or nrow/ncol of one hop."""
    if a is b:
        return True
    if _num_lit(a) and _num_lit(b):
        return a.value == b.value
    return a.op == "u" and b.op == "u" and a.p.get("o") == b.p.get("o") and a.p.get("o") in ("nrow", "ncol") \
        and a.inputs[0] is b.inputs[0]


def _const_datagen_value(h):
    """The scalar of a constant datagen matrix(c, rows, cols) / rand(min=c, max=c), else None
    (HopRewriteUtils.isDataGenOpWithConstantValue)."""
    if h.op != "bi":
        return None
    if h.p.get("name") == "matrix":
        args = _bi_args(h)
        d = args.get("data")
        if d is not None and d.dt == "S" and d.op == "lit" and _num_lit(d):
            return d
    return None


def _one_by_one(h):
    """h is a 1 x 1 matrix by construction: matrix(x, rows=1, cols=1) or as.matrix(scalar).
    (Propagated hop dimensions are not trusted for rewrites that change the operator: a
    variable's size can differ between the iterations of a loop or the calls of a function.)"""
    if h.op == "u" and h.p.get("o") == "cast_matrix" and h.inputs and h.inputs[0].dt == "S":
        return True
    if h.op == "bi" and h.p.get("name") == "matrix" and h.inputs and h.inputs[0].dt == "S":
        args = _bi_args(h)
        return set(args) == {"data", "rows", "cols"} and _is_lit(args["rows"], 1) and _is_lit(args["cols"], 1)
    return False


def _is_diag(h):
    return h.op == "bi" and h.p.get("name") == "diag" and len(h.inputs) == 1 and not h.named


def _col_vector(h):
    """h is an n x 1 matrix by construction (diag(h) builds a diagonal matrix)."""
    return _vec_kind(h) == "col"


def _square_product(X, Y):
    """X %*% Y is square by construction: X %*% t(X) or t(Y) %*% Y."""
    return (Y.op == "t" and Y.inputs[0] is X) or (X.op == "t" and X.inputs[0] is Y)


def _fuse_rand(R, sc, o):
    """rand(rows, cols, min=a, max=b) op s as one rand with shifted / scaled bounds (uniform
    pdf, sparsity 1, literal bounds and a literal non-negative factor), else None."""
    if R.op != "bi" or R.p.get("name") != "rand" or not _num_lit(sc):
        return None
    npos = R.p.get("npos", len(R.inputs) - len(R.named))
    if npos:
        return None
    args = dict(zip(R.named, R.inputs[npos:]))
    if set(args) - {"rows", "cols", "min", "max", "seed", "pdf", "sparsity"}:
        return None
    pdf = args.get("pdf")
    if pdf is not None and not (pdf.op == "lit" and str(pdf.value).lower() == "uniform"):
        return None
    sp = args.get("sparsity")
    if sp is not None and not _is_lit(sp, 1):
        return None
    lo, hi = args.get("min", lit(0.0)), args.get("max", lit(1.0))
    if not (_num_lit(lo) and _num_lit(hi)):
        return None
    v = sc.value
    if o == "*":
        if v < 0:
            return None
        lo2, hi2 = lo.value * v, hi.value * v
    elif o == "+":
        lo2, hi2 = lo.value + v, hi.value + v
    else:
        lo2, hi2 = lo.value - v, hi.value - v
    args = dict(args)
    args["min"], args["max"] = lit(float(lo2)), lit(float(hi2))
    names = list(args)
    return Hop("bi", [args[k] for k in names], {"name": "rand", "npos": 0}, named=names, dt="M", dim1=R.dim1,
               dim2=R.dim2, pos=R.pos)


def _empty(h):
    """(rows, cols) hops of an all-zero datagen matrix(0, rows, cols) (nnz == 0 by
    construction), else None."""
    if h.op != "bi" or h.p.get("name") != "matrix" or not h.inputs or not _is_lit(h.inputs[0], 0):
        return None
    args = _bi_args(h)
    if set(args) - {"data", "rows", "cols"} or args.get("rows") is None or args.get("cols") is None:
        return None
    return args["rows"], args["cols"]


def _zeros(r, c, pos):
    return Hop("bi", [lit(0), r, c], {"name": "matrix", "npos": 1}, named=["rows", "cols"], dt="M", pos=pos)


def _nrow(x, pos):
    return Hop("u", [x], {"o": "nrow"}, dt="S", pos=pos)


def _ncol(x, pos):
    return Hop("u", [x], {"o": "ncol"}, dt="S", pos=pos)


def _same_dims(X, r, c):
    """The (rows, cols) hops r, c describe X's dimensions: nrow(X) / ncol(X), or literals equal
    to X's known dimensions."""
    def one(d, hop, which):
        if hop.op == "u" and hop.p.get("o") == which and hop.inputs[0] is X:
            return True
        return d >= 0 and _num_lit(hop) and hop.value == d
    return X.dt == "M" and one(X.dim1, r, "nrow") and one(X.dim2, c, "ncol")


_EMPTY_SAFE_UNARY = {"abs", "sqrt", "round", "floor", "ceil", "sign", "neg", "sin", "tan", "asin", "atan", "sinh",
                     "tanh"}


class Rewriter:
    def __init__(self, config=None):
        self.config = config
        self.memo = {}
        self.enabled = True if config is None else getattr(config, "rewrites", True)
        self.fuse = True if config is None else getattr(config, "fusion", True)
        self.stats = {}
        self.multi = set()       # ids of hops with more than one consumer (see count_consumers)

    def _count(self, name):
        self.stats[name] = self.stats.get(name, 0) + 1

    def rewrite(self, h: Hop) -> Hop:
        r = self.memo.get(h.id)
        if r is not None:
            return r
        new_inputs = [self.rewrite(c) for c in h.inputs]
        if any(a is not b for a, b in zip(new_inputs, h.inputs)):
            n = Hop(h.op, new_inputs, dict(h.p), list(h.named), h.dt, h.dim1, h.dim2, h.pos)
            # keep identity for non-pure hops (fcall/sink) so ordering references stay valid
            if h.op in ("fcall", "sink", "tread", "fout") or (h.op == "bi" and h.p.get("name") in H.NONDETERMINISTIC):
                h.inputs = new_inputs
                n = h
        else:
            n = h
        if h.id in self.multi:
            self.multi.add(n.id)
        if self.enabled:
            for _ in range(8):
                m = self.apply_rules(n)
                if m is n:
                    break
                n = m
        self.memo[h.id] = n
        return n

    # ------------------------------------------------------------------ rules
    def apply_rules(self, h: Hop) -> Hop:
        m = self._rw_empty(h)
        if m is not h:
            return m
        if h.op == "b" and len(h.inputs) == 2:
            # rules that check the consumers of the products they look through themselves
            o = h.p["o"]
            if o in ("+", "-"):
                m = self._rw_distributive(h)
                if m is not h:
                    return m
            if o == "*" and h.dt == "M":
                m = self._rw_emult_chain(h)
                if m is not h:
                    return m
        m = self._rw_algebraic(h)
        if m is not h:
            return m
        m = self._rw_more(h)
        if m is not h:
            return m
        m = self._rw_extra(h)
        if m is not h:
            return m
        op = h.op
        if op == "b":
            return self._rw_binary(h)
        if op == "u":
            x = h.inputs[0]
            if x.op == "lit" and x.value is not None and h.p["o"] not in ("nrow", "ncol", "length",
                                                                           "cast_matrix", "cast_frame",
                                                                           "cast_list") \
                    and h.p["o"] not in ("cumsum", "cumprod", "cummin", "cummax"):
                try:
                    return lit(S.unary(h.p["o"], x.value))
                except (DMLRuntimeError, TypeError, ValueError):
                    return h
            if h.p["o"] == "neg" and x.op == "u" and x.p["o"] == "neg":
                return x.inputs[0]
            return h
        if op == "t":
            x = h.inputs[0]
            if x.op == "t":
                self._count("t(t(X))")
                return x.inputs[0]
            return h
        if op == "agg":
            return self._rw_agg(h)
        if op == "mm":
            return self._rw_mm(h)
        if op == "bi" and h.p.get("name") in ("table", "ctable"):
            return self._match_onehot(h)
        if op == "bi" and h.p.get("name") in ("cbind", "append"):
            return self._match_cbind_const(h)
        return h

    # ------------------------------------------------------------------ algebraic simplification
    # (reference: hops/rewrite/RewriteAlgebraicSimplificationStatic.java and the size-guarded
    # rules of RewriteAlgebraicSimplificationDynamic.java; each rule names its method there)
    def _hit(self, name, h):
        self._count(name)
        return h

    def _rw_algebraic(self, h):
        op = h.op
        # rules that look through an intermediate apply only when this hop is its sole
        # consumer (the reference's parent-count checks): otherwise the intermediate is
        # computed anyway and the rewrite would duplicate work
        if any(c.id in self.multi for c in h.inputs if c.op not in ("lit", "tread")):
            return h
        if op == "agg":
            x = h.inputs[0]
            o, d = h.p["o"], h.p["dir"]
            # removeUnnecessaryAggregates: sum(rowSums(X)) / sum(colSums(X)) -> sum(X), same for min / max
            if d == "all" and x.op == "agg" and x.p["dir"] in ("row", "col") and x.p["o"] == o \
                    and o in ("sum", "min", "max"):
                return self._hit("unnecessary-aggregate",
                                 Hop("agg", [x.inputs[0]], {"o": o, "dir": "all"}, dt="S", dim1=0, dim2=0, pos=h.pos))
            # full aggregates are transpose-invariant (simplifyUnaryAggReorgOperation)
            if d == "all" and x.op == "t" and o in ("sumsq", "min", "max", "mean", "prod"):
                return self._hit("agg-transpose", Hop("agg", [x.inputs[0]], dict(h.p), dt="S", dim1=0, dim2=0,
                                                      pos=h.pos))
            # pushdownUnaryAggTransposeOperation: colSums(t(X)) -> t(rowSums(X)) (and row <-> col)
            if d in ("row", "col") and x.op == "t" and o in ("sum", "mean", "min", "max", "sumsq", "prod"):
                inner = Hop("agg", [x.inputs[0]], {"o": o, "dir": "col" if d == "row" else "row"}, dt="M",
                            pos=h.pos)
                return self._hit("agg-transpose-pushdown", Hop("t", [inner], dt="M", pos=h.pos))
            # pushdownSumBinaryMult: sum(s * X) -> s * sum(X), sum(X / s) -> sum(X) / s
            if d == "all" and o == "sum" and x.op == "b" and x.p["o"] in ("*", "/"):
                a, b = x.inputs
                if x.p["o"] == "*" and a.dt == "S" and b.dt == "M":
                    a, b = b, a
                if a.dt == "M" and b.dt == "S":
                    inner = Hop("agg", [a], {"o": "sum", "dir": "all"}, dt="S", dim1=0, dim2=0, pos=h.pos)
                    return self._hit("sum-scalar-pushdown", Hop("b", [inner, b], {"o": x.p["o"]}, dt="S", pos=h.pos))
            # sum(-X) -> -sum(X)
            if d == "all" and o == "sum" and x.op == "u" and x.p["o"] == "neg" and x.dt == "M":
                inner = Hop("agg", [x.inputs[0]], {"o": "sum", "dir": "all"}, dt="S", dim1=0, dim2=0, pos=h.pos)
                return self._hit("sum-neg-pushdown", Hop("u", [inner], {"o": "neg"}, dt="S", pos=h.pos))
            # simplifyTraceMatrixMult: trace(X %*% Y) -> sum(X * t(Y))
            if d == "all" and o == "trace" and x.op == "mm" and not x.p.get("transA"):
                A, B = x.inputs
                prod = Hop("b", [A, Hop("t", [B], dt="M", pos=h.pos)], {"o": "*"}, dt="M", pos=h.pos)
                return self._hit("trace-mm", Hop("agg", [prod], {"o": "sum", "dir": "all"}, dt="S", dim1=0, dim2=0,
                                                 pos=h.pos))
            # simplifySumDiagToTrace: sum(diag(X)) -> trace(X) (X square: diag returns its diagonal)
            if d == "all" and o == "sum" and x.op == "bi" and x.p.get("name") == "diag" and len(x.inputs) == 1:
                X = x.inputs[0]
                if X.op == "tsmm":      # square by construction (hop dims are not trusted)
                    return self._hit("sum-diag-trace", Hop("agg", [X], {"o": "trace", "dir": "all"}, dt="S", dim1=0,
                                                           dim2=0, pos=h.pos))
            # simplifyColSumsMVMult / simplifyRowSumsMVMult for operands that are vectors by
            # construction (aggregate outputs, transposes of them, 1-column datagens: dims of
            # hops inside re-used function bodies are not trusted):
            # colSums(X * y) -> t(y) %*% X (y: column vector), rowSums(X * v) -> X %*% t(v) (v: row vector)
            if d in ("row", "col") and o == "sum" and x.op == "b" and x.p["o"] == "*" and x.dt == "M":
                for X, v in ((x.inputs[0], x.inputs[1]), (x.inputs[1], x.inputs[0])):
                    if X.dt != "M" or v.dt != "M":
                        continue
                    # (a 1x1 "vector" broadcasts as a scalar: the product keeps the original
                    # aggregate as its run-time fallback, p["mvagg"])
                    if d == "col" and _vec_kind(v) == "col" and _vec_kind(X) is None:
                        return self._hit("colsums-mv", Hop("mm", [v, X], {"transA": True, "mvagg": "col"}, dt="M",
                                                           pos=h.pos))
                    if d == "row" and _vec_kind(v) == "row" and _vec_kind(X) is None:
                        return self._hit("rowsums-mv", Hop("mm", [X, Hop("t", [v], dt="M", pos=h.pos)],
                                                           {"mvagg": "row"}, dt="M", pos=h.pos))
            return h
        if op == "u":
            x = h.inputs[0]
            o = h.p["o"]
            # idempotent unary operators: abs(abs(X)) -> abs(X) (round/floor/ceil/sign likewise)
            if o in ("abs", "round", "floor", "ceil", "sign") and x.op == "u" and x.p["o"] == o:
                return self._hit("idempotent-unary", x)
            # simplifyNotOverComparisons: !(A == B) -> A != B, !(A < B) -> A >= B, ...
            if o == "not" and x.op == "b" and x.p["o"] in _NOT_CMP:
                return self._hit("not-over-comparison", Hop("b", list(x.inputs), {"o": _NOT_CMP[x.p["o"]]},
                                                            dt=x.dt, pos=h.pos))
            return h
        if op == "b":
            a, b = h.inputs
            o = h.p["o"]
            # A + (-B) -> A - B, A - (-B) -> A + B, (-A) + B -> B - A, (-A) * (-B) -> A * B
            if o in ("+", "-") and b.op == "u" and b.p["o"] == "neg" and (a.dt == "M" or b.dt == "M"):
                return self._hit("binary-negation", Hop("b", [a, b.inputs[0]], {"o": "-" if o == "+" else "+"},
                                                        dt=h.dt, pos=h.pos))
            if o == "+" and a.op == "u" and a.p["o"] == "neg" and (a.dt == "M" or b.dt == "M"):
                return self._hit("binary-negation", Hop("b", [b, a.inputs[0]], {"o": "-"}, dt=h.dt, pos=h.pos))
            if o in ("*", "/") and a.op == "u" and a.p["o"] == "neg" and b.op == "u" and b.p["o"] == "neg":
                return self._hit("binary-negation", Hop("b", [a.inputs[0], b.inputs[0]], {"o": o}, dt=h.dt, pos=h.pos))
            # fuseBinarySubDAGToUnaryOperation: 1 / (1 + exp(-X)) -> sigmoid(X)
            if o == "/" and _is_lit(a, 1) and b.op == "b" and b.p["o"] == "+" and b.dt == "M":
                l, r = b.inputs
                e = r if _is_lit(l, 1) else (l if _is_lit(r, 1) else None)
                if e is not None and e.op == "u" and e.p["o"] == "exp" and e.inputs[0].op == "u" \
                        and e.inputs[0].p["o"] == "neg":
                    return self._hit("sigmoid", Hop("u", [e.inputs[0].inputs[0]], {"o": "sigmoid"}, dt="M", pos=h.pos))
            # simplifyMultiBinaryToBinaryOperation: X * X -> X ^ 2 (one operand read)
            if o == "*" and a is b and a.dt == "M":
                return self._hit("square", Hop("b", [a, lit(2)], {"o": "^"}, dt="M", pos=h.pos))
            # pushdownBinaryOperationOnDiag (Dynamic.java:1068): diag(v) * s -> diag(v * s) for a
            # column vector v and a scalar s (n cells scaled instead of n x n)
            if o == "*":
                for d_, s_ in ((a, b), (b, a)):
                    if _is_diag(d_) and s_.dt == "S" and _col_vector(d_.inputs[0]):
                        v = d_.inputs[0]
                        vs = Hop("b", [v, s_], {"o": "*"}, dt="M", dim1=v.dim1, dim2=1, pos=h.pos)
                        return self._hit("diag-binary-pushdown", Hop("bi", [vs], dict(d_.p), dt="M", dim1=d_.dim1,
                                                                     dim2=d_.dim2, pos=h.pos))
            # literal chains: (X + c1) + c2 -> X + (c1 + c2), (X * c1) * c2 -> X * (c1 * c2)
            if o in ("+", "*") and _num_lit(b) and a.op == "b" and a.p["o"] == o and a.dt == "M" \
                    and _num_lit(a.inputs[1]):
                c = S.binary(o, a.inputs[1].value, b.value)
                return self._hit("literal-chain", Hop("b", [a.inputs[0], lit(c)], {"o": o}, dt="M", pos=h.pos))
            return h
        if op == "t":
            x = h.inputs[0]
            # t(t(A) %*% t(B))... and t(X) %*% t(Y) handled in _rw_mm; t(s * X) keeps scalars outside
            return h
        if op == "mm" and not h.p.get("transA"):
            a, b = h.inputs
            # simplifyTransposeMatrixMult-style: t(X) %*% t(Y) -> t(Y %*% X) (one transpose)
            if a.op == "t" and b.op == "t" and a.inputs[0] is not b.inputs[0]:
                inner = Hop("mm", [b.inputs[0], a.inputs[0]], {}, dt="M", pos=h.pos)
                return self._hit("transpose-mm", Hop("t", [inner], dt="M", pos=h.pos))
            return h
        if op == "bi":
            name = h.p.get("name")
            # simplifyDiagMatrixMult (Dynamic.java:1012): diag(X %*% Y) -> rowSums(X * t(Y)) when
            # X %*% Y is square (its diagonal without the n x n product)
            if name == "diag" and len(h.inputs) == 1 and h.inputs[0].op == "tsmm":
                # the same for an already fused tsmm: diag(X %*% t(X)) = rowSums(X ^ 2),
                # diag(t(X) %*% X) = t(colSums(X ^ 2))
                X = h.inputs[0].inputs[0]
                left = h.inputs[0].p.get("left", True)
                sq = Hop("agg", [X], {"o": "sumsq", "dir": "col" if left else "row"}, dt="M", pos=h.pos)
                return self._hit("diag-matrix-mult", Hop("t", [sq], dt="M", pos=h.pos) if left else sq)
            if name == "diag" and len(h.inputs) == 1 and h.inputs[0].op == "mm" and not h.inputs[0].p.get("transA"):
                X, Y = h.inputs[0].inputs
                if _square_product(X, Y):
                    prod = Hop("b", [X, Hop("t", [Y], dt="M", pos=h.pos)], {"o": "*"}, dt="M", pos=h.pos)
                    return self._hit("diag-matrix-mult", Hop("agg", [prod], {"o": "sum", "dir": "row"}, dt="M",
                                                             pos=h.pos))
            # removeUnnecessaryReorgOperation: rev(rev(X)) -> X
            if name == "rev" and len(h.inputs) == 1 and h.inputs[0].op == "bi" \
                    and h.inputs[0].p.get("name") == "rev" and len(h.inputs[0].inputs) == 1:
                return self._hit("rev-rev", h.inputs[0].inputs[0])
            # removeUnnecessaryReshape: matrix(X, rows=nrow(X), cols=ncol(X)) -> X
            if name == "matrix" and h.inputs and h.inputs[0].dt == "M":
                args = _bi_args(h)
                X, r, c = args.get("data"), args.get("rows"), args.get("cols")
                if set(args) <= {"data", "rows", "cols"} and r is not None and c is not None \
                        and r.op == "u" and r.p["o"] == "nrow" and r.inputs[0] is X \
                        and c.op == "u" and c.p["o"] == "ncol" and c.inputs[0] is X:
                    return self._hit("unnecessary-reshape", X)
            return h
        if op == "rix":
            # removeUnnecessaryRightIndexing: X[1:nrow(X), 1:ncol(X)] -> X
            src, rl, ru, cl, cu = h.inputs
            if src.dt == "M" and not h.p.get("list") and _full_range(src, rl, ru, "nrow") and _full_range(src, cl, cu, "ncol"):
                return self._hit("unnecessary-indexing", src)
            return h
        if op == "lix" and not h.p.get("list") and not h.p.get("inplace"):
            return self._rw_lix_chain(h)
        return h

    # ------------------------------------------------------------------ round-5 rules
    def _rw_more(self, h):
        """Further rules of RewriteAlgebraicSimplification{Static,Dynamic}.java (line numbers
        in each comment).  Rules that look through an intermediate require this hop to be its
        sole consumer, as the reference's parent-count checks do."""
        op = h.op
        sole = not any(c.id in self.multi for c in h.inputs if c.op not in ("lit", "tread"))
        if op == "agg" and len(h.inputs) == 1:
            x = h.inputs[0]
            o, d = h.p["o"], h.p["dir"]
            # simplifyNnzComputation (Dynamic:2469): sum(X != 0) -> nnz(X) (no boolean matrix)
            if d == "all" and o == "sum" and sole and x.op == "b" and x.p["o"] == "!=" and x.dt == "M":
                a, b = x.inputs
                X = a if _is_lit(b, 0) else (b if _is_lit(a, 0) else None)
                if X is not None and X.dt == "M":
                    return self._hit("nnz", Hop("bi", [X], {"name": "_nnz", "npos": 1}, dt="S", dim1=0, dim2=0,
                                                pos=h.pos))
            # simplifyColwiseAggregate (Dynamic:525) / simplifyRowwiseAggregate (:581):
            # colSums(X) of a row vector is X; of a column vector it is sum(X) (1 x 1);
            # rowSums likewise with rows and columns swapped
            if d in ("row", "col") and o in ("sum", "mean", "min", "max"):
                kind = _vec_kind(x)
                if (d == "col" and kind == "row") or (d == "row" and kind == "col"):
                    return self._hit("colwise-aggregate", x)
                if (d == "col" and kind == "col") or (d == "row" and kind == "row"):
                    full = Hop("agg", [x], {"o": o, "dir": "all"}, dt="S", dim1=0, dim2=0, pos=h.pos)
                    return self._hit("colwise-aggregate", Hop("u", [full], {"o": "cast_matrix"}, dt="M", dim1=1,
                                                              dim2=1, pos=h.pos))
            return h
        if op == "b" and h.p["o"] in ("+", "-") and h.dt == "M" and not self.fuse:
            # fuseAxpyBinaryOperationChain (Dynamic:2173): X + s * Y -> +*(X, s, Y), X - s * Y ->
            # -*(X, s, Y) with s a scalar.  With operator fusion on, the Cell template fuses the
            # chain (and its CP fallback runs it as one axpy, ops/cell.py), so this is for
            # fusion-off plans.
            a, b = h.inputs

            def split(m):
                if m.op != "b" or m.p["o"] != "*" or m.dt != "M" or m.id in self.multi:
                    return None
                p, q = m.inputs
                if p.dt == "S" and q.dt == "M":
                    return p, q
                if q.dt == "S" and p.dt == "M":
                    return q, p
                return None
            sgn = 1 if h.p["o"] == "+" else -1
            for X, m in ((a, b), (b, a)) if sgn > 0 else ((a, b),):
                sy = split(m) if X.dt == "M" else None
                if sy is not None:
                    return self._hit("fuse-axpy", Hop("bi", [X, sy[0], sy[1], H.lit(float(sgn), h.pos)],
                                                      {"name": "_axpy", "npos": 4}, dt="M", dim1=h.dim1,
                                                      dim2=h.dim2, pos=h.pos))
            return h
        if op == "u" and h.p["o"] in ("cumsum", "cumprod", "cummin", "cummax"):
            # removeUnnecessaryCumulativeOp (Dynamic:346): a cumulative aggregate of one row is the row
            x = h.inputs[0]
            if _vec_kind(x) == "row":
                return self._hit("unnecessary-cumulative", x)
            return h
        if op == "t":
            x = h.inputs[0]
            # fuseDatagenAndReorgOperation (Dynamic:487): t(matrix(s, rows=r, cols=c)) -> matrix(s, c, r)
            if x.op == "bi" and x.p.get("name") == "matrix" and x.inputs and x.inputs[0].dt == "S" and sole:
                args = _bi_args(x)
                if set(args) == {"data", "rows", "cols"}:
                    return self._hit("datagen-reorg", Hop("bi", [args["data"], args["cols"], args["rows"]],
                                                          {"name": "matrix", "npos": 1}, named=["rows", "cols"],
                                                          dt="M", dim1=x.dim2, dim2=x.dim1, pos=h.pos))
            # simplifyTransposedAppend (Static:1117): t(cbind(t(A), t(B))) -> rbind(A, B) (and rbind -> cbind)
            if x.op == "bi" and x.p.get("name") in ("cbind", "append", "rbind") and sole and not x.named \
                    and len(x.inputs) >= 2 and all(c.op == "t" for c in x.inputs) \
                    and x.id not in self.multi:
                name = "rbind" if x.p["name"] in ("cbind", "append") else "cbind"
                return self._hit("transposed-append", Hop("bi", [c.inputs[0] for c in x.inputs],
                                                          {"name": name, "npos": len(x.inputs)}, dt="M", pos=h.pos))
            return h
        if op == "bi":
            name = h.p.get("name")
            # foldMultipleAppendOperations (Static:523): cbind(cbind(A, B), C) -> cbind(A, B, C)
            if name in ("cbind", "rbind") and not h.named and h.inputs and all(c.dt == "M" for c in h.inputs):
                flat, changed = [], False
                for c in h.inputs:
                    if c.op == "bi" and c.p.get("name") == name and not c.named and c.id not in self.multi \
                            and all(g.dt == "M" for g in c.inputs):
                        flat.extend(c.inputs)
                        changed = True
                    else:
                        flat.append(c)
                if changed:
                    return self._hit("fold-append", Hop("bi", flat, {"name": name, "npos": len(flat)}, dt="M",
                                                        pos=h.pos))
            if name == "order":
                return self._rw_order(h)
            if name == "rand" and sole:
                return h
            return h
        if op == "b" and len(h.inputs) == 2 and h.dt == "M":
            a, b = h.inputs
            o = h.p["o"]
            # fuseMinusNzBinaryOperation (Static:1670): X - s * (X != 0) -> X -nz s (sparse-safe)
            if o == "-" and b.op == "b" and b.p["o"] == "*" and b.id not in self.multi and a.dt == "M":
                for sc, nz in ((b.inputs[0], b.inputs[1]), (b.inputs[1], b.inputs[0])):
                    if sc.dt == "S" and nz.op == "b" and nz.p["o"] == "!=" and nz.id not in self.multi \
                            and ((nz.inputs[0] is a and _is_lit(nz.inputs[1], 0)) or
                                 (nz.inputs[1] is a and _is_lit(nz.inputs[0], 0))):
                        return self._hit("minus-nz", Hop("bi", [a, sc], {"name": "_minus_nz", "npos": 2}, dt="M",
                                                         dim1=a.dim1, dim2=a.dim2, pos=h.pos))
            # fuseLogNzBinaryOperation (Static:1734): (X != 0) * log(X) -> log_nz(X) (sparse-safe)
            if o == "*":
                for nz, lg in ((a, b), (b, a)):
                    if nz.op == "b" and nz.p["o"] == "!=" and lg.op in ("u", "b") and lg.p.get("o") == "log" \
                            and nz.id not in self.multi and lg.id not in self.multi:
                        X = lg.inputs[0]
                        if (nz.inputs[0] is X and _is_lit(nz.inputs[1], 0)) or \
                                (nz.inputs[1] is X and _is_lit(nz.inputs[0], 0)):
                            args = [X] + (list(lg.inputs[1:]) if lg.op == "b" else [])
                            return self._hit("log-nz", Hop("bi", args, {"name": "_log_nz", "npos": len(args)},
                                                           dt="M", dim1=X.dim1, dim2=X.dim2, pos=h.pos))
            # fuseDatagenAndBinaryOperation (Static:347): rand(min=a, max=b) * s -> rand(min=a*s,
            # max=b*s) for s >= 0, rand(...) + s -> rand(min=a+s, max=b+s) (uniform, dense)
            if o in ("*", "+", "-") and sole:
                for R, sc, left in ((a, b, True), (b, a, False)):
                    if o == "-" and not left:
                        continue
                    g = _fuse_rand(R, sc, o)
                    if g is not None and R.id not in self.multi:
                        return self._hit("datagen-binary", g)
            # simplifyBushyBinaryOperation (Static:838): X * (Y * (Z %*% v)) -> (X * Y) * (Z %*% v)
            # for equal-sized X, Y (the cellwise product of the two matrices first; the mv
            # product broadcasts once)
            # (cellwise * with matrix-vector broadcasting is associative for every valid
            # operand shape combination, so no size checks are needed)
            if o == "*" and b.op == "b" and b.p["o"] == "*" and b.id not in self.multi and a.dt == "M" \
                    and a.op != "mm":
                Y, mv = b.inputs
                if mv.op != "mm":
                    Y, mv = mv, Y
                if mv.op == "mm" and _vec_kind(mv.inputs[1]) == "col" and Y.dt == "M" and Y.op != "mm":
                    xy = Hop("b", [a, Y], {"o": "*"}, dt="M", pos=h.pos)
                    return self._hit("bushy-binary", Hop("b", [xy, mv], {"o": "*"}, dt="M", pos=h.pos))
            return h
        if op == "rix" and not h.p.get("list"):
            # simplifySlicedMatrixMult (Static:1343): (X %*% Y)[i, j] -> X[i, ] %*% Y[, j]
            src, rl, ru, cl, cu = h.inputs

            def single(lo, hi):
                if lo.op == "lit" and lo.value is None:
                    return False
                return lo is hi or (_num_lit(lo) and _num_lit(hi) and lo.value == hi.value)
            if src.op == "mm" and not src.p.get("transA") and src.id not in self.multi and single(rl, ru) \
                    and single(cl, cu):
                X, Y = src.inputs
                none = lit(None)
                xr = Hop("rix", [X, rl, ru, none, none], {}, dt="M", dim1=1, dim2=X.dim2, pos=h.pos)
                yc = Hop("rix", [Y, none, none, cl, cu], {}, dt="M", dim1=Y.dim1, dim2=1, pos=h.pos)
                return self._hit("sliced-matrix-mult", Hop("mm", [xr, yc], {}, dt="M", dim1=1, dim2=1, pos=h.pos))
            return h
        return h

    def _rw_extra(self, h):
        """The remaining algebraic rules of RewriteAlgebraicSimplification{Static,Dynamic}.java
        (line numbers in each comment)."""
        op = h.op
        sole = not any(c.id in self.multi for c in h.inputs if c.op not in ("lit", "tread"))
        if op == "agg" and len(h.inputs) == 1 and h.p["o"] == "sum" and h.p["dir"] == "all":
            x = h.inputs[0]
            # pushdownSumOnAdditiveBinary (Dynamic:1151): sum(A+B) -> sum(A)+sum(B), sum(A-B) ->
            # sum(A)-sum(B) for equal-size matrices (lets sum(X^2) / tak+* rules see each term)
            if sole and x.op == "b" and x.p["o"] in ("+", "-") and x.dt == "M":
                A, B = x.inputs
                if A.dt == "M" and B.dt == "M" and _equal_size(A, B):
                    s1 = Hop("agg", [A], {"o": "sum", "dir": "all"}, dt="S", dim1=0, dim2=0, pos=h.pos)
                    s2 = Hop("agg", [B], {"o": "sum", "dir": "all"}, dt="S", dim1=0, dim2=0, pos=h.pos)
                    return self._hit("pushdown-sum-additive",
                                     Hop("b", [s1, s2], {"o": x.p["o"]}, dt="S", dim1=0, dim2=0, pos=h.pos))
        if op == "mm" and not h.p.get("transA") and len(h.inputs) == 2:
            a, b = h.inputs
            # reorderMinusMatrixMult (Dynamic:2313): (0-A) %*% B -> 0-(A %*% B) (and the right
            # form) when the product is smaller than A -- the negation runs on the product
            for i, m in enumerate((a, b)):
                if m.op == "b" and m.p.get("o") == "-" and _is_lit(m.inputs[0], 0) and m.inputs[1].dt == "M" \
                        and sole and _smaller(h, m.inputs[1]):
                    ins = [a, b]
                    ins[i] = m.inputs[1]
                    prod = Hop("mm", ins, dict(h.p), dt="M", dim1=h.dim1, dim2=h.dim2, pos=h.pos)
                    return self._hit("reorder-minus-mm", Hop("b", [lit(0), prod], {"o": "-"}, dt="M", dim1=h.dim1,
                                                            dim2=h.dim2, pos=h.pos))
            # simplifyReverseOperation (Static:700): table(seq(1,n), seq(n,1,-1)) %*% X -> rev(X)
            if a.op == "bi" and a.p.get("name") in ("table", "ctable") and not a.named and len(a.inputs) == 2:
                n1 = _basic_1n_seq(a.inputs[0])
                n2 = _basic_n1_seq(a.inputs[1])
                if n1 is not None and n2 is not None and _same_hop_value(n1, n2):
                    return self._hit("reverse-operation", Hop("bi", [b], {"name": "rev", "npos": 1}, dt="M",
                                                             dim1=b.dim1, dim2=b.dim2, pos=h.pos))
            # (the same table after the seq-ctable rewrite: the one-hot of seq(n, 1, -1), n x n)
            if a.op == "bi" and a.p.get("name") == "_onehot" and _is_lit(a.inputs[1], -1) \
                    and _is_lit(a.inputs[2], -1) and _basic_n1_seq(a.inputs[0]) is not None:
                return self._hit("reverse-operation", Hop("bi", [b], {"name": "rev", "npos": 1}, dt="M",
                                                         dim1=b.dim1, dim2=b.dim2, pos=h.pos))
        if op == "b" and len(h.inputs) == 2 and h.dt == "M":
            l, r = h.inputs
            o = h.p["o"]
            # canonicalizeMatrixMultScalarAdd (Static:640): eps + U%*%V -> U%*%V + eps and
            # U%*%V - eps -> U%*%V + (-eps) (one form for the wdivmm / wcemm epsilon matchers)
            if o == "+" and l.dt == "S" and r.op in ("mm", "tsmm"):
                return self._hit("canonical-mm-scalar-add", Hop("b", [r, l], {"o": "+"}, dt="M", dim1=h.dim1,
                                                               dim2=h.dim2, pos=h.pos))
            if o == "-" and r.dt == "S" and l.op in ("mm", "tsmm"):
                neg = lit(-r.value) if _num_lit(r) else Hop("u", [r], {"o": "neg"}, dt="S", dim1=0, dim2=0, pos=h.pos)
                return self._hit("canonical-mm-scalar-add", Hop("b", [l, neg], {"o": "+"}, dt="M", dim1=h.dim1,
                                                               dim2=h.dim2, pos=h.pos))
        if op == "bi":
            name = h.p.get("name")
            # removeUnnecessaryIfElseOperation (Dynamic:444)
            if name == "ifelse" and len(h.inputs) == 3 and not h.named:
                e, A, B = h.inputs
                if e.op == "lit" and isinstance(e.value, (bool, int, float)) and A.dt == B.dt:
                    pick = A if bool(e.value) else B
                    if A.dt == "S" or (A.dt == "M" and _equal_size(A, B)):
                        return self._hit("ifelse-removal", pick)
                if A is B and e.dt == "S" and A.dt == "M":
                    return self._hit("ifelse-removal", A)
            # simplifyCTableWithConstMatrixInputs (Static:672): table(X, matrix(1,..), matrix(7,..))
            # -> table(X, 1, 7) (no constant vectors materialised)
            if name in ("table", "ctable") and not h.named and len(h.inputs) in (2, 3, 4, 5):
                ins = list(h.inputs)
                changed = False
                for i in range(1, min(3, len(ins))):
                    c = _const_datagen_value(ins[i])
                    if c is not None:
                        ins[i] = c
                        changed = True
                if changed and ins[0].dt == "M":
                    return self._hit("ctable-const-inputs", Hop("bi", ins, dict(h.p), [], dt="M", pos=h.pos))
                # simplifyTableSeqExpand pattern b (Dynamic:2531): table(v, seq(1,nrow(v)), m, nrow(v))
                # -> t(one-hot of v) (pattern a is the seq-ctable rewrite)
                if len(ins) == 4 and h.inputs[0].dt == "M":
                    n = _basic_1n_seq(h.inputs[1])
                    if n is not None and _same_hop_value(n, h.inputs[3]):
                        oh = Hop("bi", [h.inputs[0], lit(-1), h.inputs[2]], {"name": "_onehot", "npos": 3}, dt="M",
                                 pos=h.pos)
                        return self._hit("table-seq-expand", Hop("t", [oh], {}, dt="M", pos=h.pos))
            # simplifyGroupedAggregate (Static:1641): aggregate(target=v, groups=g, fn="count")
            # counts group members: target := groups (v is never read)
            if name == "aggregate" and h.named:
                args = dict(zip(h.named, h.inputs[len(h.inputs) - len(h.named):]))
                fn = args.get("fn")
                tgt, grp = args.get("target"), args.get("groups")
                if fn is not None and fn.op == "lit" and fn.value == "count" and tgt is not None \
                        and grp is not None and tgt is not grp and (_vec_kind(tgt) == "col" or tgt.dim2 == 1):
                    ins = list(h.inputs)
                    ins[len(h.inputs) - len(h.named) + h.named.index("target")] = args["groups"]
                    return self._hit("grouped-aggregate-count", Hop("bi", ins, dict(h.p), list(h.named), dt="M",
                                                                   pos=h.pos))
            # simplifyOuterSeqExpand (Static:1766): outer(v, t(seq(1,m)), "==") -> the exact-match
            # expansion of v into m indicator columns (no outer operator over a sequence)
            if name == "outer" and len(h.inputs) == 3 and h.inputs[2].op == "lit" and h.inputs[2].value == "==":
                v, w = h.inputs[0], h.inputs[1]
                if w.op == "t":
                    m = _basic_1n_seq(w.inputs[0])
                    if m is not None and v.dt == "M":
                        return self._hit("outer-seq-expand", Hop("bi", [v, m], {"name": "_seq_expand", "npos": 2},
                                                                dt="M", pos=h.pos))
        return h

    def _rw_order(self, h):
        """simplifyConstantSort (Static:1383): order of a constant matrix is the matrix (its
        index is 1..n); simplifyOrderedSort (Static:1421): order of an ascending seq is the seq
        (decreasing: rev(seq); index.return: 1..n or n..1)."""
        npos = h.p.get("npos", len(h.inputs) - len(h.named))
        args = {n: h.inputs[npos + j] for j, n in enumerate(h.named)}
        pos_names = ["target", "by", "decreasing", "index.return"]
        for i in range(npos):
            args[pos_names[i]] = h.inputs[i]
        X = args.get("target")
        if X is None or set(args) - set(pos_names):
            return h
        dec = args.get("decreasing")
        ixr = args.get("index.return")
        if (dec is not None and not (dec.op == "lit" and isinstance(dec.value, bool))) or \
                (ixr is not None and not (ixr.op == "lit" and isinstance(ixr.value, bool))):
            return h
        dec = bool(dec.value) if dec is not None else False
        ixr = bool(ixr.value) if ixr is not None else False
        n = _nrow(X, h.pos)

        def seq(a, b, step):
            return Hop("bi", [a, b, lit(step)], {"name": "seq", "npos": 3}, dt="M", pos=h.pos)
        if X.op == "bi" and X.p.get("name") == "matrix" and X.inputs and _num_lit(X.inputs[0]) \
                and set(_bi_args(X)) == {"data", "rows", "cols"}:
            # stable sort of equal keys: the identity permutation
            return self._hit("constant-sort", seq(lit(1), n, 1) if ixr else X)
        if X.op == "bi" and X.p.get("name") == "seq" and not X.named and X.p.get("npos", 0) in (2, 3):
            sa = X.inputs
            step = sa[2] if len(sa) == 3 else lit(1)
            if not (_num_lit(step) and step.value > 0 and _num_lit(sa[0]) and _num_lit(sa[1])
                    and sa[0].value <= sa[1].value) or (args.get("by") is not None and not _is_lit(args["by"], 1)):
                return h
            if ixr:
                return self._hit("ordered-sort", seq(n, lit(1), -1) if dec else seq(lit(1), n, 1))
            return self._hit("ordered-sort", Hop("bi", [X], {"name": "rev", "npos": 1}, dt="M", pos=h.pos) if dec
                             else X)
        # fuseOrderOperationChain (Dynamic:2245): order(order(X, by=b1), by=b2) with equal
        # `decreasing` and data results -> order(X, by=[b2, b1]): the outer stable sort keeps the
        # inner order among its ties, i.e. one lexicographic sort on (b2, b1)
        if not ixr and X.op == "bi" and X.p.get("name") == "order" and X.id not in self.multi:
            inner = self._order_args(X)
            by2 = args.get("by", lit(1))
            if inner is not None and not inner[3] and inner[2] == dec and _num_lit(by2):
                X0, by1 = inner[0], inner[1]
                keys = [int(by2.value)] + by1
                data = lit(" ".join(str(k) for k in keys))
                bym = Hop("bi", [data, lit(len(keys)), lit(1)], {"name": "matrix", "npos": 1},
                          ["rows", "cols"], dt="M", dim1=len(keys), dim2=1, pos=h.pos)
                return self._hit("order-chain", Hop("bi", [X0, bym, lit(dec)], {"name": "order", "npos": 1},
                                                    ["by", "decreasing"], dt="M", dim1=X0.dim1, dim2=X0.dim2,
                                                    pos=h.pos))
        return h

    def _order_args(self, h):
        """(target, [by columns], decreasing, index.return) of an order hop with literal
        arguments (by: an int or a literal column-index matrix), else None."""
        npos = h.p.get("npos", len(h.inputs) - len(h.named))
        names = ["target", "by", "decreasing", "index.return"]
        args = {n: h.inputs[npos + j] for j, n in enumerate(h.named)}
        for i in range(npos):
            args[names[i]] = h.inputs[i]
        if "target" not in args or set(args) - set(names):
            return None
        by = args.get("by", lit(1))
        if _num_lit(by):
            cols = [int(by.value)]
        elif by.op == "bi" and by.p.get("name") == "matrix" and by.inputs and by.inputs[0].op == "lit" \
                and isinstance(by.inputs[0].value, str):
            try:
                cols = [int(float(t)) for t in by.inputs[0].value.replace(",", " ").split()]
            except ValueError:
                return None
        else:
            return None
        flags = []
        for k in ("decreasing", "index.return"):
            v = args.get(k)
            if v is not None and not (v.op == "lit" and isinstance(v.value, bool)):
                return None
            flags.append(bool(v.value) if v is not None else False)
        return args["target"], cols, flags[0], flags[1]

    def _rw_lix_chain(self, h):
        """fuseLeftIndexingChainToAppend (reference RewriteAlgebraicSimplificationDynamic.java:285):
        X[,1] = A; X[,2] = B -> X = cbind(A, B) for a two-column X (rows likewise -> rbind)."""
        inner = h.inputs[0]
        if inner.op != "lix" or inner.p.get("list") or inner.p.get("inplace") or inner.id in self.multi:
            return h
        X = inner.inputs[0]

        def empty(x):
            return x.op == "lit" and x.value is None

        for full, sel, dim, name in (((2, 3), (4, 5), 1, "cbind"), ((4, 5), (2, 3), 0, "rbind")):
            if not all(empty(z.inputs[i]) for z in (h, inner) for i in full):
                continue
            if not (_is_lit(inner.inputs[sel[0]], 1) and _is_lit(inner.inputs[sel[1]], 1)
                    and _is_lit(h.inputs[sel[0]], 2) and _is_lit(h.inputs[sel[1]], 2)):
                continue
            ncl = X.dim2 if dim == 1 else X.dim1
            e = _empty(X) if X.op == "bi" else None
            if e is not None and _num_lit(e[dim]):
                ncl = e[dim].value
            A, B = inner.inputs[1], h.inputs[1]
            if ncl == 2 and A.dt == "M" and B.dt == "M":
                return self._hit("lix-chain-append", Hop("bi", [A, B], {"name": name, "npos": 2}, dt="M", pos=h.pos))
        return h

    # ------------------------------------------------------------------ empty operands
    # (reference RewriteAlgebraicSimplificationDynamic: simplifyEmptyAggregate :747,
    # simplifyEmptyUnaryOperation :776, simplifyEmptyReorgOperation :800, simplifyEmptyMatrixMult
    # :879, simplifyEmptyBinaryOperation; "empty" = an all-zero datagen, known without sizes)
    def _rw_empty(self, h):
        op = h.op
        if op == "agg" and len(h.inputs) == 1:
            e = _empty(h.inputs[0])
            if e is None or h.p["o"] not in ("sum", "sumsq", "mean", "min", "max", "prod"):
                return h
            d = h.p["dir"]
            if d == "all":
                return self._hit("empty-aggregate", lit(0.0))
            r, c = e
            return self._hit("empty-aggregate", _zeros(r, lit(1), h.pos) if d == "row" else _zeros(lit(1), c, h.pos))
        if op == "u" and h.dt == "M" and h.p.get("o") in _EMPTY_SAFE_UNARY and _empty(h.inputs[0]) is not None:
            return self._hit("empty-unary", h.inputs[0])
        if op == "t":
            e = _empty(h.inputs[0])
            if e is not None:
                return self._hit("empty-reorg", _zeros(e[1], e[0], h.pos))
            return h
        if op == "mm" and len(h.inputs) == 2:
            A, B = h.inputs
            tA = h.p.get("transA", False)
            eA, eB = _empty(A), _empty(B)
            if eB is not None:
                rows = eA[1 if tA else 0] if eA is not None else (_ncol(A, h.pos) if tA else _nrow(A, h.pos))
                return self._hit("empty-matrix-mult", _zeros(rows, eB[1], h.pos))
            if eA is not None:
                return self._hit("empty-matrix-mult", _zeros(eA[1] if tA else eA[0], _ncol(B, h.pos), h.pos))
            return h
        if op == "b" and h.dt == "M" and len(h.inputs) == 2:
            a, b = h.inputs
            o = h.p["o"]
            ea, eb = _empty(a), _empty(b)
            if o == "*":
                for X, e, E in ((a, eb, b), (b, ea, a)):
                    if e is None:
                        continue
                    if X.dt == "S" or _same_dims(X, *e):
                        return self._hit("empty-binary", E)
            if o in ("+", "-") and eb is not None and _same_dims(a, *eb):
                return self._hit("empty-binary", a)
            if o == "+" and ea is not None and _same_dims(b, *ea):
                return self._hit("empty-binary", b)
            if o == "-" and ea is not None and _same_dims(b, *ea):
                return self._hit("empty-binary", Hop("u", [b], {"o": "neg"}, dt="M", pos=h.pos))
        return h

    # ------------------------------------------------------------------ chains of products
    def _rw_distributive(self, h):
        """simplifyDistributiveBinaryOperation (reference RewriteAlgebraicSimplificationStatic
        .java:760): (X - Y*X) -> (1-Y)*X, (Y*X - X) -> (Y-1)*X, and the same for +; one
        cellwise pass and one operator less, X and Y matrices."""
        a, b = h.inputs
        o = h.p["o"]
        if a.dt != "M" or b.dt != "M":
            return h
        if a.op == "b" and a.p["o"] == "*" and a.id not in self.multi:
            c1, c2 = a.inputs
            if c1.dt == "M" and c2.dt == "M" and c1 is not c2 and (b is c1 or b is c2):
                Y = c2 if b is c1 else c1
                inner = Hop("b", [Y, lit(1)], {"o": o}, dt="M", pos=h.pos)
                return self._hit("distributive-binary", Hop("b", [inner, b], {"o": "*"}, dt="M", pos=h.pos))
        if b.op == "b" and b.p["o"] == "*" and b.id not in self.multi:
            c1, c2 = b.inputs
            if c1.dt == "M" and c2.dt == "M" and c1 is not c2 and (a is c1 or a is c2):
                Y = c2 if a is c1 else c1
                inner = Hop("b", [lit(1), Y], {"o": o}, dt="M", pos=h.pos)
                return self._hit("distributive-binary", Hop("b", [inner, a], {"o": "*"}, dt="M", pos=h.pos))
        return h

    def _rw_emult_chain(self, h):
        """RewriteElementwiseMultChainOptimization (reference
        hops/rewrite/RewriteElementwiseMultChainOptimization.java:56): a chain of >= 3 cellwise
        multiplicands with a repeated one, e.g. (B * A) * B -> A * B^2; scalars are multiplied
        first, repeated operands become powers.  Chains through intermediates with other
        consumers are left alone (their values are needed anyway)."""
        leaves, count = [], {}

        def collect(x, top):
            if x.op == "b" and x.p["o"] == "*" and x.dt == "M" and (top or x.id not in self.multi):
                for c in x.inputs:
                    collect(c, False)
                return
            if x.id not in count:
                leaves.append(x)
                count[x.id] = 0
            count[x.id] += 1
        collect(h, True)
        if sum(count.values()) < 3 or max(count.values()) < 2:
            return h
        scal = [x for x in leaves if x.dt == "S"]
        mats = [x for x in leaves if x.dt != "S"]
        terms = []
        for x in scal + mats:
            k = count[x.id]
            if k == 1:
                terms.append(x)
            elif x.dt == "S":
                for _ in range(k):
                    terms.append(x)
            else:
                terms.append(Hop("b", [x, lit(k)], {"o": "^"}, dt="M", pos=h.pos))
        r = terms[0]
        for t in terms[1:]:
            r = Hop("b", [r, t], {"o": "*"}, dt="M" if (r.dt == "M" or t.dt == "M") else "S", pos=h.pos)
        if r.dt != "M":
            return h
        return self._hit("emult-chain", r)

    def _match_cbind_const(self, h):
        """cbind(X, matrix(1, rows=n, cols=1)) -> _cbind_const(X, 1, n): the intercept column
        of the regression scripts becomes a constant-column view (ops/augmented.py) instead
        of an N x (D+1) copy; the builtin checks n == nrow(X) at run time."""
        if len(h.inputs) != 2 or h.named or h.p.get("npos", 2) != 2:
            return h
        X, Mx = h.inputs
        if X.dt != "M" or Mx.op != "bi" or Mx.p.get("name") != "matrix" or not _is_lit(Mx.inputs[0], 1):
            return h
        args = _bi_args(Mx)
        rows, cols = args.get("rows"), args.get("cols")
        if rows is None or cols is None or not _is_lit(cols, 1) or set(args) - {"data", "rows", "cols"}:
            return h
        self._count("cbind-const")
        return Hop("bi", [X, Mx.inputs[0], rows], {"name": "_cbind_const", "npos": 3}, dt="M", pos=h.pos)

    def _rw_binary(self, h):
        a, b = h.inputs
        o = h.p["o"]
        if a.op == "lit" and b.op == "lit" and a.value is not None and b.value is not None:
            try:
                return lit(S.binary(o, a.value, b.value))
            except DMLRuntimeError:
                return h
        # identities only when the non-literal side is a matrix (keeps scalar value types exact)
        if a.dt == "M" and b.op == "lit":
            if (o in ("*", "/", "^") and _is_lit(b, 1)) or (o in ("+", "-") and _is_lit(b, 0)):
                self._count("identity")
                return a
        if b.dt == "M" and a.op == "lit":
            if (o == "*" and _is_lit(a, 1)) or (o == "+" and _is_lit(a, 0)):
                self._count("identity")
                return b
        if o in ("*", "/") and self.fuse and a.dt == "M" and b.dt == "M":
            q = _wquat_guard(_match_wquat_cell(o, a, b, h), self.multi)
            if q is not None:
                self._count("wquat-" + q.p["kind"])
                return q
        # remove unnecessary outer product with ones: A op (v %*% matrix(1,1,k))
        if o in CELLWISE:
            if b.op == "mm" and not b.p.get("transA") and _is_ones_matrix(b.inputs[1], rows1=True):
                if a.dt == "M":
                    self._count("outer-ones")
                    return Hop("b", [a, b.inputs[0]], dict(h.p), dt="M", pos=h.pos)
            if a.op == "mm" and not a.p.get("transA") and _is_ones_matrix(a.inputs[1], rows1=True):
                if b.dt == "M":
                    self._count("outer-ones")
                    return Hop("b", [a.inputs[0], b], dict(h.p), dt="M", pos=h.pos)
        return h

    def _rw_agg(self, h):
        x = h.inputs[0]
        o, d = h.p["o"], h.p["dir"]
        if d == "all" and o in ("sum", "sumsq") and self.fuse:
            q = _wquat_guard(_match_wquat_agg(o, x, h), self.multi)
            if q is not None:
                self._count("wquat-" + q.p["kind"])
                return q
        if o == "sum":
            if x.op == "b" and x.p["o"] == "^" and _is_lit(x.inputs[1], 2) and x.inputs[0].dt != "S":
                if d == "all" and (_col_vector(x.inputs[0]) or x.inputs[0].dim2 == 1):
                    # simplifyDotProductSum (Dynamic:2075): sum(v^2) is the dot product v'v -- here
                    # the fused sum of squares, which reads v once and needs no transpose
                    self._count("dot-product-sum")
                self._count("sumsq")
                return Hop("agg", [x.inputs[0]], {"o": "sumsq", "dir": d}, dt=h.dt, pos=h.pos)
            if d == "all" and x.op == "b" and x.p["o"] == "*" and x.inputs[0].dt == "M" and x.inputs[1].dt == "M":
                if x.inputs[0] is x.inputs[1]:
                    self._count("sumsq")
                    return Hop("agg", [x.inputs[0]], {"o": "sumsq", "dir": "all"}, dt="S", pos=h.pos)
                self._count("tak+*")
                return Hop("tak", [x.inputs[0], x.inputs[1]], {}, dt="S", pos=h.pos)
            if d == "all" and x.op == "t":
                return Hop("agg", [x.inputs[0]], dict(h.p), dt="S", pos=h.pos)
        return h

    def _rw_mm(self, h):
        a, b = h.inputs
        transA = h.p.get("transA", False)
        if not transA:
            # simplifyScalarMatrixMult (Dynamic.java:922): y %*% X -> as.scalar(y) * X and
            # X %*% y -> X * as.scalar(y) for a 1 x 1 y
            # -- only when X's inner dimension is statically 1, so a mismatched product still
            # raises instead of silently becoming a scaling
            for y, X, inner in ((a, b, b.dim1), (b, a, a.dim2)):
                if _one_by_one(y) and X.dt == "M" and inner == 1:
                    sc = Hop("u", [y], {"o": "cast_scalar"}, dt="S", dim1=0, dim2=0, pos=h.pos)
                    return self._hit("scalar-matrix-mult", Hop("b", [X, sc], {"o": "*"}, dt="M", dim1=X.dim1,
                                                               dim2=X.dim2, pos=h.pos))
            # (X ^ 2) %*% v -> rowSums(X ^ 2 * t(v)) for a column vector v (the rowSums_X_sq
            # idiom of MultiLogReg / GLM with icpt=2): a row aggregate the Cell template fuses
            # with the square, so X ^ 2 is never materialised (a 10M x 1K fp32 X ^ 2 costs more
            # than the two fused passes over X together)
            # Over a constant-column view cbind(X, c) (MultiLogReg's icpt = 2 scaling) the square
            # is split off the view first: (X ^ 2) %*% v[1:D, ] + c ^ 2 * v[D + 1, 1], so it stays
            # over X as a fused row aggregate (the generated row kernels read dense rows only)
            if a.op == "b" and a.p.get("o") == "^" and _is_lit(a.inputs[1], 2) and a.inputs[0].op == "bi" \
                    and a.inputs[0].p.get("name") == "_cbind_const" and b.dt == "M" \
                    and (_col_vector(b) or (b.dim2 == 1 and b.dim1 > 1)):
                X, c, _n = a.inputs[0].inputs
                none = Hop("lit", p={"v": None, "vt": "STRING"}, dt="S", pos=h.pos)
                nr = Hop("u", [b], {"o": "nrow"}, dt="S", dim1=0, dim2=0, pos=h.pos)
                top = Hop("b", [nr, H.lit(1, h.pos)], {"o": "-"}, dt="S", dim1=0, dim2=0, pos=h.pos)
                d1 = b.dim1 - 1 if b.dim1 and b.dim1 > 0 else -1
                vtop = Hop("rix", [b, H.lit(1, h.pos), top, none, none], {}, dt="M", dim1=d1, dim2=1, pos=h.pos)
                vlast = Hop("rix", [b, nr, nr, none, none], {}, dt="M", dim1=1, dim2=1, pos=h.pos)
                xsq = Hop("b", [X, H.lit(2, h.pos)], {"o": "^"}, dt="M", dim1=X.dim1, dim2=X.dim2, pos=h.pos)
                prod = self._rw_mm(Hop("mm", [xsq, vtop], dict(h.p), dt="M", dim1=X.dim1, dim2=1, pos=h.pos))
                c2 = Hop("b", [c, c], {"o": "*"}, dt="S", dim1=0, dim2=0, pos=h.pos)
                sv = Hop("u", [vlast], {"o": "cast_scalar"}, dt="S", dim1=0, dim2=0, pos=h.pos)
                corr = Hop("b", [sv, c2], {"o": "*"}, dt="S", dim1=0, dim2=0, pos=h.pos)
                return self._hit("square-matrix-mult-cbind", Hop("b", [prod, corr], {"o": "+"}, dt="M",
                                                                 dim1=X.dim1, dim2=1, pos=h.pos))
            if a.op == "b" and a.p.get("o") == "^" and _is_lit(a.inputs[1], 2) and a.inputs[0].dt == "M" \
                    and not (a.inputs[0].op == "bi" and a.inputs[0].p.get("name") == "_cbind_const") \
                    and b.dt == "M" and (_col_vector(b) or (b.dim2 == 1 and b.dim1 > 1)):
                tv = Hop("t", [b], {}, dt="M", dim1=1, dim2=b.dim1, pos=h.pos)
                prod = Hop("b", [a, tv], {"o": "*"}, dt="M", dim1=a.dim1, dim2=a.dim2, pos=h.pos)
                return self._hit("square-matrix-mult", Hop("agg", [prod], {"o": "sum", "dir": "row"}, dt="M",
                                                          dim1=a.dim1, dim2=1, pos=h.pos))
            # simplifyMatrixMultDiag (Dynamic.java:960): diag(v) %*% Y -> v * Y for a column
            # vector v (a row scaling instead of an n x n diagonal matrix and a product)
            if _is_diag(a) and _col_vector(a.inputs[0]) and b.dt == "M":
                v = a.inputs[0]
                return self._hit("matrix-mult-diag", Hop("b", [b, v], {"o": "*"}, dt="M", dim1=b.dim1, dim2=b.dim2,
                                                         pos=h.pos))
        # (-A) %*% B -> -(A %*% B): keeps t(X) visible to the transpose / fusion rules
        if a.op == "u" and a.p["o"] == "neg" and a.dt == "M":
            self._count("neg-pushdown")
            inner = self._rw_mm(Hop("mm", [a.inputs[0], b], dict(h.p), dt="M", pos=h.pos))
            return Hop("u", [inner], {"o": "neg"}, dt="M", pos=h.pos)
        if b.op == "u" and b.p["o"] == "neg" and b.dt == "M":
            self._count("neg-pushdown")
            inner = self._rw_mm(Hop("mm", [a, b.inputs[0]], dict(h.p), dt="M", pos=h.pos))
            return Hop("u", [inner], {"o": "neg"}, dt="M", pos=h.pos)
        if not transA:
            g = self._match_pmm(a, b, h)
            if g is not None:
                return g
        if not transA and a.op == "t":
            X = a.inputs[0]
            if b is X:
                self._count("tsmm")
                return Hop("tsmm", [X], {"left": True}, dt="M", pos=h.pos)
            self._count("t(X)%*%Y")
            n = Hop("mm", [X, b], {"transA": True}, dt="M", pos=h.pos)
            return self._rw_mm(n)
        if not transA and b.op == "t" and b.inputs[0] is a:
            self._count("tsmm")
            return Hop("tsmm", [a], {"left": False}, dt="M", pos=h.pos)
        if self.fuse:
            q = _wquat_guard(_match_wdivmm(a, b, transA, h), self.multi)
            if q is not None:
                self._count("wquat-wdivmm")
                return q
        if transA and self.fuse:
            X = a
            m = self._match_mmchain(X, b)
            if m is not None:
                return m
        return h

    def _match_pmm(self, a, b, h):
        """table(seq(1, n), I [, n, L]) %*% B  ->  gather rows B[I] (0 where I is out of range).
        The reference compiles this permutation-matrix product to PMMJ instead of
        materialising the (sparse) selection matrix; a dense n x L selection matrix would
        cost n*L cells here."""
        if a.op == "bi" and a.p.get("name") == "_onehot":     # already rewritten seq-ctable
            y, n, k = a.inputs
            if _is_lit(n, -1):
                return None
            self._count("pmm-gather")
            return Hop("bi", [y, b, n, k], {"name": "_gather_rows", "npos": 4}, dt="M", pos=h.pos)
        if a.op != "bi" or a.p.get("name") not in ("table", "ctable") or a.named:
            return None
        npos = a.p.get("npos", len(a.inputs))
        if npos not in (2, 4):
            return None
        sq = a.inputs[0]
        if sq.op != "bi" or sq.p.get("name") != "seq" or sq.named:
            return None
        sargs = sq.inputs[:sq.p.get("npos", len(sq.inputs))]
        if len(sargs) < 2 or not _is_lit(sargs[0], 1) or (len(sargs) > 2 and not _is_lit(sargs[2], 1)):
            return None
        nrows = a.inputs[2] if npos == 4 else sargs[1]
        ncols = a.inputs[3] if npos == 4 else lit(-1)
        self._count("pmm-gather")
        return Hop("bi", [a.inputs[1], b, nrows, ncols], {"name": "_gather_rows", "npos": 4}, dt="M", pos=h.pos)

    def _match_onehot(self, h):
        """table(seq(1, N), y [, N, K])  ->  one-hot of y (no materialised row-index sequence;
        the reference's ctable with a sequence input is the same special case,
        CtableCPInstruction / LibMatrixReorg 'seq-ctable')."""
        if h.named:
            return h
        npos = h.p.get("npos", len(h.inputs))
        if npos not in (2, 4):
            return h
        sq = h.inputs[0]
        if sq.op != "bi" or sq.p.get("name") != "seq" or sq.named or h.inputs[1].dt == "S":
            return h
        sargs = sq.inputs[:sq.p.get("npos", len(sq.inputs))]
        if len(sargs) < 2 or not _is_lit(sargs[0], 1) or (len(sargs) > 2 and not _is_lit(sargs[2], 1)):
            return h
        n = h.inputs[2] if npos == 4 else sargs[1]
        k = h.inputs[3] if npos == 4 else lit(-1)
        if npos == 2:
            n = lit(-1)      # as many rows as labels (seq(1, nrow(y)) is the usual form)
        self._count("seq-ctable")
        return Hop("bi", [h.inputs[1], n, k], {"name": "_onehot", "npos": 3}, dt="M", pos=h.pos)

    def _match_mmchain(self, X, g):
        def is_xv(n):
            return n.op == "mm" and not n.p.get("transA") and n.inputs[0] is X

        # XtXv
        if is_xv(g):
            self._count("mmchain")
            return Hop("mmchain", [X, g.inputs[1]], {"type": "XtXv"}, dt="M")
        if g.op == "b":
            o = g.p["o"]
            l, r = g.inputs
            if o == "*":
                if is_xv(r) and l.dt == "M":
                    self._count("mmchain")
                    return Hop("mmchain", [X, r.inputs[1], l], {"type": "XtwXv"}, dt="M")
                if is_xv(l) and r.dt == "M":
                    self._count("mmchain")
                    return Hop("mmchain", [X, l.inputs[1], r], {"type": "XtwXv"}, dt="M")
            if o == "-" and is_xv(l) and r.dt == "M":
                self._count("mmchain")
                return Hop("mmchain", [X, l.inputs[1], r], {"type": "XtXvy"}, dt="M")
            # multinomial logreg Hessian-vector product:  Q - P * rowSums(Q),  Q = P * (X %*% V)
            if o == "-":
                Q = l
                if Q.op == "b" and Q.p["o"] == "*":
                    P = None
                    q0, q1 = Q.inputs
                    if is_xv(q1):
                        P, xv = q0, q1
                    elif is_xv(q0):
                        P, xv = q1, q0
                    if P is not None and r.op == "b" and r.p["o"] == "*":
                        r0, r1 = r.inputs
                        for pp, rs in ((r0, r1), (r1, r0)):
                            if pp is P and rs.op == "agg" and rs.p["o"] == "sum" and rs.p["dir"] == "row" \
                                    and rs.inputs[0] is Q:
                                self._count("mmchain-row")
                                return Hop("mmchain", [X, xv.inputs[1], P], {"type": "XtPSXv"}, dt="M")
        return None


# ----------------------------------------------------------------------------
# weighted quaternary operators (reference: hops/rewrite/RewriteAlgebraicSimplificationDynamic
# #simplifyWeighted{SquaredLoss,Sigmoid,DivMM,CrossEntropy,UnaryMM}; executed by
# ops/quaternary.py with sampled products at the non-zeros of sparse W / X)
# ----------------------------------------------------------------------------
_WUMM_UOPS = {"exp", "log", "abs", "sqrt", "sin", "cos", "tan", "tanh", "sign", "round", "floor", "ceil"}


def _uv(h):
    """(U, V) when h is U %*% t(V)."""
    if h.op == "mm" and not h.p.get("transA") and h.inputs[1].op == "t" and h.inputs[0].dt == "M":
        return h.inputs[0], h.inputs[1].inputs[0]
    return None


def _uv_eps(h):
    """(U, V, eps) for U %*% t(V) [+ eps] (eps a scalar)."""
    m = _uv(h)
    if m is not None:
        return m[0], m[1], None
    if h.op == "b" and h.p["o"] == "+":
        for x, e in ((h.inputs[0], h.inputs[1]), (h.inputs[1], h.inputs[0])):
            m = _uv(x)
            if m is not None and e.dt == "S":
                return m[0], m[1], e
    return None


def _is_neg(h):
    if h.op == "u" and h.p["o"] == "neg":
        return h.inputs[0]
    if h.op == "b" and h.p["o"] == "-" and _is_lit(h.inputs[0], 0):
        return h.inputs[1]
    return None


def _wq(kind, ins, p, dt, h, uv=None):
    q = dict(p)
    q["kind"] = kind
    if uv is not None:
        q["_uvid"] = uv.id          # consumed by _wquat_guard
    return Hop("wquat", ins, q, dt=dt, pos=h.pos)


def _known(d):
    return d is not None and d >= 0


def _wquat_guard(q, multi):
    """The reference's applicability checks for the weighted quaternary rewrites
    (hops/rewrite/RewriteAlgebraicSimplificationDynamic#simplifyWeighted*): W / X, U and V
    must have matching sizes where known (a broadcast vector W is not a weight matrix), and
    the U %*% t(V) product must have no other consumer -- otherwise the dense product is
    needed anyway and fusing would compute it twice."""
    if q is None:
        return None
    uvid = q.p.pop("_uvid", None)
    if uvid is not None and uvid in multi:
        return None
    W, U, V = q.inputs[0], q.inputs[1], q.inputs[2]
    if _known(W.dim1) and _known(U.dim1) and W.dim1 != U.dim1:
        return None
    if _known(W.dim2) and _known(V.dim1) and W.dim2 != V.dim1:
        return None
    if len(q.inputs) > 3 and q.p["kind"] == "wsloss" and q.inputs[3].dt == "M":
        W2 = q.inputs[3]
        if (_known(W2.dim1) and _known(W.dim1) and W2.dim1 != W.dim1) or \
                (_known(W2.dim2) and _known(W.dim2) and W2.dim2 != W.dim2):
            return None
    return q


def count_consumers(roots):
    """Ids of hops referenced by more than one parent (or by a root list more than once)."""
    seen, cnt = set(), {}
    stack = list(roots)
    for r in roots:
        cnt[r.id] = cnt.get(r.id, 0) + 1
    while stack:
        h = stack.pop()
        if h.id in seen:
            continue
        seen.add(h.id)
        for c in h.inputs:
            cnt[c.id] = cnt.get(c.id, 0) + 1
            stack.append(c)
    return {k for k, v in cnt.items() if v > 1}


def _match_wquat_agg(o, x, h):
    if o == "sumsq":
        if x.op != "b" or x.p["o"] != "-":
            return None
        A, B = x.inputs
        for X, R in ((A, B), (B, A)):
            if X.dt != "M":
                continue
            m = _uv(R)
            if m is not None:
                return _wq("wsloss", [X, m[0], m[1]], {"type": "none"}, "S", h, R)
            if X is A and R.op == "b" and R.p["o"] == "*":
                for W, P in (R.inputs, R.inputs[::-1]):
                    m = _uv(P)
                    if m is not None and W.dt == "M":
                        return _wq("wsloss", [X, m[0], m[1], W], {"type": "pre"}, "S", h, P)
        return None
    if x.op == "wquat" and x.p["kind"] == "wumm" and x.p["uop"] == "log" and x.p.get("op") == "*":
        return _wq("wcemm", list(x.inputs), {}, "S", h)
    if x.op != "b" or x.p["o"] != "*":
        return None
    for W, P in (x.inputs, x.inputs[::-1]):
        if W.dt != "M":
            continue
        # sum(W * (X - U%*%t(V))^2)
        if P.op == "b" and P.p["o"] == "^" and _is_lit(P.inputs[1], 2):
            dd = P.inputs[0]
            if dd.op == "b" and dd.p["o"] == "-":
                for X, R in (dd.inputs, dd.inputs[::-1]):
                    m = _uv(R)
                    if m is None or X.dt != "M":
                        continue
                    if W.op == "b" and W.p["o"] == "!=" and W.inputs[0] is X and _is_lit(W.inputs[1], 0):
                        return _wq("wsloss", [X, m[0], m[1]], {"type": "post_nz"}, "S", h, R)
                    return _wq("wsloss", [X, m[0], m[1], W], {"type": "post"}, "S", h, R)
        # sum(X * log(U%*%t(V) [+ eps]))
        if P.op == "u" and P.p["o"] == "log":
            m = _uv_eps(P.inputs[0])
            if m is not None:
                U, V, e = m
                return _wq("wcemm", [W, U, V] + ([e] if e is not None else []), {"eps": e is not None}, "S", h, P.inputs[0])
    return None


def _match_wquat_cell(o, a, b, h):
    if o == "*":
        for W, P in ((a, b), (b, a)):
            lg = False
            s = P
            if s.op == "u" and s.p["o"] == "log" and s.inputs[0].op == "u" and s.inputs[0].p["o"] == "sigmoid":
                lg, s = True, s.inputs[0]
            if s.op == "u" and s.p["o"] == "sigmoid":
                z = s.inputs[0]
                n = _is_neg(z)
                m = _uv(n if n is not None else z)
                if m is not None:
                    return _wq("wsigmoid", [W, m[0], m[1]], {"minus": n is not None, "log": lg}, "M", h,
                               n if n is not None else z)
    cands = [(a, b)] if o == "/" else [(a, b), (b, a)]
    for X, P in cands:
        if P.op == "u" and P.p["o"] in _WUMM_UOPS:
            m = _uv(P.inputs[0])
            if m is not None:
                return _wq("wumm", [X, m[0], m[1]], {"uop": P.p["o"], "op": o}, "M", h, P.inputs[0])
        if P.op == "b" and P.p["o"] == "^" and _is_lit(P.inputs[1], 2):
            m = _uv(P.inputs[0])
            if m is not None:
                return _wq("wumm", [X, m[0], m[1]], {"uop": "^2", "op": o}, "M", h, P.inputs[0])
    return None


def _match_wdivmm(a, b, transA, h):
    """(W / (U%*%t(V) [+eps])) %*% V,  t(U) %*% (W / (U%*%t(V) [+eps])), and the W * (U%*%t(V))
    forms."""
    q, other = (b, a) if transA else (a, b)
    if q.op != "b" or q.p["o"] not in ("/", "*") or q.inputs[0].dt != "M":
        return None
    mult = q.p["o"] == "*"
    cands = [(q.inputs[0], q.inputs[1])]
    if mult:
        cands.append((q.inputs[1], q.inputs[0]))
    for W, R in cands:
        Xm = None
        if mult and R.op == "b" and R.p["o"] == "-" and R.inputs[1].dt == "M" and _uv(R.inputs[0]):
            # W * (U %*% t(V) - X): the residual form of ALS gradients (reference
            # WDivMMType MULT_MINUS_LEFT / MULT_MINUS_RIGHT)
            Xm = R.inputs[1]
            m = _uv(R.inputs[0]) + (None,)
            uvh = R.inputs[0]
        else:
            m = _uv_eps(R) if not mult else (_uv(R) + (None,) if _uv(R) else None)
            uvh = R
        if m is None:
            continue
        U, V, e = m
        if (transA and other is U) or (not transA and other is V):
            ins = [W, U, V] + ([e] if e is not None else []) + ([Xm] if Xm is not None else [])
            return _wq("wdivmm", ins, {"left": transA, "mult": mult, "eps": e is not None, "minus": Xm is not None},
                       "M", h, uvh)
    return None


def cse(roots):
    """Hash-consing common subexpression elimination over a set of roots."""
    table = {}
    memo = {}

    def visit(h):
        r = memo.get(h.id)
        if r is not None:
            return r
        new_inputs = [visit(c) for c in h.inputs]
        if any(a is not b for a, b in zip(new_inputs, h.inputs)):
            h.inputs = new_inputs
        if h.op in ("fcall", "sink", "fout", "lix") or (h.op == "bi" and h.p.get("name") in H.NONDETERMINISTIC
                                                        | {"exists", "time", "eval", "list"}):
            memo[h.id] = h
            return h
        if h.op == "lit":
            v = h.value
            k = ("lit", S.vtype_of(v), "NaN" if isinstance(v, float) and v != v else v)
        else:
            k = h.key()
        old = table.get(k)
        if old is None:
            table[k] = h
            old = h
        memo[h.id] = old
        return old

    return [visit(r) for r in roots], visit


_ROWGEN = __import__('os').environ.get('SYSML_ROWGEN', '1') != '0'   # Row / Outer templates on
_VECGEN = __import__('os').environ.get('SYSML_VECGEN', '1') != '0'   # Vector template on
# the hand-matched softmax gradient / objective operators (smgrad / smobj, chain4m kernels); off:
# the Row template plans the same passes as generated multi-output programs
SOFTMAX_MATCHER = __import__('os').environ.get('SYSML_SOFTMAX_MATCHER', '1') != '0'
# horizontal Cell batches (codegen.batch_cells): same-program updates of many small operands in
# one launch
CELL_BATCH = __import__('os').environ.get('SYSML_CELL_BATCH', '1') != '0'


def fuse_conv_bias(bb, config=None):
    """bias_add(conv2d(X, W, ...), b) -> conv2d(X, W, ..., bias = b) when the convolution has no
    other consumer (reference: hops/DnnOp CONV2D_BIAS_ADD): the bias is added in the
    convolution kernel's epilogue instead of a second pass over the output -- on every path,
    the 1x1 convolutions' image-blocked GEMM (gemm.hip sysml_gemm_dnn) included.  Returns the
    number of fused pairs."""
    live = getattr(bb, "live_out", None)
    tops = list(bb.roots) + list(bb.env_out.values())
    outs = {h.id for h in bb.roots} | {h.id for k, h in bb.env_out.items() if live is None or k in live}
    shared = count_consumers(tops)             # ids with more than one consumer
    n = 0
    for h in H.walk(tops):
        if not (h.op == "bi" and h.p.get("name") == "bias_add" and len(h.inputs) == 2 and not h.named):
            continue
        c, b = h.inputs
        if not (c.op == "bi" and c.p.get("name") == "conv2d" and "bias" not in c.named) or c.id in outs \
                or c.id in shared:
            continue
        h.p = dict(c.p)
        h.inputs = list(c.inputs) + [b]
        h.named = list(c.named) + ["bias"]
        n += 1
    return n


def _same_index(a, b):
    return a is b or (a.op == "lit" and b.op == "lit" and a.value is not None and a.value == b.value)


def vectorize_indexing(bb):
    """RewriteIndexingVectorization.vectorizeRightIndexing (reference
    hops/rewrite/RewriteIndexingVectorization.java:43): several single-cell reads X[i, j1],
    X[i, j2], ... of one row (literal columns) become one row-segment read X[i, jmin:jmax]
    and cell reads of that small vector (likewise for one column): one pass over X instead of
    one per cell.  Returns the number of rewritten reads."""
    live = getattr(bb, "live_out", None)
    tops = list(bb.roots) + list(bb.env_out.values())
    groups = {}
    for h in H.walk(tops):
        if h.op != "rix" or h.p.get("list") or len(h.inputs) != 5 or h.inputs[0].dt != "M":
            continue
        src, rl, ru, cl, cu = h.inputs
        if _same_index(rl, ru) and rl.value is not None and _num_lit(cl) and _same_index(cl, cu) \
                and isinstance(cl.value, int):
            key = ("r", src.id, rl.id if rl.op != "lit" else ("lit", rl.value))
            groups.setdefault(key, []).append((h, cl.value))
        elif _same_index(cl, cu) and cl.value is not None and _num_lit(rl) and _same_index(rl, ru) \
                and isinstance(rl.value, int):
            key = ("c", src.id, cl.id if cl.op != "lit" else ("lit", cl.value))
            groups.setdefault(key, []).append((h, rl.value))
    n = 0
    for (kind, _, _), hs in groups.items():
        idx = {j for _, j in hs}
        if len(idx) < 2:
            continue
        lo, hi = min(idx), max(idx)
        if hi - lo + 1 > 4 * len(idx):
            continue                      # sparse accesses: the segment would read mostly unused cells
        h0 = hs[0][0]
        src, rl, ru, cl, cu = h0.inputs
        none = Hop("lit", p={"v": None, "vt": "STRING"}, dt="S", pos=h0.pos)
        if kind == "r":
            seg = Hop("rix", [src, rl, ru, lit(lo), lit(hi)], {}, dt="M", pos=h0.pos)
        else:
            seg = Hop("rix", [src, lit(lo), lit(hi), cl, cu], {}, dt="M", pos=h0.pos)
        for h, j in hs:
            k = lit(j - lo + 1)
            h.inputs = [seg, none, none, k, k] if kind == "r" else [seg, k, k, none, none]
            n += 1
    return n


def rewrite_block(bb, config=None):
    """Rewrite a BasicBlock's DAG in place (roots + env_out)."""
    rw = Rewriter(config)
    rw.multi = count_consumers(list(bb.roots) + list(bb.env_out.values()))
    bb.roots = [rw.rewrite(r) for r in bb.roots]
    bb.env_out = {k: rw.rewrite(v) for k, v in bb.env_out.items()}
    roots, visit = cse(bb.roots)
    bb.roots = roots
    bb.env_out = {k: visit(v) for k, v in bb.env_out.items()}
    if rw.enabled:
        n = vectorize_indexing(bb)
        if n:
            rw.stats["indexing-vectorization"] = n
    if rw.enabled and rw.fuse:
        n = fuse_conv_bias(bb, config)
        if n:
            rw.stats["conv2d-bias-add"] = n
        n = fuse_softmax_grad(bb) if SOFTMAX_MATCHER else 0
        if n:
            rw.stats["softmax-grad"] = n
            nobj = sum(1 for h in H.walk(list(bb.roots) + list(bb.env_out.values())) if h.op == "smobj")
            if nobj:
                rw.stats["softmax-objective"] = nobj
        from .codegen import fuse_cells, fuse_rows, fuse_outer
        if _ROWGEN:
            n = fuse_outer(bb)
            if n:
                rw.stats["outer-fused-ops"] = n
            n = fuse_rows(bb)
            if n:
                rw.stats["row-fused-ops"] = n
                from .codegen import merge_row_programs
                m = merge_row_programs(bb)
                if m:
                    rw.stats["row-multi-output"] = m
        if _VECGEN and (config is None or getattr(config, "gpu", True)):
            # Vector template: only a GPU backend has launches and round trips to save
            from .vecgen import fuse_vectors
            n = fuse_vectors(bb)
            if n:
                rw.stats["vector-fused-ops"] = n
        n = fuse_cells(bb, single=_VECGEN and (config is None or getattr(config, "gpu", True)), stats=rw.stats)
        if n:
            rw.stats["cell-fused-ops"] = n
        if CELL_BATCH and (config is None or getattr(config, "gpu", True)):
            from .codegen import batch_cells
            n = batch_cells(bb)
            if n:
                rw.stats["cell-batched"] = n
    return rw.stats


# ----------------------------------------------------------------------------
# two-output row template: X %*% V and t(X) %*% (softmax(cbind(X %*% V, 0))[, 1:K] - Y)
# ----------------------------------------------------------------------------
def _agg_row(h, o):
    return h.op == "agg" and h.p.get("o") == o and h.p.get("dir") == "row"


def _match_softmax_grad(G):
    """G = mm(X, g, transA) with g = P[, 1:cu] - Y, P = E / rowSums(E), E = exp(L - rowMaxs(L)),
    L = cbind(U, matrix(0, N, 1)), U = X %*% V  ->  (X, U, V, Y, cu) or None.
    This is the candidate-point evaluation of MultiLogReg's trust-region step (the
    reference's codegen forms a Row template for it, hops/codegen/template/TemplateRow.java)."""
    if G.op != "mm" or not G.p.get("transA"):
        return None
    X, g = G.inputs
    if g.op != "b" or g.p.get("o") != "-" or g.inputs[0].op != "rix":
        return None
    rx, Y = g.inputs
    P, rl, ru, cl, cu = rx.inputs
    def empty(x):
        return x.op == "lit" and x.value is None
    if not (empty(rl) and empty(ru) and _is_lit(cl, 1)) or Y.dt != "M":
        return None
    if P.op != "b" or P.p.get("o") != "/":
        return None
    E, s = P.inputs
    if not (_agg_row(s, "sum") and s.inputs[0] is E and E.op == "u" and E.p.get("o") == "exp"):
        return None
    L2 = E.inputs[0]
    if L2.op != "b" or L2.p.get("o") != "-":
        return None
    L, mx = L2.inputs
    if not (_agg_row(mx, "max") and mx.inputs[0] is L and L.op == "bi" and L.p.get("name") == "cbind"
            and len(L.inputs) == 2 and not L.named):
        return None
    U, Z = L.inputs
    if not (U.op == "mm" and not U.p.get("transA") and U.inputs[0] is X):
        return None
    if not (Z.op == "bi" and Z.p.get("name") == "matrix" and Z.inputs and _is_lit(Z.inputs[0], 0)):
        return None
    zc = _bi_args(Z).get("cols")
    if zc is None or not _is_lit(zc, 1):
        return None
    return X, U, U.inputs[1], Y, cu, (P, L2, s)


def _same_var(a, b):
    """Same hop, or transient reads of the same variable (a loop-invariant read in the body and
    its hoisted twin: the variable is not reassigned in between)."""
    return a is b or (a.op == "tread" and b.op == "tread" and a.p.get("name") == b.p.get("name"))


def _full_cols_rix(Y, cu):
    """Y = Ybase[, 1:cu] (all rows, possibly hoisted out of the loop by LICM)  ->  Ybase, else None."""
    if Y.op == "tread" and Y.p.get("licm_def") is not None:
        Y = Y.p["licm_def"]
    if Y.op != "rix":
        return None
    b, rl, ru, cl, cu2 = Y.inputs

    def empty(x):
        return x.op == "lit" and x.value is None
    if empty(rl) and empty(ru) and _is_lit(cl, 1) and (cu2 is cu or (cu2.op == "lit" and cu.op == "lit"
                                                                     and cu2.value == cu.value)):
        return b
    return None


def _objective_terms(order, Yb, L2, s):
    """The two data terms of the multinomial-logreg objective over the matched softmax:
    sum(Yb * L2) (as agg-sum of a product or a tak+* dot) and sum(log(rowSums(E)))."""
    s1 = s2 = None
    yop = None

    def pair(ins):
        if len(ins) != 2:
            return None
        a, b = ins
        if b is L2 and _same_var(a, Yb):
            return a
        if a is L2 and _same_var(b, Yb):
            return b
        return None
    for h in order:
        if s1 is None:
            if h.op == "tak":
                y = pair(h.inputs)
                if y is not None:
                    s1, yop = h, y
            elif h.op == "agg" and h.p.get("o") == "sum" and h.p.get("dir") == "all":
                x = h.inputs[0]
                if x.op == "b" and x.p.get("o") == "*":
                    y = pair(x.inputs)
                    if y is not None:
                        s1, yop = h, y
        if s2 is None and h.op == "agg" and h.p.get("o") == "sum" and h.p.get("dir") == "all":
            x = h.inputs[0]
            if x.op == "u" and x.p.get("o") == "log" and x.inputs[0] is s:
                s2 = h
    return s1, s2, yop


def _reaches(roots, target):
    seen = set()
    stack = list(roots)
    while stack:
        h = stack.pop()
        if h is target:
            return True
        if h.id in seen:
            continue
        seen.add(h.id)
        stack.extend(h.inputs)
    return False


def fuse_softmax_grad(bb):
    """Replace every matched (U, G) pair by the outputs of one `smgrad` hop (one pass over X)."""
    seen = set()
    order = []

    def walk(h):
        if h.id in seen:
            return
        seen.add(h.id)
        for c in h.inputs:
            walk(c)
        order.append(h)

    for r in list(bb.roots) + list(bb.env_out.values()):
        walk(r)
    def apply(repl):
        memo = {}

        def sub(h):
            r = repl.get(h.id)
            if r is not None:
                return r
            if h.id in memo:
                return h
            memo[h.id] = True
            h.inputs = [sub(c) for c in h.inputs]
            return h

        # the fused hop's own inputs must not be rewritten to its outputs
        for r in repl.values():
            F = r.inputs[0]
            if F.id not in memo:
                memo[F.id] = True
                F.inputs = [sub(c) for c in F.inputs]
        bb.roots = [sub(h) for h in bb.roots]
        bb.env_out = {k: sub(v) for k, v in bb.env_out.items()}

    nfused = 0
    done = set()
    for h in order:
        m = _match_softmax_grad(h)
        if m is None:
            continue
        X, U, V, Y, cu, (P, L2, srow) = m
        if U.id in done:
            continue
        done.add(U.id)
        # objective form (op smobj): the probabilities, the gradient and the objective's data
        # terms in one pass, when nothing else reads X %*% V or the intermediate matrices
        Yb = _full_cols_rix(Y, cu)
        if Yb is not None:
            s1, s2, yop = _objective_terms(order, Yb, L2, srow)
            if s1 is not None and s2 is not None:
                F = Hop("smobj", [X, V, yop, cu], {}, dt="U", pos=h.pos)
                repl = {P.id: Hop("fout", [F], {"i": 0}, dt="M", pos=P.pos),
                        h.id: Hop("fout", [F], {"i": 1}, dt="M", pos=h.pos),
                        s1.id: Hop("fout", [F], {"i": 2}, dt="S", pos=s1.pos),
                        s2.id: Hop("fout", [F], {"i": 3}, dt="S", pos=s2.pos)}
                saved = (list(bb.roots), dict(bb.env_out), [list(x.inputs) for x in order])
                apply(repl)
                live = bb.live_out
                outs = [v for k, v in bb.env_out.items() if live is None or k in live]
                if not _reaches(list(bb.roots) + outs, U):
                    nfused += 1
                    continue
                # another consumer still needs X %*% V: undo, fuse (U, G) only
                bb.roots, bb.env_out = saved[0], saved[1]
                for x, ins in zip(order, saved[2]):
                    x.inputs = ins
        F = Hop("smgrad", [X, V, Y, cu], {}, dt="U", pos=h.pos)
        apply({U.id: Hop("fout", [F], {"i": 0}, dt="M", pos=U.pos),
               h.id: Hop("fout", [F], {"i": 1}, dt="M", pos=h.pos)})
        nfused += 1
    return nfused


def rewrite_pred(pred, config=None):
    rw = Rewriter(config)
    pred.root = rw.rewrite(pred.root)
    if pred.root.op == "lit":
        pred.is_const = True
        pred.const = pred.root.value
