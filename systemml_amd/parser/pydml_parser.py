"""PyDML (Python-like DML) front end (reference: parser/pydml/Pydml.g4 and
PydmlSyntacticValidator.java).

Produces the same AST as the DML parser, applying PyDML's translation rules:
  * indentation blocks, `if/elif/else:`, `for i in a:b` / `for i in range(a, b[, s])`,
    `parfor`, `while`, `def f(x: matrix[float]) -> (y: matrix[float]):`, `defExternal`
  * 0-based, upper-exclusive slicing  X[a:b, c]  →  DML X[a+1:b, c+1]
  * operators  ** (power), // (int div), % (mod), and/or, True/False;  no %*% — dot(A, B)
  * builtins with an `axis` argument (sum/mean/var/sd/min/max/argmin/argmax/cumsum)
    map to row/column aggregates; `X.shape(0)`, `X.reshape(r, c)`, `len`, `full`,
    `random.normal/uniform/poisson`, `norm.cdf`..., `load`/`save`, `scalar/float/int/bool`,
    `transpose`, `power`, `range`, `percentile`, `arcsin/arccos/arctan`, `minimum/maximum`,
    `concatenate` (cbind), `print`.
"""
from __future__ import annotations

import os

from . import ast as A
from .dml_parser import BaseParser, normalize_vtype, normalize_dtype

_BP = {
    "|": 10, "or": 10,
    "&": 20, "and": 20,
    ">": 30, ">=": 30, "<": 30, "<=": 30, "==": 30, "!=": 30,
    "+": 40, "-": 40,
    "*": 50, "/": 50,
    "//": 60, "%": 60,
    "**": 80,
}
_OPMAP = {"**": "^", "//": "%/%", "%": "%%", "and": "&", "or": "|"}
KEYWORDS = {"if", "elif", "else", "for", "parfor", "while", "def", "defExternal", "in", "source", "setwd",
            "ifdef", "True", "False", "implemented", "as", "and", "or"}


def _lit(v, vt, pos):
    return A.Literal(v, vt, pos=pos)


class PyDMLParser(BaseParser):
    pydml = True

    def parse(self) -> A.Program:
        stmts, funcs, imports = [], {}, []
        while self.tok.kind != "EOF":
            if self.tok.kind in ("NEWLINE", "DEDENT", "INDENT"):
                self.i += 1
                continue
            if self.is_kw("def") or self.is_kw("defExternal"):
                f = self.parse_function_def()
                funcs[f.name] = f
                continue
            s = self.parse_statement()
            if s is None:
                continue
            if isinstance(s, A.Import):
                imports.append(s)
            stmts.append(s)
        return A.Program(stmts, funcs, imports, source_path=self.filename)

    # -- helpers -----------------------------------------------------------------
    def end_stmt(self):
        self.skip_semis()
        if self.tok.kind == "NEWLINE":
            self.i += 1
        elif self.tok.kind not in ("EOF", "DEDENT"):
            self.error("expected end of statement")

    def parse_suite(self):
        self.expect_op(":")
        if self.tok.kind != "NEWLINE":
            s = self.parse_statement()
            return [s] if s is not None else []
        self.i += 1
        while self.tok.kind == "NEWLINE":
            self.i += 1
        if self.tok.kind != "INDENT":
            self.error("expected an indented block")
        self.i += 1
        body = []
        while self.tok.kind not in ("DEDENT", "EOF"):
            if self.tok.kind == "NEWLINE":
                self.i += 1
                continue
            s = self.parse_statement()
            if s is not None:
                body.append(s)
        if self.tok.kind == "DEDENT":
            self.i += 1
        return body

    def _paren_opt_expr(self):
        return self.parse_expr()

    # -- statements ------------------------------------------------------------------
    def parse_statement(self):
        t = self.tok
        p = self.pos()
        if t.kind == "STRING":            # docstring
            self.i += 1
            self.end_stmt()
            return None
        if t.kind == "ID":
            v = t.value
            if v == "source" and self.is_op("(", self.peek()):
                self.i += 2
                path = self._string()
                self.expect_op(")")
                self.expect_kw("as")
                ns = self.expect_id()
                self.end_stmt()
                return A.Import(path, ns, pos=p)
            if v == "setwd":
                self.i += 2
                path = self._string()
                self.expect_op(")")
                self.end_stmt()
                return A.SetWd(path, pos=p)
            if v == "if":
                self.i += 1
                pred = self._paren_opt_expr()
                then = self.parse_suite()
                return self._parse_else(A.If(pred, then, [], pos=p))
            if v in ("for", "parfor"):
                self.i += 1
                paren = self.accept_op("(")
                var = self.expect_id()
                self.expect_kw("in")
                start, end, incr = self._parse_iterable()
                params = {}
                while self.accept_op(","):
                    pn = self.expect_id()
                    self.expect_op("=")
                    params[pn] = self.parse_expr()
                if paren:
                    self.expect_op(")")
                body = self.parse_suite()
                return A.For(var, start, end, incr, body, parfor=(v == "parfor"), params=params, pos=p)
            if v == "while":
                self.i += 1
                pred = self._paren_opt_expr()
                body = self.parse_suite()
                return A.While(pred, body, pos=p)
            if self.is_op("(", self.peek()) and v not in KEYWORDS:
                call = self.parse_primary()
                self.end_stmt()
                return A.ExprStmt(call, pos=p)
        if self.is_op("["):
            self.i += 1
            targets = [self._data_identifier()]
            while self.accept_op(","):
                targets.append(self._data_identifier())
            self.expect_op("]")
            self.expect_op("=")
            val = self.parse_expr()
            self.end_stmt()
            return A.MultiAssign(targets, val, pos=p)
        target = self._data_identifier()
        if self.accept_op("+="):
            val = self.parse_expr()
            self.end_stmt()
            return A.Assign(target, val, accumulate=True, pos=p)
        self.expect_op("=")
        if self.is_kw("ifdef") and self.is_op("(", self.peek()):
            self.i += 2
            cp = self._data_identifier()
            self.expect_op(",")
            dflt = self.parse_expr()
            self.expect_op(")")
            self.end_stmt()
            return A.Assign(target, dflt, ifdef=cp, pos=p)
        val = self.parse_expr()
        self.end_stmt()
        return A.Assign(target, val, pos=p)

    def _parse_else(self, node):
        if self.is_kw("elif"):
            p = self.pos()
            self.i += 1
            pred = self._paren_opt_expr()
            body = self.parse_suite()
            inner = self._parse_else(A.If(pred, body, [], pos=p))
            node.else_body = [inner]
        elif self.is_kw("else"):
            self.i += 1
            node.else_body = self.parse_suite()
        return node

    def _string(self):
        t = self.tok
        if t.kind != "STRING":
            self.error("expected string")
        self.i += 1
        return t.value

    def _parse_iterable(self):
        t = self.tok
        if t.kind == "ID" and t.value in ("range", "seq") and self.is_op("(", self.peek()):
            self.i += 2
            a = self.parse_expr()
            self.expect_op(",")
            b = self.parse_expr()
            c = None
            if self.accept_op(","):
                c = self.parse_expr()
            self.expect_op(")")
            return a, b, c
        a = self.parse_expr()
        self.expect_op(":")
        b = self.parse_expr()
        return a, b, None

    def _data_identifier(self):
        t = self.tok
        p = self.pos()
        if t.kind == "CMD":
            self.i += 1
            return A.CmdParam(t.value, pos=p)
        if t.kind != "ID" or t.value in KEYWORDS:
            self.error("expected identifier")
        self.i += 1
        if self.is_op("["):
            return self._index(t.value, p)
        return A.Ident(t.value, pos=p)

    def _index(self, name, p):
        """0-based, upper-exclusive → DML 1-based inclusive."""
        self.expect_op("[")
        rows = self._range(name, ("]", ","), "nrow")
        cols = None
        if self.accept_op(","):
            cols = self._range(name, ("]",), "ncol")
        self.expect_op("]")
        return A.Indexed(name, rows, cols, pos=p)

    def _range(self, name, stops, dimfn):
        r = A.IndexRange()
        if any(self.is_op(s) for s in stops):
            return r
        one = _lit(1, "INT", self.pos())
        if self.is_op(":"):
            self.i += 1
            r.is_range = True
            r.lower = one
            if not any(self.is_op(s) for s in stops):
                r.upper = self.parse_expr()
            else:
                r.upper = A.Call(dimfn, [A.Arg(None, A.Ident(name))])
            return r
        lo = self.parse_expr()
        r.lower = A.BinOp("+", lo, one)
        if self.accept_op(":"):
            r.is_range = True
            if not any(self.is_op(s) for s in stops):
                r.upper = self.parse_expr()
            else:
                r.upper = A.Call(dimfn, [A.Arg(None, A.Ident(name))])
        return r

    # -- function definitions -----------------------------------------------------
    def parse_function_def(self):
        p = self.pos()
        kind = self.expect_id()
        name = self.expect_id()
        self.expect_op("(")
        inputs = self._typed_args()
        self.expect_op(")")
        outputs = []
        if self.accept_op("->"):
            self.expect_op("(")
            outputs = self._typed_args()
            self.expect_op(")")
        if kind == "defExternal":
            self.expect_kw("implemented")
            self.expect_kw("in")
            self.expect_op("(")
            params = {}
            while not self.is_op(")"):
                k = self.expect_id()
                self.expect_op("=")
                params[k] = self._string()
                if not self.accept_op(","):
                    break
            self.expect_op(")")
            self.end_stmt()
            return A.FunctionDef(name, inputs, outputs, [], external=True, ext_params=params, pos=p)
        body = self.parse_suite()
        return A.FunctionDef(name, inputs, outputs, body, pos=p)

    def _typed_args(self):
        args = []
        while not self.is_op(")"):
            nm = self.expect_id()
            self.expect_op(":")
            t = self.expect_id()
            if self.accept_op("["):
                vt = self.expect_id()
                self.expect_op("]")
                dt, vtn = normalize_dtype(t), normalize_vtype(vt)
            else:
                dt, vtn = "SCALAR", normalize_vtype(t)
            dflt = None
            if self.accept_op("="):
                dflt = self.parse_expr()
            args.append(A.Param(nm, dt, vtn, dflt))
            if not self.accept_op(","):
                break
        return args

    # -- expressions ------------------------------------------------------------------
    def parse_expr(self, rbp=0):
        left = self.parse_prefix()
        while True:
            t = self.tok
            key = t.value if (t.kind == "OP" or (t.kind == "ID" and t.value in ("and", "or"))) else None
            if key not in _BP:
                break
            bp = _BP[key]
            if bp <= rbp:
                break
            self.i += 1
            p = A.Pos(t.line, t.col, self.filename)
            right = self.parse_expr(bp - 1 if key == "**" else bp)
            left = A.BinOp(_OPMAP.get(key, key), left, right, pos=p)
        return left

    def parse_prefix(self):
        t = self.tok
        p = self.pos()
        if t.kind == "OP" and t.value in ("-", "+"):
            self.i += 1
            operand = self.parse_expr(75)
            if t.value == "-" and isinstance(operand, A.Literal) and operand.vtype in ("INT", "DOUBLE"):
                return _lit(-operand.value, operand.vtype, p)
            return A.UnOp(t.value, operand, pos=p)
        if (t.kind == "OP" and t.value == "!") or (t.kind == "ID" and t.value == "not"):
            self.i += 1
            return A.UnOp("!", self.parse_expr(25), pos=p)
        return self.parse_primary()

    def parse_primary(self):
        t = self.tok
        p = self.pos()
        if t.kind in ("INT", "DOUBLE", "STRING"):
            self.i += 1
            return _lit(t.value, t.kind, p)
        if t.kind == "CMD":
            self.i += 1
            return A.CmdParam(t.value, pos=p)
        if self.is_op("("):
            self.i += 1
            e = self.parse_expr()
            self.expect_op(")")
            return e
        if self.is_op("["):
            self.i += 1
            items = [self.parse_expr()]
            while self.accept_op(","):
                items.append(self.parse_expr())
            self.expect_op("]")
            return A.ExprList(items, pos=p)
        if t.kind == "ID":
            v = t.value
            if v in ("True", "False", "TRUE", "FALSE"):
                self.i += 1
                return _lit(v in ("True", "TRUE"), "BOOLEAN", p)
            self.i += 1
            if self.is_op("("):
                return self._call(v, p)
            if self.is_op("[") and self.tok.line == t.line:
                return self._index(v, p)
            return A.Ident(v, pos=p)
        self.error("unexpected token in expression")

    def _call(self, name, p):
        self.expect_op("(")
        args = []
        while not self.is_op(")"):
            pname = None
            if self.tok.kind == "ID" and self.is_op("=", self.peek()):
                pname = self.tok.value
                self.i += 2
            args.append(A.Arg(pname, self.parse_expr()))
            if not self.accept_op(","):
                break
        self.expect_op(")")
        return translate_call(name, args, p)


_AXIS_FN = {
    "sum": ("sum", "rowSums", "colSums"), "mean": ("mean", "rowMeans", "colMeans"),
    "avg": ("mean", "rowMeans", "colMeans"), "var": ("var", "rowVars", "colVars"),
    "sd": ("sd", "rowSds", "colSds"), "max": ("max", "rowMaxs", "colMaxs"),
    "min": ("min", "rowMins", "colMins"), "argmax": (None, "rowIndexMax", None),
    "argmin": (None, "rowIndexMin", None), "cumsum": ("cumsum", None, "cumsum"),
    "transpose": ("t", None, None), "trace": ("trace", None, None),
}
_RENAME = {"len": "length", "concatenate": "cbind", "minimum": "pmin", "maximum": "pmax",
           "scalar": "as.scalar", "float": "as.double", "int": "as.integer", "bool": "as.logical",
           "load": "read", "save": "write", "arcsin": "asin", "arccos": "acos", "arctan": "atan",
           "percentile": "quantile", "range": "seq", "full": "matrix"}


def translate_call(name, args, p):
    ns = None
    if "." in name and not name.startswith(("as.", "index.", "empty.", "lower.", "upper.")):
        ns, name = name.rsplit(".", 1)
    pos_args = [a for a in args if a.name is None]
    named = {a.name: a.value for a in args if a.name is not None}
    if ns is not None:
        if name == "shape":
            fn = "nrow" if (isinstance(pos_args[0].value, A.Literal) and pos_args[0].value.value == 0) else "ncol"
            return A.Call(fn, [A.Arg(None, A.Ident(ns))], pos=p)
        if name == "reshape":
            return A.Call("matrix", [A.Arg(None, A.Ident(ns))] + [A.Arg(n, a.value) for n, a in
                                                                zip(("rows", "cols"), pos_args)], pos=p)
        if ns == "random":
            pdf = {"normal": "normal", "uniform": "uniform", "poisson": "poisson"}[name]
            out = [A.Arg("pdf", _lit(pdf, "STRING", p))]
            names = {"normal": ("rows", "cols", "sparsity", "seed"), "uniform": ("rows", "cols", "min", "max",
                                                                                  "sparsity", "seed"),
                     "poisson": ("rows", "cols", "lambda", "sparsity", "seed")}[name]
            for n, a in zip(names, pos_args):
                out.append(A.Arg(n, a.value))
            out += [A.Arg(k, v) for k, v in named.items()]
            return A.Call("rand", out, pos=p)
        cdfs = {"norm": "pnorm", "expon": "pexp", "chi": "pchisq", "f": "pf", "t": "pt"}
        if name == "cdf" and ns in cdfs:
            return A.Call(cdfs[ns], args, pos=p)
        return A.Call(name, args, namespace=ns, pos=p)
    if name in _AXIS_FN:
        full, row, col = _AXIS_FN[name]
        axis = named.pop("axis", None)
        rest = [a for a in args if a.name != "axis"]
        if axis is None:
            if name in ("max", "min") and len(pos_args) > 1:
                return A.Call(name, rest, pos=p)
            return A.Call(full or name, rest, pos=p)
        ax = axis.value if isinstance(axis, A.Literal) else None
        fn = col if ax == 0 else row
        if fn is None:
            raise ValueError(f"{name}(axis={ax}) not supported")
        return A.Call(fn, rest, pos=p)
    if name == "dot":
        return A.BinOp("%*%", pos_args[0].value, pos_args[1].value, pos=p)
    if name == "power":
        return A.BinOp("^", pos_args[0].value, pos_args[1].value, pos=p)
    if name == "full":
        return A.Call("matrix", args, pos=p)
    if name == "matrix" and pos_args and isinstance(pos_args[0].value, A.Literal) and \
            pos_args[0].value.vtype == "STRING":
        return A.Call("matrix", args, pos=p)
    return A.Call(_RENAME.get(name, name), args, pos=p)


def parse_pydml(src: str, filename: str = "") -> A.Program:
    return PyDMLParser(src, filename).parse()


def parse_pydml_file(path: str) -> A.Program:
    with open(path) as f:
        return parse_pydml(f.read(), filename=os.path.abspath(path))
