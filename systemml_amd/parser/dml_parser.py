"""Hand-written recursive-descent / Pratt parser for DML.

Implements the language of the reference ANTLR grammar
(reference: src/main/java/org/apache/sysml/parser/dml/Dml.g4:45-190) with the
same operator precedence ladder (tightest first):

    ^ (right assoc)  >  unary -,+  >  %*%  >  %/% %%  >  * /  >  + -
    >  relational  >  !  >  & &&  >  | ||

Statements: import (`source(..) as ns`), `setwd`, (multi-)assignment incl.
`ifdef($p, default)` and `+=`, left-indexed assignment, if/else, for, parfor,
while, function and externalFunction definitions.
"""
from __future__ import annotations

import os
from typing import List

from . import ast as A
from .errors import ParseError
from .lexer import tokenize, Token

KEYWORDS = {"if", "else", "for", "parfor", "while", "function", "externalFunction",
            "return", "in", "source", "setwd", "ifdef", "TRUE", "FALSE", "implemented"}

# binding powers for binary operators
_BP = {
    "|": 10, "||": 10,
    "&": 20, "&&": 20,
    ">": 30, ">=": 30, "<": 30, "<=": 30, "==": 30, "!=": 30,
    "+": 40, "-": 40,
    "*": 50, "/": 50,
    "%/%": 60, "%%": 60,
    "%*%": 70,
    "^": 80,
}
_NOT_BP = 25      # operand of '!' binds tighter than & and |, looser than relational
_UNARY_BP = 75    # operand of unary -/+ : looser than ^, tighter than %*%


class BaseParser:
    pydml = False

    def __init__(self, src: str, filename: str = ""):
        self.filename = filename
        self.toks: List[Token] = tokenize(src, pydml=self.pydml, filename=filename)
        self.i = 0

    # -- token helpers -------------------------------------------------------
    @property
    def tok(self) -> Token:
        return self.toks[self.i]

    def peek(self, k=1) -> Token:
        j = min(self.i + k, len(self.toks) - 1)
        return self.toks[j]

    def pos(self, t=None) -> A.Pos:
        t = t or self.tok
        return A.Pos(t.line, t.col, self.filename)

    def error(self, msg, t=None):
        t = t or self.tok
        raise ParseError(f"{self.filename or '<script>'} line {t.line}:{t.col}: {msg} (near {t.value!r})")

    def is_op(self, v, t=None):
        t = t or self.tok
        return t.kind == "OP" and t.value == v

    def is_kw(self, v, t=None):
        t = t or self.tok
        return t.kind == "ID" and t.value == v

    def accept_op(self, v):
        if self.is_op(v):
            self.i += 1
            return True
        return False

    def expect_op(self, v):
        if not self.is_op(v):
            self.error(f"expected '{v}'")
        self.i += 1

    def expect_kw(self, v):
        if not self.is_kw(v):
            self.error(f"expected '{v}'")
        self.i += 1

    def expect_id(self):
        t = self.tok
        if t.kind != "ID":
            self.error("expected identifier")
        self.i += 1
        return t.value

    def skip_semis(self):
        while self.is_op(";"):
            self.i += 1


class DMLParser(BaseParser):
    pydml = False

    def parse(self) -> A.Program:
        stmts, funcs, imports = [], {}, []
        while self.tok.kind != "EOF":
            if self._at_function_def():
                f = self.parse_function_def()
                funcs[f.name] = f
            else:
                s = self.parse_statement()
                if isinstance(s, A.Import):
                    imports.append(s)
                stmts.append(s)
            self.skip_semis()
        return A.Program(stmts, funcs, imports, source_path=self.filename)

    # -- statements ----------------------------------------------------------
    def _at_function_def(self):
        t = self.tok
        return (t.kind == "ID" and t.value not in KEYWORDS and
                (self.is_op("=", self.peek()) or self.is_op("<-", self.peek())) and
                self.peek(2).kind == "ID" and self.peek(2).value in ("function", "externalFunction"))

    def parse_block(self) -> List[A.Stmt]:
        if self.accept_op("{"):
            body = []
            while not self.is_op("}"):
                if self.tok.kind == "EOF":
                    self.error("unexpected end of input in block")
                body.append(self.parse_statement())
                self.skip_semis()
            self.expect_op("}")
            return body
        s = self.parse_statement()
        self.skip_semis()
        return [s]

    def parse_statement(self) -> A.Stmt:
        t = self.tok
        p = self.pos()
        if t.kind == "ID":
            v = t.value
            if v == "source" and self.is_op("(", self.peek()):
                self.i += 2
                path = self._expect_string()
                self.expect_op(")")
                self.expect_kw("as")
                ns = self.expect_id()
                self.skip_semis()
                return A.Import(path, ns, pos=p)
            if v == "setwd" and self.is_op("(", self.peek()):
                self.i += 2
                path = self._expect_string()
                self.expect_op(")")
                self.skip_semis()
                return A.SetWd(path, pos=p)
            if v == "if":
                self.i += 1
                self.expect_op("(")
                pred = self.parse_expr()
                self.expect_op(")")
                then = self.parse_block()
                els = []
                if self.is_kw("else"):
                    self.i += 1
                    els = self.parse_block()
                return A.If(pred, then, els, pos=p)
            if v in ("for", "parfor"):
                self.i += 1
                self.expect_op("(")
                var = self.expect_id()
                self.expect_kw("in")
                start, end, incr = self._parse_iterable()
                params = {}
                while self.accept_op(","):
                    pn = self.expect_id()
                    self.expect_op("=")
                    params[pn] = self.parse_expr()
                self.expect_op(")")
                body = self.parse_block()
                return A.For(var, start, end, incr, body, parfor=(v == "parfor"), params=params, pos=p)
            if v == "while":
                self.i += 1
                self.expect_op("(")
                pred = self.parse_expr()
                self.expect_op(")")
                body = self.parse_block()
                return A.While(pred, body, pos=p)
            if self.is_op("(", self.peek()) and v not in KEYWORDS:
                call = self.parse_primary()
                self.skip_semis()
                if not isinstance(call, A.Call):
                    self.error("expected function call statement")
                return A.ExprStmt(call, pos=p)
        if self.is_op("["):
            # multi-assignment [a, b] = f(...)
            self.i += 1
            targets = [self._parse_data_identifier()]
            while self.accept_op(","):
                targets.append(self._parse_data_identifier())
            self.expect_op("]")
            if not (self.accept_op("=") or self.accept_op("<-")):
                self.error("expected '=' in multi-assignment")
            val = self.parse_expr()
            if not isinstance(val, A.Call):
                self.error("multi-assignment requires a function call on the right-hand side")
            self.skip_semis()
            return A.MultiAssign(targets, val, pos=p)
        target = self._parse_data_identifier()
        if self.accept_op("+="):
            val = self.parse_expr()
            self.skip_semis()
            return A.Assign(target, val, accumulate=True, pos=p)
        if not (self.accept_op("=") or self.accept_op("<-")):
            self.error("expected assignment")
        if self.is_kw("ifdef") and self.is_op("(", self.peek()):
            start = self.i
            self.i += 2
            cp = self._parse_data_identifier()
            if not isinstance(cp, A.CmdParam):
                self.error("ifdef requires a command-line parameter ($name)")
            self.expect_op(",")
            dflt = self.parse_expr()
            close = self.tok
            self.expect_op(")")
            nxt = self.tok
            if nxt.kind == "EOF" or nxt.line != close.line or (nxt.kind == "OP" and nxt.value in (";", "}")):
                self.skip_semis()
                return A.Assign(target, dflt, ifdef=cp, pos=p)
            self.i = start          # ifdef(...) inside a larger expression
        val = self.parse_expr()
        self.skip_semis()
        return A.Assign(target, val, pos=p)

    def _expect_string(self):
        t = self.tok
        if t.kind != "STRING":
            self.error("expected string literal")
        self.i += 1
        return t.value

    def _parse_iterable(self):
        # ID '(' from ',' to (',' incr)? ')'  |  from ':' to
        t = self.tok
        if t.kind == "ID" and t.value == "seq" and self.is_op("(", self.peek()):
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

    def _parse_data_identifier(self):
        t = self.tok
        p = self.pos()
        if t.kind == "CMD":
            self.i += 1
            return A.CmdParam(t.value, pos=p)
        if t.kind != "ID" or t.value in KEYWORDS:
            self.error("expected identifier")
        self.i += 1
        if self.is_op("["):
            return self._parse_index(t.value, p)
        return A.Ident(t.value, pos=p)

    def _parse_index(self, name, p):
        self.expect_op("[")
        rows = self._parse_range(("]", ","))
        cols = None
        if self.accept_op(","):
            cols = self._parse_range(("]",))
        self.expect_op("]")
        return A.Indexed(name, rows, cols, pos=p)

    def _parse_range(self, stops):
        r = A.IndexRange()
        if any(self.is_op(s) for s in stops):
            return r
        if self.is_op(":"):           # implicit lower bound (PyDML style)
            self.i += 1
            r.is_range = True
            if not any(self.is_op(s) for s in stops):
                r.upper = self.parse_expr()
            return r
        r.lower = self.parse_expr()
        if self.accept_op(":"):
            r.is_range = True
            if not any(self.is_op(s) for s in stops):
                r.upper = self.parse_expr()
        return r

    # -- function definitions --------------------------------------------------
    def parse_function_def(self) -> A.FunctionDef:
        p = self.pos()
        name = self.expect_id()
        if not (self.accept_op("=") or self.accept_op("<-")):
            self.error("expected '=' in function definition")
        kind = self.expect_id()
        self.expect_op("(")
        inputs = self._parse_typed_args(")")
        self.expect_op(")")
        outputs = []
        if self.is_kw("return"):
            self.i += 1
            self.expect_op("(")
            outputs = self._parse_typed_args(")")
            self.expect_op(")")
        if kind == "externalFunction":
            self.expect_kw("implemented")
            self.expect_kw("in")
            self.expect_op("(")
            params = {}
            while not self.is_op(")"):
                k = self.expect_id()
                self.expect_op("=")
                params[k] = self._expect_string()
                if not self.accept_op(","):
                    break
            self.expect_op(")")
            self.skip_semis()
            return A.FunctionDef(name, inputs, outputs, [], external=True, ext_params=params, pos=p)
        self.expect_op("{")
        body = []
        while not self.is_op("}"):
            if self.tok.kind == "EOF":
                self.error("unexpected end of input in function body")
            body.append(self.parse_statement())
            self.skip_semis()
        self.expect_op("}")
        self.skip_semis()
        return A.FunctionDef(name, inputs, outputs, body, pos=p)

    def _parse_typed_args(self, stop):
        args = []
        while not self.is_op(stop):
            dtype, vtype = self._parse_type()
            nm = self.expect_id()
            dflt = None
            if self.accept_op("="):
                dflt = self.parse_expr()
            args.append(A.Param(nm, dtype, vtype, dflt))
            if not self.accept_op(","):
                break
        return args

    def _parse_type(self):
        t = self.expect_id()
        if self.accept_op("["):
            vt = self.expect_id()
            self.expect_op("]")
            return normalize_dtype(t), normalize_vtype(vt)
        return "SCALAR", normalize_vtype(t)

    # -- expressions -------------------------------------------------------------
    def parse_expr(self, rbp=0) -> A.Expr:
        left = self.parse_prefix()
        while True:
            t = self.tok
            if t.kind != "OP" or t.value not in _BP:
                break
            op = t.value
            bp = _BP[op]
            if bp <= rbp:
                break
            self.i += 1
            p = A.Pos(t.line, t.col, self.filename)
            if op == "^":
                right = self.parse_expr(bp - 1)   # right associative
            else:
                right = self.parse_expr(bp)
            left = A.BinOp(_norm_binop(op), left, right, pos=p)
        return left

    def parse_prefix(self) -> A.Expr:
        t = self.tok
        p = self.pos()
        if t.kind == "OP" and t.value in ("-", "+"):
            self.i += 1
            operand = self.parse_expr(_UNARY_BP)
            if t.value == "-" and isinstance(operand, A.Literal) and operand.vtype in ("INT", "DOUBLE"):
                return A.Literal(-operand.value, operand.vtype, pos=p)
            return A.UnOp(t.value, operand, pos=p)
        if t.kind == "OP" and t.value == "!":
            self.i += 1
            return A.UnOp("!", self.parse_expr(_NOT_BP), pos=p)
        return self.parse_primary()

    def parse_primary(self) -> A.Expr:
        t = self.tok
        p = self.pos()
        k = t.kind
        if k == "INT":
            self.i += 1
            return A.Literal(t.value, "INT", pos=p)
        if k == "DOUBLE":
            self.i += 1
            return A.Literal(t.value, "DOUBLE", pos=p)
        if k == "STRING":
            self.i += 1
            return A.Literal(t.value, "STRING", pos=p)
        if k == "CMD":
            self.i += 1
            return A.CmdParam(t.value, pos=p)
        if k == "OP" and t.value == "(":
            self.i += 1
            e = self.parse_expr()
            self.expect_op(")")
            return e
        if k == "OP" and t.value == "[":
            self.i += 1
            items = [self.parse_expr()]
            while self.accept_op(","):
                items.append(self.parse_expr())
            self.expect_op("]")
            return A.ExprList(items, pos=p)
        if k == "ID":
            v = t.value
            if v in ("TRUE", "FALSE"):
                self.i += 1
                return A.Literal(v == "TRUE", "BOOLEAN", pos=p)
            self.i += 1
            if self.is_op("("):
                return self._parse_call(v, p)
            if self.is_op("[") and self.tok.line == t.line:
                # an index bracket on a following line starts a new multi-assignment
                # statement ([a, b] = f(..)) rather than indexing this identifier
                return self._parse_index(v, p)
            return A.Ident(v, pos=p)
        self.error("unexpected token in expression")

    def _parse_call(self, name, p):
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
        ns = None
        if "::" in name:
            ns, name = name.split("::", 1)
        return A.Call(name, args, namespace=ns, pos=p)


def _norm_binop(op):
    return {"&&": "&", "||": "|"}.get(op, op)


def normalize_dtype(t):
    t = t.lower()
    return {"matrix": "MATRIX", "frame": "FRAME", "scalar": "SCALAR", "list": "LIST"}.get(t, t.upper())


def normalize_vtype(t):
    t = t.lower()
    return {"int": "INT", "integer": "INT", "double": "DOUBLE", "float": "DOUBLE",
            "string": "STRING", "str": "STRING", "boolean": "BOOLEAN", "bool": "BOOLEAN",
            "unknown": "UNKNOWN"}.get(t, "UNKNOWN")


def parse_dml(src: str, filename: str = "") -> A.Program:
    return DMLParser(src, filename).parse()


def parse_dml_file(path: str) -> A.Program:
    with open(path, "r") as f:
        return parse_dml(f.read(), filename=os.path.abspath(path))
