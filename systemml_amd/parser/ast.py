"""AST node types for DML / PyDML programs.

Mirrors the statement/expression taxonomy of the reference parser
(reference: src/main/java/org/apache/sysml/parser/{Statement,Expression,
AssignmentStatement,IfStatement,ForStatement,WhileStatement,FunctionStatement,
BinaryExpression,BuiltinFunctionExpression,...}.java) but as light-weight
Python dataclasses: the compiler (systemml_amd.compiler) consumes these
directly to build HOP DAGs.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple, Any


@dataclass
class Pos:
    line: int = 0
    col: int = 0
    file: str = ""

    def __str__(self):
        return f"{self.file or '<script>'} line {self.line}:{self.col}"


# ----------------------------------------------------------------------------
# Expressions
# ----------------------------------------------------------------------------
class Expr:
    pos: Pos


@dataclass
class Literal(Expr):
    value: Any
    vtype: str  # 'INT' | 'DOUBLE' | 'BOOLEAN' | 'STRING'
    pos: Pos = field(default_factory=Pos)


@dataclass
class Ident(Expr):
    name: str
    pos: Pos = field(default_factory=Pos)


@dataclass
class CmdParam(Expr):
    """$name or $1 command line parameter reference (unresolved)."""
    name: str
    pos: Pos = field(default_factory=Pos)


@dataclass
class IndexRange:
    """One dimension of an index expression. lower None => all; upper None => single index."""
    lower: Optional[Expr] = None
    upper: Optional[Expr] = None
    is_range: bool = False   # True when 'a:b' syntax used


@dataclass
class Indexed(Expr):
    name: str
    rows: IndexRange
    cols: Optional[IndexRange]  # None when no comma given (X[i] form)
    pos: Pos = field(default_factory=Pos)


@dataclass
class BinOp(Expr):
    op: str
    left: Expr
    right: Expr
    pos: Pos = field(default_factory=Pos)


@dataclass
class UnOp(Expr):
    op: str   # '-', '+', '!'
    operand: Expr
    pos: Pos = field(default_factory=Pos)


@dataclass
class Arg:
    name: Optional[str]
    value: Expr


@dataclass
class Call(Expr):
    name: str
    args: List[Arg]
    namespace: Optional[str] = None
    pos: Pos = field(default_factory=Pos)


@dataclass
class ExprList(Expr):
    """[a, b, c] list of expressions (used for multi-assignment targets)."""
    items: List[Expr]
    pos: Pos = field(default_factory=Pos)


# ----------------------------------------------------------------------------
# Statements
# ----------------------------------------------------------------------------
class Stmt:
    pos: Pos


@dataclass
class Assign(Stmt):
    target: Expr            # Ident or Indexed
    value: Expr
    accumulate: bool = False   # '+='
    ifdef: Optional[CmdParam] = None   # x = ifdef($p, default)
    pos: Pos = field(default_factory=Pos)


@dataclass
class MultiAssign(Stmt):
    targets: List[Expr]
    value: Call
    pos: Pos = field(default_factory=Pos)


@dataclass
class ExprStmt(Stmt):
    """A call used as a statement (print, write, stop, user function without outputs)."""
    call: Call
    pos: Pos = field(default_factory=Pos)


@dataclass
class If(Stmt):
    pred: Expr
    then_body: List[Stmt]
    else_body: List[Stmt]
    pos: Pos = field(default_factory=Pos)


@dataclass
class For(Stmt):
    var: str
    start: Expr
    end: Expr
    incr: Optional[Expr]
    body: List[Stmt]
    parfor: bool = False
    params: dict = field(default_factory=dict)
    pos: Pos = field(default_factory=Pos)


@dataclass
class While(Stmt):
    pred: Expr
    body: List[Stmt]
    pos: Pos = field(default_factory=Pos)


@dataclass
class Param:
    name: str
    dtype: str    # 'MATRIX' | 'SCALAR' | 'FRAME' | 'LIST'
    vtype: str    # 'DOUBLE' | 'INT' | 'BOOLEAN' | 'STRING' | 'UNKNOWN'
    default: Optional[Expr] = None


@dataclass
class FunctionDef(Stmt):
    name: str
    inputs: List[Param]
    outputs: List[Param]
    body: List[Stmt]
    external: bool = False
    ext_params: dict = field(default_factory=dict)
    namespace: str = ".defaultNS"
    pos: Pos = field(default_factory=Pos)


@dataclass
class Import(Stmt):
    path: str
    namespace: str
    pos: Pos = field(default_factory=Pos)


@dataclass
class SetWd(Stmt):
    path: str
    pos: Pos = field(default_factory=Pos)


@dataclass
class Program:
    statements: List[Stmt]
    functions: dict            # name -> FunctionDef  (default namespace)
    imports: List[Import]
    namespaces: dict = field(default_factory=dict)  # ns -> {name: FunctionDef}
    source_path: str = ""
