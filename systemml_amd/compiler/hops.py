"""High-level operator (HOP) DAG.

A HOP DAG is built per basic statement block (reference:
src/main/java/org/apache/sysml/hops/Hop.java and subclasses; construction in
parser/DMLTranslator.java:constructHops).  Instead of ~20 Java subclasses we
use one node type with an ``op`` discriminator:

  lit      literal scalar                          (LiteralOp)
  tread    transient read of a variable            (DataOp TRANSIENTREAD)
  b        binary cellwise / scalar op             (BinaryOp)
  u        unary cellwise / scalar op              (UnaryOp)
  agg      unary aggregate (sum/min/…; all/row/col) (AggUnaryOp)
  mm       matrix multiply, optional transA        (AggBinaryOp)
  tsmm     t(X)%*%X / X%*%t(X)                     (AggBinaryOp → MMTSJ lop)
  mmchain  t(X)%*%(w*(X%*%v)) family + row-fused   (AggBinaryOp → MapMultChain / codegen Row)
  tak      sum(X*Y) / sum(X*Y*Z)                   (AggUnaryOp → TernaryAggregate)
  t        transpose                               (ReorgOp)
  rix/lix  right / left indexing                   (IndexingOp / LeftIndexingOp)
  bi       any other builtin, dispatched by name   (Unary/Binary/Ternary/Nary/ParameterizedBuiltin/DataGen/Convolution ops)
  fcall    user function call (multi-output)       (FunctionOp)
  fout     i-th output of an fcall
  sink     side-effecting builtin (print/write/stop/assert)

Sizes are propagated where statically known (dim1/dim2, -1 = unknown) and used
by rewrites (e.g. mmchain requires a vector) and the memory estimator.
"""
from __future__ import annotations

import itertools

_ids = itertools.count(1)

# builtins that must never be merged by CSE or constant folded (non-deterministic / side effects)
NONDETERMINISTIC = {"rand", "sample", "time", "read"}
SIDE_EFFECT = {"print", "write", "stop", "assert", "printf"}


class Hop:
    __slots__ = ("id", "op", "inputs", "p", "dim1", "dim2", "dt", "parents", "slot",
                 "named", "pos", "exec_type", "phys")

    def __init__(self, op, inputs=(), p=None, named=None, dt="U", dim1=-1, dim2=-1, pos=None):
        self.id = next(_ids)
        self.op = op
        self.inputs = list(inputs)
        self.p = p if p is not None else {}
        self.named = named or []      # names for trailing named args of 'bi' hops
        self.dt = dt                  # 'M','S','F','L','U'
        self.dim1 = dim1
        self.dim2 = dim2
        self.parents = []
        self.slot = -1
        self.pos = pos
        self.exec_type = None         # CP | GPU | DIST (compiler/cost.py); None: decided at run time
        self.phys = None              # physical operator of matrix products (cost.physical_op)

    # convenience
    @property
    def is_lit(self):
        return self.op == "lit"

    @property
    def value(self):
        return self.p.get("v")

    def key(self):
        """Structural key for common-subexpression elimination."""
        pk = tuple(sorted((k, _hashable(v)) for k, v in self.p.items()))
        return (self.op, pk, tuple(self.named), tuple(h.id for h in self.inputs))

    def __repr__(self):
        extra = ""
        if self.op == "lit":
            extra = repr(self.value)
        elif self.op in ("tread", "twrite"):
            extra = self.p["name"]
        elif "o" in self.p:
            extra = str(self.p["o"])
        elif "name" in self.p:
            extra = self.p["name"]
        return f"({self.id}) {self.op}{'(' + extra + ')' if extra else ''} [{','.join(str(h.id) for h in self.inputs)}] {self.dt}[{self.dim1}x{self.dim2}]"


def _hashable(v):
    if isinstance(v, list):
        return tuple(_hashable(x) for x in v)
    if isinstance(v, dict):
        return tuple(sorted((k, _hashable(x)) for k, x in v.items()))
    if isinstance(v, float) and v != v:
        return "NaN"
    return v


def lit(v, pos=None):
    if isinstance(v, bool):
        vt = "BOOLEAN"
    elif isinstance(v, int):
        vt = "INT"
    elif isinstance(v, float):
        vt = "DOUBLE"
    else:
        vt = "STRING"
    return Hop("lit", p={"v": v, "vt": vt}, dt="S", dim1=0, dim2=0, pos=pos)


def walk(roots):
    """Post-order traversal (each hop once)."""
    seen = set()
    out = []
    stack = [(r, False) for r in reversed(roots)]
    while stack:
        h, done = stack.pop()
        if done:
            out.append(h)
            continue
        if h.id in seen:
            continue
        seen.add(h.id)
        stack.append((h, True))
        for c in reversed(h.inputs):
            if c.id not in seen:
                stack.append((c, False))
    return out


def explain_dag(roots, indent=""):
    lines = []
    for h in walk(roots):
        et = f" {h.exec_type}" if h.exec_type else (" (exec type at run time)" if h.dt == "M" and
                                                     h.op not in ("lit", "tread") else "")
        if getattr(h, "phys", None):
            et += f" {h.phys}"
        if h.dt == "M" and h.dim1 >= 0 and h.dim2 >= 0:
            mb = h.dim1 * h.dim2 * 8 / 1e6
            et += f" [{mb:.3g}MB]"
        lines.append(f"{indent}{h!r}{et}")
    return "\n".join(lines)
