"""Lazily evaluated, numpy-like matrix API that generates DML (reference:
src/main/python/systemml/defmatrix.py).

    import systemml_amd.api.defmatrix as sml
    m1 = sml.matrix(np.ones((3, 3)) + 2)
    m2 = (m1 @ m1.t() + 1).sum(axis=1)
    m2.toNumPy()                  # builds one DML program for the whole DAG and runs it

Every operation creates a node holding a DML expression over its inputs; `eval()` (or any
conversion to numpy / pandas, printing, `save`) walks the DAG once, emits one statement per
node, binds the numpy / torch leaves as in-memory inputs and executes the program on the
backend.  Results are cached in the nodes, so later expressions reuse them as inputs.
"""
from __future__ import annotations

import itertools

import numpy as np

_ids = itertools.count(1)
_lazy = True
_config = None


def set_lazy(is_lazy):
    global _lazy
    _lazy = bool(is_lazy)


def set_config(config):
    """DMLConfig for evaluation (default: the framework default, i.e. GPU when present)."""
    global _config
    _config = config


def _name():
    return f"mVar{next(_ids)}"


def _lit(v):
    if isinstance(v, bool):
        return "TRUE" if v else "FALSE"
    if isinstance(v, (int, float, np.integer, np.floating)):
        return repr(float(v))
    if isinstance(v, str):
        return '"' + v.replace('"', '\\"') + '"'
    raise TypeError(f"unsupported scalar {type(v).__name__}")


class matrix:
    """A lazily evaluated matrix: either data (numpy / torch / scipy / pandas) or a DML op."""

    def __init__(self, data=None, op=None, inputs=(), shape=None):
        self.name = _name()
        self.op = op                       # DML expression with {0}, {1}, ... placeholders
        self.inputs = list(inputs)
        self.data = None
        self.scalar = False
        self._shape = shape
        if op is None:
            d = data
            if hasattr(d, "to_numpy"):
                d = d.to_numpy()
            if not (hasattr(d, "toarray") or hasattr(d, "detach")):
                d = np.asarray(d, dtype=np.float64)
                if d.ndim == 1:
                    d = d.reshape(-1, 1)
            self.data = d
            self._shape = tuple(d.shape)
        elif not _lazy:
            self.eval()

    # ------------------------------------------------------------------ evaluation
    def _dml(self, order, seen):
        if self.name in seen:
            return
        seen.add(self.name)
        for x in self.inputs:
            if isinstance(x, matrix):
                x._dml(order, seen)
        order.append(self)

    def eval(self):
        if self.data is not None:
            return self
        from .executor import run
        order = []
        self._dml(order, set())
        lines, inputs = [], {}
        for node in order:
            if node.data is not None:
                inputs[node.name] = node.data
                continue
            args = [x.name if isinstance(x, matrix) else _lit(x) for x in node.inputs]
            lines.append(f"{node.name} = " + node.op.format(*args))
        res = run("\n".join(lines), inputs=inputs, outputs=[self.name], config=_config)
        v = res[self.name]
        if hasattr(v, "detach"):
            if getattr(v, "layout", None) is not None and "sparse" in str(v.layout):
                v = v.to_dense()
            v = v.detach().double().cpu().numpy()
        elif hasattr(v, "decompress"):
            v = v.decompress().double().cpu().numpy()
        self.data = v
        self.scalar = not isinstance(v, np.ndarray)
        return self

    def toNumPy(self):
        self.eval()
        return np.asarray(self.data) if not self.scalar else self.data

    def toPandas(self):
        import pandas as pd
        return pd.DataFrame(self.toNumPy())

    def __array__(self, dtype=None, copy=None):
        a = np.asarray(self.toNumPy(), dtype=np.float64)
        return a.astype(dtype) if dtype is not None else a

    def __float__(self):
        return float(self.toNumPy())

    def save(self, file, format="csv"):
        from ..io.writers import write_matrix
        import torch
        write_matrix(torch.as_tensor(np.atleast_2d(self.toNumPy())), file, format)

    def __repr__(self):
        if self.data is None:
            return f"<systemml_amd.defmatrix.matrix lazy: {self.op}>"
        return f"matrix(\n{self.data!r})"

    def print_ast(self):
        lines = []

        def rec(n, d):
            lines.append("  " * d + (n.op or f"data{n._shape}"))
            for x in n.inputs:
                if isinstance(x, matrix):
                    rec(x, d + 1)
                else:
                    lines.append("  " * (d + 1) + repr(x))
        rec(self, 0)
        s = "\n".join(lines)
        print(s)
        return s

    # ------------------------------------------------------------------ shape
    @property
    def shape(self):
        if self._shape is None:
            self.eval()
            self._shape = np.shape(self.data)
        return self._shape

    def get_shape(self):
        return self.shape

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _op(op, *inputs, shape=None):
        ins = [x if isinstance(x, (matrix, bool, int, float, str, np.integer, np.floating)) else matrix(x)
               for x in inputs]
        return matrix(op=op, inputs=ins, shape=shape)

    def _bin(self, other, o, rev=False):
        if rev:
            return matrix._op("{0} " + o + " {1}", other, self)
        return matrix._op("{0} " + o + " {1}", self, other)

    def _fn(self, fn):
        return matrix._op(fn + "({0})", self, shape=self._shape)

    # arithmetic
    def __add__(self, o): return self._bin(o, "+")
    def __sub__(self, o): return self._bin(o, "-")
    def __mul__(self, o): return self._bin(o, "*")
    def __truediv__(self, o): return self._bin(o, "/")
    __div__ = __truediv__
    def __floordiv__(self, o): return self._bin(o, "%/%")
    def __mod__(self, o): return self._bin(o, "%%")
    def __pow__(self, o): return self._bin(o, "^")
    def __radd__(self, o): return self._bin(o, "+", True)
    def __rsub__(self, o): return self._bin(o, "-", True)
    def __rmul__(self, o): return self._bin(o, "*", True)
    def __rtruediv__(self, o): return self._bin(o, "/", True)
    __rdiv__ = __rtruediv__
    def __rfloordiv__(self, o): return self._bin(o, "%/%", True)
    def __rmod__(self, o): return self._bin(o, "%%", True)
    def __rpow__(self, o): return self._bin(o, "^", True)
    def __neg__(self): return matrix._op("-{0}", self, shape=self._shape)
    negative = __neg__
    def __lt__(self, o): return self._bin(o, "<")
    def __le__(self, o): return self._bin(o, "<=")
    def __gt__(self, o): return self._bin(o, ">")
    def __ge__(self, o): return self._bin(o, ">=")
    def __eq__(self, o): return self._bin(o, "==")
    def __ne__(self, o): return self._bin(o, "!=")
    def __and__(self, o): return self._bin(o, "&")
    def __or__(self, o): return self._bin(o, "|")
    __hash__ = object.__hash__
    def logical_not(self): return matrix._op("!{0}", self, shape=self._shape)

    def dot(self, other):
        return matrix._op("{0} %*% {1}", self, other)
    __matmul__ = dot

    def __rmatmul__(self, other):
        return matrix._op("{0} %*% {1}", other, self)

    def transpose(self):
        return matrix._op("t({0})", self)
    t = transpose

    @property
    def T(self):
        return self.transpose()

    # element-wise functions
    def exp(self): return self._fn("exp")
    def log(self, y=None):
        return self._fn("log") if y is None else matrix._op("log({0}, {1})", self, y)
    def log1p(self): return matrix._op("log(1 + {0})", self, shape=self._shape)
    def expm1(self): return matrix._op("exp({0}) - 1", self, shape=self._shape)
    def exp2(self): return matrix._op("2 ^ {0}", self, shape=self._shape)
    def log2(self): return matrix._op("log({0}, 2)", self, shape=self._shape)
    def log10(self): return matrix._op("log({0}, 10)", self, shape=self._shape)
    def square(self): return matrix._op("{0} ^ 2", self, shape=self._shape)
    def reciprocal(self): return matrix._op("1 / {0}", self, shape=self._shape)
    def abs(self): return self._fn("abs")
    def sqrt(self): return self._fn("sqrt")
    def round(self): return self._fn("round")
    def floor(self): return self._fn("floor")
    def ceil(self): return self._fn("ceil")
    ceiling = ceil
    def sin(self): return self._fn("sin")
    def cos(self): return self._fn("cos")
    def tan(self): return self._fn("tan")
    def sinh(self): return self._fn("sinh")
    def cosh(self): return self._fn("cosh")
    def tanh(self): return self._fn("tanh")
    def arcsin(self): return self._fn("asin")
    def arccos(self): return self._fn("acos")
    def arctan(self): return self._fn("atan")
    def sign(self): return self._fn("sign")
    def deg2rad(self): return matrix._op("{0} * 3.141592653589793 / 180", self, shape=self._shape)
    def rad2deg(self): return matrix._op("{0} * 180 / 3.141592653589793", self, shape=self._shape)
    def cumsum(self, axis=0): return self._fn("cumsum")
    def ones_like(self): return matrix._op("({0} * 0) + 1", self, shape=self._shape)
    def zeros_like(self): return matrix._op("{0} * 0", self, shape=self._shape)
    def remainder(self, o): return self._bin(o, "%%")
    mod = remainder

    def logaddexp(self, o):
        return matrix._op("log(exp({0}) + exp({1}))", self, o)

    def logaddexp2(self, o):
        return matrix._op("log(2 ^ {0} + 2 ^ {1}, 2)", self, o)

    def ldexp(self, o):
        return matrix._op("{0} * 2 ^ {1}", self, o)

    def hstack(self, other):
        return matrix._op("cbind({0}, {1})", self, other)

    def vstack(self, other):
        return matrix._op("rbind({0}, {1})", self, other)

    # aggregates
    def _agg(self, full, row, col, axis):
        if axis is None:
            return matrix._op(full + "({0})", self)
        return matrix._op((row if axis == 1 else col) + "({0})", self)

    def sum(self, axis=None): return self._agg("sum", "rowSums", "colSums", axis)
    def mean(self, axis=None): return self._agg("mean", "rowMeans", "colMeans", axis)
    def max(self, other=None, axis=None):
        if other is not None:
            return matrix._op("max({0}, {1})", self, other)
        return self._agg("max", "rowMaxs", "colMaxs", axis)
    def min(self, other=None, axis=None):
        if other is not None:
            return matrix._op("min({0}, {1})", self, other)
        return self._agg("min", "rowMins", "colMins", axis)
    def var(self, axis=None): return self._agg("var", "rowVars", "colVars", axis)
    def sd(self, axis=None): return self._agg("sd", "rowSds", "colSds", axis)
    std = sd
    def prod(self): return matrix._op("prod({0})", self)
    def trace(self): return matrix._op("trace({0})", self)

    def argmax(self, axis=1):
        if axis != 1:
            return matrix._op("t(rowIndexMax(t({0})))", self)
        return matrix._op("rowIndexMax({0})", self)

    def argmin(self, axis=1):
        if axis != 1:
            return matrix._op("t(rowIndexMin(t({0})))", self)
        return matrix._op("rowIndexMin({0})", self)

    def moment(self, moment=1, axis=None):
        if axis is not None:
            raise ValueError("moment supports axis=None only")
        return matrix._op("moment({0}, " + str(int(moment)) + ")", self)

    def remove_empty(self, axis=None):
        margin = "rows" if axis in (None, 0) else "cols"
        return matrix._op('removeEmpty(target={0}, margin="' + margin + '")', self)

    def replace(self, pattern=0, replacement=0):
        return matrix._op("replace(target={0}, pattern={1}, replacement={2})", self, pattern, replacement)

    # indexing (numpy 0-based, exclusive stops -> DML 1-based inclusive)
    @staticmethod
    def _idx(ix):
        if isinstance(ix, slice):
            if ix.step not in (None, 1):
                raise ValueError("slice steps are not supported")
            lo = "" if ix.start is None else str(ix.start + 1)
            hi = "" if ix.stop is None else str(ix.stop)
            return f"{lo}:{hi}" if (lo or hi) else ""
        if isinstance(ix, (int, np.integer)):
            return str(int(ix) + 1)
        raise ValueError("only integers and slices are supported as indices")

    def __getitem__(self, key):
        if not isinstance(key, tuple):
            key = (key, slice(None))
        r, c = (self._idx(k) for k in key)
        return matrix._op("{0}[" + r + ", " + c + "]", self)

    def __setitem__(self, key, value):
        """In-place left indexing: evaluates this matrix, then applies A[r, c] = value."""
        if not isinstance(key, tuple):
            key = (key, slice(None))
        r, c = (self._idx(k) for k in key)
        from .executor import run
        ins = {"A": np.atleast_2d(self.toNumPy()).copy()}
        if isinstance(value, (matrix, np.ndarray, list)):
            ins["v"] = value.toNumPy() if isinstance(value, matrix) else np.atleast_2d(np.asarray(value, float))
            vsrc = "v"
        else:
            vsrc = _lit(value)
        res = run(f"A[{r}, {c}] = {vsrc}", inputs=ins, outputs=["A"], config=_config)
        a = res["A"]
        self.data = a.detach().double().cpu().numpy() if hasattr(a, "detach") else a
        self.op, self.inputs, self.scalar = None, [], False


# ---------------------------------------------------------------------- constructors
def full(shape, fill_value):
    return matrix._op(f"matrix({float(fill_value)!r}, rows={int(shape[0])}, cols={int(shape[1])})", shape=tuple(shape))


def zeros(shape):
    return full(shape, 0)


def ones(shape):
    return full(shape, 1)


def seq(start=None, stop=None, step=1):
    """Column vector start, start + step, ..., stop -- stop INCLUDED, as DML's seq and the
    reference's python/systemml/defmatrix.py seq (seq(3) is 0, 1, 2, 3)."""
    if start is None and stop is None:
        raise ValueError("Both start and stop cannot be None")
    if start is not None and stop is None:
        start, stop = 0, start
    start = 0 if start is None else start
    return matrix._op(f"seq({start!r}, {stop!r}, {step!r})")


def rand(rows, cols, min=0.0, max=1.0, pdf="uniform", sparsity=1.0, seed=-1):
    return matrix._op(f'rand(rows={int(rows)}, cols={int(cols)}, min={min!r}, max={max!r}, pdf="{pdf}", '
                      f"sparsity={sparsity!r}, seed={int(seed)})", shape=(rows, cols))


def load(file, format="csv"):
    return matrix._op(f'read("{file}", format="{format}")')


def solve(A, b):
    return matrix._op("solve({0}, {1})", A, b)


def hstack(a, b):
    return matrix._op("cbind({0}, {1})", a, b)


def vstack(a, b):
    return matrix._op("rbind({0}, {1})", a, b)


def eval(outputs, execute=True):
    outs = outputs if isinstance(outputs, (list, tuple)) else [outputs]
    for o in outs:
        o.eval()
    return outputs


def reset():
    """Drop nothing: results are cached per node and leaves are plain data."""
    return None
