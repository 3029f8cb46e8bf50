"""JMLC — embedded, low-latency scoring API (reference: api/jmlc/{Connection,
PreparedScript,ResultVariables,JMLCUtils}.java).

A script is compiled once (`Connection.prepareScript`) and executed many times
with different in-memory inputs; no file IO is performed for bound inputs and
outputs (persistent reads/writes of bound variables are removed at compile
time, as in the reference).

    conn = Connection()
    ps = conn.prepareScript(script_text, args={"$reg": 0.1}, inputs=["X", "W"], outputs=["Y"])
    ps.setMatrix("X", X); ps.setMatrix("W", W, reuse=True)
    Y = ps.executeScript().getMatrix("Y")
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..conf import DMLConfig, get_default_config
from ..runtime.data import FrameBlock
from . import executor as EX


class ResultVariables:
    def __init__(self, values):
        self._v = values

    def getMatrix(self, name):
        v = self._v[name]
        from ..ops import core as C
        if C.is_dist(v):
            v = C._dist().gather(v)
        if isinstance(v, torch.Tensor):
            return v.detach().to("cpu", torch.float64).numpy()
        raise TypeError(f"{name} is not a matrix")

    def getFrame(self, name):
        v = self._v[name]
        if not isinstance(v, FrameBlock):
            raise TypeError(f"{name} is not a frame")
        return [v.row(i) for i in range(v.nrow())]

    def getDouble(self, name):
        return float(self._v[name])

    def getLong(self, name):
        return int(self._v[name])

    def getString(self, name):
        from ..runtime import scalars as S
        return S.to_str(self._v[name])

    def getBoolean(self, name):
        return bool(self._v[name])

    def getVariableNames(self):
        return list(self._v.keys())

    def size(self):
        return len(self._v)


class PreparedScript:
    def __init__(self, compiled, inputs, outputs):
        self._cs = compiled
        self._input_names = list(inputs)
        self._outputs = list(outputs)
        self._bound = {}
        self._reuse = set()

    def _check(self, name):
        if name not in self._input_names:
            raise ValueError(f"'{name}' is not a declared input of this prepared script")

    def setMatrix(self, name, value, reuse=False):
        self._check(name)
        self._bound[name] = EX.convert_input(np.asarray(value, dtype=np.float64)
                                             if not isinstance(value, torch.Tensor) else value)
        if reuse:
            self._reuse.add(name)

    def setFrame(self, name, rows, reuse=False, schema=None, colnames=None):
        self._check(name)
        ncol = len(rows[0]) if rows else 0
        cols = [[r[j] for r in rows] for j in range(ncol)]
        self._bound[name] = FrameBlock(cols, schema, colnames)
        if reuse:
            self._reuse.add(name)

    def setScalar(self, name, value, reuse=False):
        self._check(name)
        self._bound[name] = value
        if reuse:
            self._reuse.add(name)

    def clearParameters(self):
        self._bound = {k: v for k, v in self._bound.items() if k in self._reuse}

    def executeScript(self):
        missing = [n for n in self._input_names if n not in self._bound]
        if missing:
            raise ValueError(f"unbound inputs: {missing}")
        values, _ = EX.execute(self._cs, dict(self._bound))
        self.clearParameters()
        return ResultVariables(values)


class Connection:
    def __init__(self, config: DMLConfig = None):
        self.config = (config or get_default_config()).copy()

    def readScript(self, path):
        with open(path) as f:
            return f.read()

    def prepareScript(self, script, args=None, inputs=(), outputs=(), parsePyDML=False):
        args = {k.lstrip("$"): v for k, v in (args or {}).items()}
        # placeholder input values let the compiler infer data types (matrix unless declared scalar)
        cs = EX.compile_script(script, args, inputs=list(inputs), outputs=list(outputs), config=self.config,
                               pydml=parsePyDML)
        return PreparedScript(cs, inputs, outputs)

    def convertToDoubleMatrix(self, text, rows, cols):
        vals = [float(t) for t in text.replace(",", " ").split()]
        return np.asarray(vals, dtype=np.float64).reshape(rows, cols)

    def close(self):
        pass
