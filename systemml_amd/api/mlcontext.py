"""MLContext programmatic API (reference: api/mlcontext/{MLContext,Script,ScriptFactory,
MLResults,Matrix,Frame,MatrixMetadata}.java and src/main/python/systemml/mlcontext.py).

    from systemml_amd import MLContext, dml
    ml = MLContext()
    script = dml("y = X %*% w").input(X=np.ones((3, 2)), w=np.ones((2, 1))).output("y")
    y = ml.execute(script).get("y").toNumPy()

Inputs accept numpy arrays, torch tensors (host or HBM), pandas DataFrames,
scipy sparse matrices, Python scalars/strings, FrameBlock / ListObject and
row-partitioned DistMatrix objects.  Outputs come back as `Matrix` / `Frame`
wrappers (lazy device→host conversion) or Python scalars.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..conf import DMLConfig, get_default_config
from ..runtime.data import FrameBlock, ListObject
from ..utils.stats import Statistics
from . import executor as EX

SCRIPTS_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts")


class Matrix:
    """Result matrix handle (reference: api/mlcontext/Matrix.java)."""

    def __init__(self, value):
        self._v = value

    def _tensor(self):
        from ..ops import core as C
        v = self._v
        if C.is_dist(v):
            v = C._dist().gather(v)
        return v

    def toNumPy(self):
        return self._tensor().detach().to("cpu", torch.float64).numpy()

    def toTorch(self):
        return self._tensor()

    def toDF(self):
        """pandas DataFrame in the reference's layout: an __INDEX column (1-based row ids) then
        C1..Cn (reference MLContextConversionUtil.matrixObjectToDataFrame)."""
        import pandas as pd
        a = self.toNumPy()
        df = pd.DataFrame(a, columns=[f"C{i + 1}" for i in range(a.shape[1])])
        df.insert(0, "__INDEX", np.arange(1, a.shape[0] + 1, dtype=np.float64))
        return df

    @property
    def shape(self):
        return tuple(self._v.shape)

    def __repr__(self):
        return "Matrix"          # reference python/systemml/mlcontext.py Matrix.__repr__


class Frame:
    def __init__(self, fb: FrameBlock):
        self._f = fb

    def toDF(self):
        import pandas as pd
        return pd.DataFrame({n: c for n, c in zip(self._f.names, self._f.columns)})

    def toFrameBlock(self):
        return self._f

    @property
    def shape(self):
        return self._f.shape


def _wrap(v):
    if isinstance(v, torch.Tensor):
        return Matrix(v)
    from ..ops import core as C
    if C.is_dist(v):
        return Matrix(v)
    if isinstance(v, FrameBlock):
        return Frame(v)
    return v


class MLResults:
    def __init__(self, values, stats=None):
        self._values = values
        self.stats = stats

    def get(self, *names):
        """One value, or a list of values for several names (reference MLResults.get)."""
        out = [_wrap(self._values[n]) for n in names]
        return out[0] if len(out) == 1 else out

    def getNumPyArray(self, name):
        return self.get(name).toNumPy()

    def getMatrix(self, name):
        return self.get(name)

    def getScalar(self, name):
        return self._values[name]

    def getDouble(self, name):
        return float(self._values[name])

    def getLong(self, name):
        return int(self._values[name])

    def getString(self, name):
        from ..runtime import scalars as S
        return S.to_str(self._values[name])

    def getBoolean(self, name):
        return bool(self._values[name])

    def getFrame(self, name):
        """The output frame as a Frame (MLResults.java:486)."""
        v = self._values[name]
        if not isinstance(v, FrameBlock):
            raise TypeError(f"output '{name}' is not a frame")
        return Frame(v)

    def getFrameAs2DStringArray(self, name):
        from .jmlc import frame_to_strings
        return frame_to_strings(self.getFrame(name).toFrameBlock())

    def getMatrixAs2DDoubleArray(self, name):
        return self.get(name).toNumPy()

    def getDataFrame(self, name):
        """The output matrix (or frame) as a pandas DataFrame (MLResults.java:287)."""
        return self.get(name).toDF()

    def getTuple(self, *names):
        """The named outputs as one tuple, each converted like get() -- matrices as Matrix,
        frames as Frame, scalars as Python values (MLResults.java:607-1990, Tuple1..Tuple22)."""
        if not 1 <= len(names) <= 22:
            raise ValueError("getTuple takes 1 to 22 output names")
        return tuple(self._get1(n) for n in names)

    def _get1(self, name):
        if name not in self._values:
            raise KeyError(f"Variable '{name}' not present")
        v = self._values[name]
        from ..runtime import scalars as S
        if type(v) is S.DevScalar:
            v = v.value()
        return _wrap(v)

    def getScript(self):
        return getattr(self, "script", None)

    def keys(self):
        return list(self._values.keys())

    def __getitem__(self, name):
        return self.get(name)

    def __repr__(self):
        return "MLResults: " + ", ".join(f"{k} ({type(_wrap(v)).__name__})" for k, v in self._values.items())


class Script:
    def __init__(self, source, pydml=False, filename=""):
        self.source = source
        self.pydml = pydml
        self.filename = filename
        self._inputs = {}
        self._outputs = []
        self._args = {}

    def input(self, *args, **kw):
        if args:
            if len(args) != 2:
                raise ValueError("input(name, value) or input(name=value)")
            kw = {args[0]: args[1]}
        for k, v in kw.items():
            if k.startswith("$"):
                self._args[k[1:]] = v
            else:
                self._inputs[k] = v
        return self

    def output(self, *names):
        self._outputs.extend(names)
        return self

    def args(self, **kw):
        self._args.update({k: (v if isinstance(v, str) else v) for k, v in kw.items()})
        return self

    def setName(self, name):
        self.filename = name
        return self

    def clearAll(self):
        self._inputs.clear()
        self._outputs.clear()
        self._args.clear()
        return self


def dml(source):
    return Script(source)


def pydml(source):
    return Script(source, pydml=True)


def dmlFromFile(path):
    with open(path) as f:
        return Script(f.read(), filename=os.path.abspath(path))


def pydmlFromFile(path):
    with open(path) as f:
        return Script(f.read(), pydml=True, filename=os.path.abspath(path))


def pydmlFromResource(rel):
    path = os.path.join(SCRIPTS_DIR, rel)
    return pydmlFromFile(path)


def getHopDAG(ml, script, lines=None, conf=None, apply_rewrites=True, with_subgraph=False):
    """Graphviz DOT text of the script's HOP DAGs (reference: mlcontext.getHopDAG, which
    renders through the JVM).  `lines` restricts the output to basic blocks starting on
    those script lines; `apply_rewrites=False` shows the DAGs before the HOP rewrites;
    `with_subgraph` draws one cluster per basic block."""
    from ..compiler.blocks import BasicBlock
    from ..compiler import hops as H
    cfg = (conf or (ml.config if ml is not None else get_default_config())).copy()
    cfg.rewrites = bool(apply_rewrites)
    cfg.fusion = bool(apply_rewrites)
    cs = EX.compile_script(script.source, script._args, inputs=script._inputs, outputs=script._outputs,
                           config=cfg, pydml=script.pydml, filename=script.filename)
    out = ["digraph HopDAG {", "  node [shape=box, fontname=Helvetica];"]
    seen = set()
    idx = [0]

    def emit(blocks):
        for b in blocks:
            if isinstance(b, BasicBlock):
                line = b.pos.line if b.pos else None
                if lines is not None and line not in lines:
                    continue
                roots = list(b.roots) + list(b.env_out.values())
                if with_subgraph:
                    out.append(f"  subgraph cluster_{idx[0]} {{ label=\"lines {line}\";")
                    idx[0] += 1
                for h in H.walk(roots):
                    if h.id in seen:
                        continue
                    seen.add(h.id)
                    label = repr(h).split(" [")[0].replace('"', "'")
                    et = f"\\n{h.exec_type}" if h.exec_type else ""
                    out.append(f'    h{h.id} [label="{label}{et}"];')
                    for c in h.inputs:
                        out.append(f"    h{c.id} -> h{h.id};")
                for name, h in b.env_out.items():
                    out.append(f'    v_{h.id}_{name} [label="{name}", shape=ellipse]; h{h.id} -> v_{h.id}_{name};')
                if with_subgraph:
                    out.append("  }")
            for attr in ("then_blocks", "else_blocks", "body"):
                if hasattr(b, attr):
                    emit(getattr(b, attr))
    emit(cs.cp.blocks)
    out.append("}")
    return "\n".join(out)


def dmlFromResource(rel):
    """Load one of the bundled scripts (systemml_amd/scripts/...)."""
    path = os.path.join(SCRIPTS_DIR, rel)
    return dmlFromFile(path)


class MLContext:
    def __init__(self, sc=None, config: DMLConfig = None):
        self.config = (config or get_default_config()).copy()
        self._stats = False
        self._explain = ""
        self._out = None
        self.last_stats = None

    # configuration (reference method names)
    def setStatistics(self, flag=True):
        self._stats = bool(flag)
        return self

    def setExplain(self, flag=True, level="hops"):
        self._explain = level if flag else ""
        return self

    def setExplainLevel(self, level):
        self._explain = level
        return self

    def setGPU(self, flag=True):
        self.config.gpu = bool(flag)
        return self

    def setForceGPU(self, flag=True):
        self.config.gpu = bool(flag)
        return self

    def setConfigProperty(self, key, value):
        self.config.set(key, value)
        return self

    def setConfig(self, path):
        self.config = DMLConfig.from_xml(path)
        return self

    def setOutput(self, fn):
        self._out = fn
        return self

    def execute(self, script: Script):
        cfg = self.config
        cfg.explain = self._explain
        stats = Statistics(enabled=self._stats) if self._stats else None
        cs = EX.compile_script(script.source, script._args, inputs=script._inputs,
                               outputs=script._outputs, config=cfg, pydml=script.pydml,
                               filename=script.filename)
        values, ctx = EX.execute(cs, script._inputs, out=self._out, stats=stats)
        if stats is not None:
            from ..ops import kernels
            for k, v in kernels.counters.items():
                stats.counters[k] = v
            ctx.print(stats.report(cfg.stats_count))
        self.last_stats = stats
        return MLResults(values, stats)

    def setStatisticsMaxHeavyHitters(self, n):
        """Number of heavy hitters in the statistics report (MLContext.java:622)."""
        self.config.stats_count = int(n)
        return self

    def getStatisticsMaxHeavyHitters(self):
        return self.config.stats_count

    def isStatistics(self):
        return self._stats

    def isExplain(self):
        return bool(self._explain)

    def getExplainLevel(self):
        return self._explain or None

    def isGPU(self):
        return bool(self.config.gpu)

    def isForceGPU(self):
        return bool(self.config.gpu)

    def resetConfig(self):
        """Back to the default configuration (MLContext.java:283)."""
        self.config = get_default_config().copy()
        return self

    def info(self):
        """Project information (MLContext.java:660 ProjectInfo): version, build and the
        native libraries / device this context runs on."""
        import torch as _t
        from ..ops import kernels
        d = {"Version": self.version(), "Main-Class": "systemml_amd", "Torch": _t.__version__,
             "HIP": getattr(_t.version, "hip", None), "GPU": _t.cuda.is_available(),
             "Native kernels": os.path.exists(kernels.LIB_PATH)}
        if _t.cuda.is_available():
            d["Device"] = _t.cuda.get_device_name(0)
        return MLContextInfo(d)

    def buildTime(self):
        from ..ops import kernels
        import time as _time
        p = kernels.LIB_PATH
        return _time.strftime("%Y-%m-%d %H:%M:%S", _time.localtime(os.path.getmtime(p))) if os.path.exists(p) \
            else None

    def close(self):
        pass

    def version(self):
        from .. import __version__
        return __version__


class MLContextInfo(dict):
    """ProjectInfo of MLContext.info(): a dict with the reference's `property()` accessor."""

    def property(self, key):
        return self.get(key)

    def __str__(self):
        return "\n".join(f"{k}: {v}" for k, v in self.items())
