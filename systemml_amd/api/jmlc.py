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

Besides scoring, the connection converts the reference's text formats into in-memory
matrices / frames (`convertToDoubleMatrix`, `convertToMatrix`, `convertToStringFrame`,
`convertToFrame`; textcell IJV is the default format, csv and mm by `format=` or the JSON
metadata string), reads files with their `.mtd` (`readDoubleMatrix`, `readStringFrame`) and
reads the legacy on-disk transform metadata of a directory or a package resource
(`readTransformMetaDataFromFile` / `readTransformMetaDataFromPath`, Connection.java:827-898)
into the frame `transformapply` / `transformdecode` take.  `PreparedScript.clone()` gives an
independent program and symbol table for concurrent scoring from threads
(PreparedScript.java:514).
"""
from __future__ import annotations

import io
import json
import logging
import os
import threading

import numpy as np
import torch

from ..conf import DMLConfig, get_default_config
from ..parser.errors import DMLRuntimeError
from ..runtime.data import FrameBlock
from . import executor as EX

log = logging.getLogger(__name__)

FORMATS = ("text", "mm", "csv")


class DMLException(RuntimeError):
    """Errors of the JMLC API (reference: api/DMLException)."""


# ----------------------------------------------------------------------------
# text parsing of matrices / frames from strings and streams
# ----------------------------------------------------------------------------
def _text_of(input):
    """A string, bytes or a readable (text or binary) stream -> str."""
    if isinstance(input, str):
        return input
    if isinstance(input, (bytes, bytearray)):
        return bytes(input).decode("utf-8")
    if hasattr(input, "read"):
        t = input.read()
        return t.decode("utf-8") if isinstance(t, (bytes, bytearray)) else t
    raise TypeError(f"expected a string or a stream, got {type(input).__name__}")


def _check_format(format):
    fmt = str(format).lower()
    if fmt not in FORMATS:
        raise IOError(f"Invalid input format (expected: csv, text or mm): {format}")
    return fmt


def split_csv(line, delim=","):
    """Tokens of one CSV line with RFC-4180 quoting, quotes kept in the token (reference
    IOUtilFunctions.splitCSV: "aa""a" and "a,b" stay one token, verbatim)."""
    if line == "":
        return [""]
    toks, pos, n, dl = [], 0, len(line), len(delim)
    while pos < n:
        if line[pos] == '"' and line.find('"', pos + 1) > 0:
            to = line.find('"', pos + 1)
            while to + 1 < n and line[to + 1] == '"':      # escaped inner quotes
                to = line.find('"', to + 2)
                if to < 0:
                    to = n - 1
                    break
            to += 1
            if to < n - 1 and not line.startswith(delim, to):
                to = line.find(delim, to + 1)
        elif line.startswith(delim, pos):
            to = pos
        else:
            to = line.find(delim, pos + 1)
        to = n if to < 0 else to
        toks.append(line[pos:to])
        pos = to + dl
    if pos == n:
        toks.append("")
    return toks


def parse_matrix_text(text, rows, cols, format="text"):
    """Dense fp64 (rows x cols) array of a matrix in textcell (i j v, 1-based), MatrixMarket
    or headerless CSV text (reference ReaderTextCell / ReaderTextCSV readMatrixFromInputStream:
    cells outside rows x cols are an error, absent cells are 0)."""
    fmt = _check_format(format)
    rows, cols = int(rows), int(cols)
    out = np.zeros((rows, cols), dtype=np.float64)
    lines = text.splitlines()
    if fmt == "csv":
        r = 0
        for ln in lines:
            if not ln.strip():
                continue
            if r >= rows:
                raise IOError(f"csv input has more than {rows} rows")
            toks = split_csv(ln.rstrip("\r"), ",")
            if len(toks) != cols:
                raise IOError(f"csv row {r + 1}: {len(toks)} columns, expected {cols}")
            out[r] = [float(t) if t.strip() else 0.0 for t in toks]
            r += 1
        return out
    k = 0
    if fmt == "mm":
        while k < len(lines) and (lines[k].startswith("%") or not lines[k].strip()):
            k += 1
        k += 1                                     # the "rows cols nnz" size line
    for ln in lines[k:]:
        t = ln.split()
        if not t or t[0].startswith("%"):
            continue
        i, j = int(t[0]), int(t[1])
        if not (1 <= i <= rows and 1 <= j <= cols):
            raise IOError(f"matrix cell ({i},{j}) out of the bounds {rows} x {cols}")
        out[i - 1, j - 1] = float(t[2]) if len(t) > 2 else 1.0
    return out


def parse_frame_text(text, rows, cols, format="text", schema=None, names=None):
    """String FrameBlock of a frame in textcell (i j value) or headerless CSV text (reference
    FrameReaderTextCell / FrameReaderTextCSV readFrameFromInputStream; CSV tokens verbatim)."""
    fmt = _check_format(format)
    rows, cols = int(rows), int(cols)
    columns = [[None] * rows for _ in range(cols)]
    if fmt == "csv":
        r = 0
        for ln in text.splitlines():
            if ln == "" or r >= rows:
                continue
            toks = split_csv(ln.rstrip("\r"), ",")
            for j in range(min(cols, len(toks))):
                columns[j][r] = toks[j] if toks[j] != "" else None
            r += 1
    else:
        for ln in text.splitlines():
            t = ln.split(" ", 2)
            if len(t) < 3 or not t[0].strip():
                continue
            i, j = int(t[0]), int(t[1])
            if not (1 <= i <= rows and 1 <= j <= cols):
                raise IOError(f"frame cell ({i},{j}) out of the bounds {rows} x {cols}")
            columns[j - 1][i - 1] = t[2].rstrip("\r")
    return FrameBlock(columns, schema or ["STRING"] * cols, names)


def frame_to_strings(fb: FrameBlock):
    """rows x cols list of strings (None stays None) -- DataConverter.convertToStringFrame."""
    from ..runtime import scalars as S
    r, c = fb.shape
    return [[None if fb.columns[j][i] is None else S.to_str(fb.columns[j][i]) for j in range(c)] for i in range(r)]


def strings_to_frame(data, schema=None, colnames=None):
    """FrameBlock of a 2-D list of strings (DataConverter.convertToFrameBlock): values are
    converted to the schema's types."""
    rows = [list(r) for r in data]
    ncol = len(rows[0]) if rows else (len(schema) if schema else 0)
    sch = [str(s).upper() for s in schema] if schema else ["STRING"] * ncol
    cols = []
    for j in range(ncol):
        vals = [r[j] if j < len(r) else None for r in rows]
        s = sch[j]
        if s in ("DOUBLE", "FP64", "FP32"):
            vals = [None if v is None or v == "" else float(v) for v in vals]
        elif s in ("INT", "INT64", "INT32"):
            vals = [None if v is None or v == "" else int(float(v)) for v in vals]
        elif s == "BOOLEAN":
            vals = [None if v is None or v == "" else (v if isinstance(v, bool) else str(v).upper() == "TRUE")
                    for v in vals]
        cols.append(vals)
    return FrameBlock(cols, sch, list(colnames) if colnames is not None else None)


def _meta_of(meta):
    md = json.loads(meta) if isinstance(meta, str) else dict(meta)
    return int(md["rows"]), int(md["cols"]), str(md.get("format", "text"))


# ----------------------------------------------------------------------------
class ResultVariables:
    """Outputs of one executeScript() call (reference ResultVariables.java)."""

    def __init__(self, values):
        self._v = dict(values)

    def _get(self, name):
        if name not in self._v or self._v[name] is None:
            raise DMLException(f"Non-existent output variable: {name}")
        return self._v[name]

    def getMatrixBlock(self, name):
        """The matrix as this framework's block (a CPU fp64 tensor): no conversion to lists."""
        v = self._get(name)
        from ..ops import core as C
        if C.is_dist(v):
            v = C._dist().gather(v)
        if isinstance(v, torch.Tensor):
            if v.layout != torch.strided:
                v = v.to_dense()
            return v.detach().to("cpu", torch.float64)
        if hasattr(v, "decompress"):
            return self._dense(v.decompress())
        if hasattr(v, "to_dense"):
            return self._dense(v.to_dense())
        raise DMLException(f"Expected matrix result '{name}' not a matrix.")

    @staticmethod
    def _dense(t):
        return t.detach().to("cpu", torch.float64)

    def getMatrix(self, name):
        return self.getMatrixBlock(name).numpy()

    def getFrameBlock(self, name):
        v = self._get(name)
        if not isinstance(v, FrameBlock):
            raise DMLException(f"Expected frame result '{name}' not a frame.")
        return v

    def getFrame(self, name):
        return frame_to_strings(self.getFrameBlock(name))

    def getScalarObject(self, name):
        v = self._get(name)
        from ..runtime import scalars as S
        if type(v) is S.DevScalar:
            v = v.value()
        if isinstance(v, torch.Tensor) and v.numel() == 1 and v.dim() == 0:
            v = v.item()
        if not isinstance(v, (bool, int, float, str, np.generic)):
            raise DMLException(f"Expected scalar result '{name}' not a scalar.")
        return v.item() if isinstance(v, np.generic) else v

    def getDouble(self, name):
        v = self.getScalarObject(name)
        return float(v) if not isinstance(v, str) else float(v)

    def getLong(self, name):
        v = self.getScalarObject(name)
        return int(float(v)) if isinstance(v, str) else int(v)

    def getString(self, name):
        from ..runtime import scalars as S
        return S.to_str(self.getScalarObject(name))

    def getBoolean(self, name):
        v = self.getScalarObject(name)
        return v.upper() == "TRUE" if isinstance(v, str) else bool(v)

    def getVariableNames(self):
        return set(self._v.keys())

    def size(self):
        return len(self._v)


class PreparedScript:
    """A precompiled DML / PyDML script with registered inputs and outputs (reference
    PreparedScript.java).  Bound inputs live in this object's symbol table; inputs bound with
    `reuse=True` survive executeScript() / clearParameters()."""

    def __init__(self, compiled, inputs, outputs, config=None, connection=None):
        self._cs = compiled
        self._input_names = list(inputs)
        self._outputs = list(outputs)
        self._bound = {}
        self._reuse = {}
        self._config = config if config is not None else compiled.config
        self._conn = connection
        self._recompile_once = set()
        self._lock = threading.Lock()

    # -- configuration ------------------------------------------------------
    def setConfigProperty(self, name, value):
        """Set one configuration property (the reference's DMLConfig text keys, e.g.
        `sysml.cp.parallel.ops`, or this framework's attribute names)."""
        self._config.set(name, value)
        self._cs.config = self._config

    def resetConfig(self):
        self._config = get_default_config().copy()
        self._cs.config = self._config

    def getDMLConfig(self):
        return self._config

    # -- bindings -----------------------------------------------------------
    def _check(self, name):
        if name not in self._input_names:
            raise DMLException(f"Unspecified input variable: {name}")

    def setMatrix(self, name, value, reuse=False):
        self._check(name)
        if isinstance(value, FrameBlock):
            raise DMLException(f"setMatrix: '{name}' got a frame")
        v = EX.convert_input(np.asarray(value, dtype=np.float64) if isinstance(value, (list, tuple)) else value)
        self._bind(name, v, reuse)

    def setFrame(self, name, frame, schema=None, colnames=None, reuse=False):
        """Bind a frame: a FrameBlock or a 2-D list of strings, with an optional schema (list of
        value types) and column names (PreparedScript.java:316-406)."""
        self._check(name)
        if isinstance(schema, bool):                  # setFrame(name, frame, reuse) positional form
            schema, reuse = None, schema
        fb = frame if isinstance(frame, FrameBlock) else strings_to_frame(frame, schema, colnames)
        self._bind(name, fb, reuse)

    def setScalar(self, name, value, reuse=False):
        self._check(name)
        if isinstance(value, np.generic):
            value = value.item()
        if not isinstance(value, (bool, int, float, str)):
            raise DMLException(f"setScalar: '{name}' is not a scalar")
        self._bind(name, value, reuse)

    def _bind(self, name, v, reuse):
        self._bound[name] = v
        if reuse:
            self._reuse[name] = v
        else:
            self._reuse.pop(name, None)

    def clearParameters(self):
        """Remove the bound values (those bound with reuse=True come back at the next
        executeScript(), as in the reference)."""
        self._bound = {}

    # -- execution ----------------------------------------------------------
    def executeScript(self):
        vals = dict(self._reuse)
        vals.update(self._bound)
        missing = [n for n in self._input_names if n not in vals]
        if missing:
            raise DMLException(f"unbound inputs: {missing}")
        with self._lock:        # one execution of this program / symbol table at a time
            values, _ = EX.execute(self._cs, vals)
        self._bound = {}
        return ResultVariables(values)

    def explain(self):
        """The compiled plan (hops per program block) as a string (PreparedScript.java:458)."""
        return EX.explain(self._cs.cp, "hops")

    def enableFunctionRecompile(self, namespace, *fnames):
        """Recompile the named functions once on every entry (PreparedScript.java:474): their
        plans are re-derived for the argument shapes of each call.  This runtime already
        re-plans every block whose operand shape signature changed (compiler/cost.py
        recompile_block), so the flag marks the function (FunctionBlock.recompile_once, read by
        the function call) and validates the names: recursive functions are skipped with a
        warning, as are unknown names."""
        from ..compiler import ipa
        ns = namespace or ".defaultNS"
        graph, _ = ipa.call_graph(self._cs.cp)
        funcs = self._cs.cp.functions
        for fn in fnames:
            key = next((k for k in funcs if k[1] == fn and (k[0] == ns or (namespace is None and k[0] in
                                                                            (".defaultNS", "", None)))), None)
            if key is None:
                log.warning("Failed to enable function recompile for non-existing '%s::%s'.", ns, fn)
                continue
            if getattr(funcs[key], "recursive", False):
                log.warning("Failed to enable function recompile for recursive '%s::%s'.", ns, fn)
                continue
            self._recompile_once.add(key)
            funcs[key].recompile_once = True

    def clone(self, deep=False):
        """An equivalent prepared script with its own program and symbol table, for concurrent
        execution from threads (PreparedScript.java:514).  The program is re-planned from the
        script source (so no plan state is shared); reused bindings are carried over."""
        a = self._cs.compile_args
        cs = EX.compile_script(self._cs.source, a["args"], inputs=a["inputs"], outputs=a["outputs"],
                               config=self._config, pydml=a["pydml"], filename=a["filename"],
                               base_dir=a["base_dir"])
        ps = PreparedScript(cs, self._input_names, self._outputs, self._config, self._conn)
        ps._reuse = dict(self._reuse)
        if self._recompile_once:
            ps._recompile_once = set(self._recompile_once)
        return ps

    def __copy__(self):
        return self.clone(False)


class Connection:
    """Entry point of the JMLC API (reference Connection.java): prepares scripts and converts
    / reads matrices, frames and transform metadata."""

    def __init__(self, config: DMLConfig = None, *cconfigs):
        self.config = (config or get_default_config()).copy()
        self.compiler_configs = set(cconfigs)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def readScript(self, path):
        with open(path) as f:
            return f.read()

    def prepareScript(self, script, args=None, inputs=(), outputs=(), parsePyDML=False):
        """Precompile `script` with the `$`-arguments `args` and register its input and output
        variables.  Also callable as prepareScript(script, inputs, outputs[, parsePyDML])
        (the reference overloads, Connection.java:190-217)."""
        if isinstance(args, (list, tuple)):                   # (script, inputs, outputs, pydml)
            args, inputs, outputs, parsePyDML = None, args, inputs, (outputs if isinstance(outputs, bool)
                                                                    else parsePyDML)
        bad = [k for k in (args or {}) if k is None or not str(k).startswith("$")]
        if bad:
            raise DMLException(f"Invalid argument names: {bad}")
        bad = [k for k in list(inputs) + list(outputs) if k is None or str(k).startswith("$")]
        if bad:
            raise DMLException(f"Invalid variable names: {bad}")
        a = {str(k)[1:]: (v if not isinstance(v, bool) else ("TRUE" if v else "FALSE"))
             for k, v in (args or {}).items()}
        cs = EX.compile_script(script, a, inputs=list(inputs), outputs=list(outputs), config=self.config,
                               pydml=parsePyDML)
        return PreparedScript(cs, inputs, outputs, self.config.copy(), self)

    # -- matrices -----------------------------------------------------------
    def readDoubleMatrix(self, fname, format=None, rows=-1, cols=-1, brlen=-1, bclen=-1, nnz=-1):
        """Read a matrix file as a dense 2-D fp64 array; format and size come from its .mtd
        unless given (Connection.java:339-394)."""
        from ..io import mtd as M
        from ..io.readers import read_matrix
        md = M.read_mtd(fname)
        if format is None and md is None:
            raise IOError(f"no metadata file for '{fname}'")
        kw = {}
        if format is not None:
            kw["format"] = format
        if rows is not None and rows > 0:
            kw["rows"] = rows
        if cols is not None and cols > 0:
            kw["cols"] = cols
        return read_matrix(fname, **kw).numpy()

    def convertToMatrix(self, input, rows_or_meta, cols=None, format="text"):
        """Matrix block (CPU fp64 tensor) of a matrix in textcell (default), csv or mm text,
        given as a string or a stream, with its size as (rows, cols) or as the JSON metadata
        string (Connection.java:471-574)."""
        if cols is None:
            rows, cols, format = _meta_of(rows_or_meta)
        else:
            rows = rows_or_meta
        return torch.from_numpy(parse_matrix_text(_text_of(input), rows, cols, format))

    def convertToDoubleMatrix(self, input, rows_or_meta, cols=None, format="text"):
        return self.convertToMatrix(input, rows_or_meta, cols, format).numpy()

    # -- frames -------------------------------------------------------------
    def readStringFrame(self, fname, format=None, rows=-1, cols=-1):
        """Read a frame file as a 2-D list of strings (Connection.java:588-634)."""
        from ..io import mtd as M
        md = M.read_mtd(fname) or {}
        fmt = (format or md.get("format", "csv")).lower()
        rows = rows if rows and rows > 0 else int(md.get("rows", -1))
        cols = cols if cols and cols > 0 else int(md.get("cols", -1))
        with open(fname) as f:
            text = f.read()
        if rows < 0 or cols < 0:
            probe = parse_frame_text(text, 1 << 30, 1 << 20, fmt) if fmt != "csv" else None
            if fmt == "csv":
                lines = [ln for ln in text.splitlines() if ln != ""]
                rows = len(lines) if rows < 0 else rows
                cols = max((len(split_csv(ln)) for ln in lines), default=0) if cols < 0 else cols
            else:
                nz = [(i, j) for j, c in enumerate(probe.columns) for i, v in enumerate(c) if v is not None]
                rows = max((i for i, _ in nz), default=-1) + 1 if rows < 0 else rows
                cols = max((j for _, j in nz), default=-1) + 1 if cols < 0 else cols
        return frame_to_strings(parse_frame_text(text, rows, cols, fmt))

    def convertToFrame(self, input, rows_or_meta, cols=None, format="text"):
        """FrameBlock of a frame in textcell (default) or csv text, as a string or a stream
        (Connection.java:711-812)."""
        if cols is None:
            rows, cols, format = _meta_of(rows_or_meta)
        else:
            rows = rows_or_meta
        return parse_frame_text(_text_of(input), rows, cols, format)

    def convertToStringFrame(self, input, rows_or_meta, cols=None, format="text"):
        return frame_to_strings(self.convertToFrame(input, rows_or_meta, cols, format))

    # -- transform metadata -------------------------------------------------
    def readTransformMetaDataFromFile(self, spec_or_path, metapath=None, colDelim=","):
        """The legacy transform metadata directory (column.names, Recode/*.map, Bin/*.bin,
        Impute/*.impute) as the frame transformapply / transformdecode take
        (Connection.java:827-857).  Without a spec, every column with a recode map is recoded
        and every column with a bin file binned."""
        spec, path = (None, spec_or_path) if metapath is None else (spec_or_path, metapath)
        from ..runtime import transform as T
        if spec is None:
            spec = _spec_from_dir(path, colDelim)
        return T.read_meta_dir(spec, path, colDelim)

    def readTransformMetaDataFromPath(self, spec_or_path, metapath=None, colDelim=","):
        """As readTransformMetaDataFromFile, with the directory resolved as a resource: relative
        to the package's script tree (`systemml_amd/scripts`), the package, the working
        directory or an entry of sys.path (Connection.java:868-898)."""
        spec, path = (None, spec_or_path) if metapath is None else (spec_or_path, metapath)
        return self.readTransformMetaDataFromFile(spec, _resource_dir(path), colDelim)

    def close(self):
        pass


def _spec_from_dir(path, sep=","):
    with open(os.path.join(path, "column.names")) as f:
        names = [c.strip().strip('"') for c in f.read().strip().split(sep)]
    rc = [i + 1 for i, n in enumerate(names) if os.path.exists(os.path.join(path, "Recode", n + ".map"))]
    bn = [i + 1 for i, n in enumerate(names) if os.path.exists(os.path.join(path, "Bin", n + ".bin"))]
    spec = {"ids": True}
    if rc:
        spec["recode"] = rc
    if bn:
        spec["bin"] = [{"id": i, "method": "equi-width"} for i in bn]
    return json.dumps(spec)


def _resource_dir(path):
    import sys
    if os.path.isabs(path) and os.path.isdir(path):
        return path
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rel = path.lstrip("/")
    for base in [os.path.join(pkg, "scripts"), pkg, os.getcwd()] + [p for p in sys.path if p]:
        cand = os.path.join(base, rel)
        if os.path.isdir(cand):
            return cand
    raise IOError(f"transform metadata resource '{path}' not found")


__all__ = ["Connection", "PreparedScript", "ResultVariables", "DMLException", "split_csv"]
