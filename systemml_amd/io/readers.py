"""Matrix / frame readers (reference: runtime/io/{ReaderTextCell,ReaderTextCSV,
ReaderBinaryBlock,FrameReaderTextCSV,...}.java and parser/DataExpression.java read()
parameter handling).

Formats: `text` (i j v triples, 1-based), `mm` (MatrixMarket coordinate/array),
`csv` (header, sep, fill, na.strings), `binary` (this framework's block format:
little-endian header + fp64/fp32/bf16 payload, memory-mapped on read).  A
directory of part files (as written by the reference's Spark backend) is read
as the concatenation of its parts.  Parsing of large text files uses the
native C++ reader when built (ops/csrc/fastio.cpp).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..parser.errors import DMLRuntimeError
from ..ops.backend import place, maybe_bf16
from ..runtime.data import FrameBlock
from . import mtd as M

BIN_MAGIC = b"SYSMLAMD"


def _files(fname):
    if os.path.isdir(fname):
        parts = sorted(os.path.join(fname, f) for f in os.listdir(fname)
                       if not f.startswith(".") and not f.startswith("_") and not f.endswith(".mtd"))
        return parts
    return [fname]


def read_matrix(fname, **kw):
    """Read a matrix file (any supported format, .mtd honoured) into a CPU fp64 tensor."""
    return torch.as_tensor(read(None, fname, **kw)).double().cpu()


def read(ctx, fname, **kw):
    md = M.read_mtd(fname) or {}
    fmt = kw.get("format", md.get("format", None))
    fmt = fmt.lower() if isinstance(fmt, str) else fmt
    dtype = kw.get("data_type", md.get("data_type", "matrix"))
    if fmt is None:
        fmt = _sniff(fname)
    if not os.path.exists(fname):
        raise DMLRuntimeError(f"read: file '{fname}' does not exist")
    rows = kw.get("rows", md.get("rows", -1))
    cols = kw.get("cols", md.get("cols", -1))
    rows = int(rows) if rows is not None else -1
    cols = int(cols) if cols is not None else -1
    if dtype == "scalar":
        with open(_files(fname)[0]) as f:
            txt = f.read().strip()
        vt = kw.get("value_type", md.get("value_type", "double"))
        if vt == "string":
            return txt
        if vt == "int":
            return int(float(txt))
        if vt == "boolean":
            return txt.upper() == "TRUE"
        return float(txt)
    if dtype == "frame":
        return read_frame(fname, fmt, rows, cols, md, **kw)
    if ctx is not None and ctx.dist is not None:
        part = _read_partitioned(ctx, fname, fmt, rows, cols, md, kw)
        if part is not None:
            return part
    if fmt == "csv":
        header = _b(kw.get("header", md.get("header", False)))
        sep = kw.get("sep", md.get("sep", ","))
        fill = _b(kw.get("fill", md.get("fill", True)))
        fill_value = float(kw.get("default", md.get("default", 0.0)))
        na = kw.get("naStrings", md.get("naStrings", None))
        arr = read_csv_matrix(fname, header, sep, fill, fill_value, na)
    elif fmt in ("text", "ijv"):
        arr = read_text_cell(fname, rows, cols)
    elif fmt == "mm":
        arr = read_matrix_market(fname)
    elif fmt in ("binary", "native"):
        from . import binaryblock as BB
        if BB.is_sequence_file(fname):
            brlen = int(kw.get("rows_in_block", md.get("rows_in_block", 1000)))
            bclen = int(kw.get("cols_in_block", md.get("cols_in_block", brlen)))
            arr = BB.read_binary_block(fname, rows, cols, brlen, bclen)
        else:
            return _post(read_binary(fname), ctx)
    else:
        raise DMLRuntimeError(f"read: unsupported format '{fmt}'")
    if rows > 0 and cols > 0 and arr.shape != (rows, cols):
        if arr.shape[0] <= rows and arr.shape[1] <= cols:
            full = np.zeros((rows, cols))
            full[:arr.shape[0], :arr.shape[1]] = arr
            arr = full
        else:
            raise DMLRuntimeError(f"read: dimensions {arr.shape} do not match metadata {rows}x{cols}")
    return _post(torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float64)), ctx)


def _read_partitioned(ctx, fname, fmt, rows, cols, md, kw):
    """SPMD read: each rank parses / maps only its own row block (reference analogue: the
    per-partition HDFS splits a Spark job reads).  Binary files are memory-mapped and
    sliced; single-file CSVs go through the native row-range parser.  Returns None when the
    matrix stays replicated (fewer than `sysml.dist.minrows` rows) or the format has no
    partitioned reader."""
    from ..parallel import dist as D
    from ..ops import native
    dctx = ctx.dist
    minr = ctx.config.dist_min_rows
    files = _files(fname)
    if fmt in ("binary", "native"):
        from . import binaryblock as BB
        if BB.is_sequence_file(fname):
            if rows <= 0 or cols <= 0 or rows < minr:
                return None
            brlen = int(kw.get("rows_in_block", md.get("rows_in_block", 1000)))
            bclen = int(kw.get("cols_in_block", md.get("cols_in_block", brlen)))
            s, e = dctx.partition(rows)
            loc = BB.read_binary_block(fname, rows, cols, brlen, bclen, row_range=(s, e))
            return D.local_block(dctx, torch.from_numpy(loc), rows, cols)
        with open(fname, "rb") as f:
            head = f.read(32)
        r, c = (int(v) for v in np.frombuffer(head[8:24], dtype=np.int64))
        if r < minr:
            return None
        code = int(np.frombuffer(head[24:28], dtype=np.int32)[0])
        dt = {0: np.float64, 1: np.float32, 2: np.uint16}[code]
        s, e = dctx.partition(r)
        arr = np.memmap(fname, dtype=dt, mode="r", offset=32 + s * c * np.dtype(dt).itemsize, shape=(e - s, c))
        loc = torch.from_numpy(np.array(arr)).view(torch.bfloat16) if code == 2 else \
            torch.from_numpy(np.array(arr, dtype=np.float64))
        return D.local_block(dctx, loc, r, c)
    if fmt != "csv" or len(files) != 1 or native.lib() is None:
        return None
    header = _b(kw.get("header", md.get("header", False)))
    sep = kw.get("sep", md.get("sep", ","))
    if kw.get("naStrings", md.get("naStrings")) is not None or not _b(kw.get("fill", md.get("fill", True))) \
            or float(kw.get("default", md.get("default", 0.0))) != 0.0 or len(sep) != 1:
        return None
    thr = os.cpu_count() or 8
    if rows <= 0:
        got = native.parse_csv_rows(files[0], 0, 0, sep, header, thr)
        if got is None:
            return None
        rows = got[1]
    if rows < minr:
        return None
    s, e = dctx.partition(rows)
    got = native.parse_csv_rows(files[0], s, e, sep, header, thr)
    if got is None:
        return None
    arr, total = got
    if total != rows:
        raise DMLRuntimeError(f"read: {fname} has {total} rows, metadata says {rows}")
    if cols > 0 and arr.shape[1] != cols:
        if arr.shape[1] > cols:
            raise DMLRuntimeError(f"read: dimensions do not match metadata {rows}x{cols}")
        arr = np.hstack([arr, np.zeros((arr.shape[0], cols - arr.shape[1]))])
    ncols = arr.shape[1] if cols <= 0 else cols
    if arr.shape[0] == 0:
        arr = np.zeros((0, ncols))
    # column count of an empty local block: agree on the global maximum
    ncols = int(dctx.allreduce_scalar(float(ncols), "max"))
    if arr.shape[1] != ncols:
        arr = np.zeros((arr.shape[0], ncols)) if arr.shape[0] == 0 else arr
    return D.local_block(dctx, torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float64)), rows, ncols)


def _post(t, ctx):
    if ctx is not None and ctx.dist is not None and t.shape[0] >= ctx.config.dist_min_rows:
        from ..parallel import dist as D
        return D.scatter_rows(ctx, t)
    from ..ops import sparse as SP
    t = SP.maybe_sparse(t)
    if SP.is_sparse(t):
        return place_sparse(t)
    return maybe_compress(maybe_bf16(place(t)), ctx.config if ctx is not None else None)


def maybe_compress(t, config):
    """Compressed linear algebra for read-only inputs (reference: sysml.compressed.linalg)."""
    mode = getattr(config, "compressed_linalg", "false") if config is not None else "false"
    if mode not in ("true", "auto") or not isinstance(t, torch.Tensor) or t.dim() != 2:
        return t
    from ..ops import compress as CMP
    c = CMP.compress(t)
    if CMP.is_compressed(c) and (mode == "true" or c.ratio() >= 3.0):
        return c
    return t


def place_sparse(t):
    from ..ops.backend import backend
    return t.to(device=backend.device, dtype=backend.dtype)


def _b(v):
    if isinstance(v, str):
        return v.strip().upper() == "TRUE"
    return bool(v)


def _sniff(fname):
    f = _files(fname)[0]
    with open(f, "rb") as fh:
        head = fh.read(64)
    if head.startswith(BIN_MAGIC) or head.startswith(b"SEQ"):
        return "binary"
    if head.startswith(b"%%MatrixMarket"):
        return "mm"
    txt = head.decode("latin1", "ignore")
    if "," in txt:
        return "csv"
    return "text"


def read_text_cell(fname, rows=-1, cols=-1):
    from ..ops import native
    chunks = []
    for f in _files(fname):
        a = native.parse_ijv(f)
        if a is None:
            a = np.loadtxt(f, ndmin=2) if os.path.getsize(f) > 0 else np.zeros((0, 3))
        chunks.append(a)
    ijv = np.concatenate(chunks) if chunks else np.zeros((0, 3))
    if ijv.size == 0:
        return np.zeros((max(rows, 0), max(cols, 0)))
    i = ijv[:, 0].astype(np.int64) - 1
    j = ijv[:, 1].astype(np.int64) - 1
    r = rows if rows > 0 else int(i.max()) + 1
    c = cols if cols > 0 else int(j.max()) + 1
    out = np.zeros((r, c))
    out[i, j] = ijv[:, 2]
    return out


def read_matrix_market(fname):
    with open(fname) as f:
        header = f.readline()
        if not header.startswith("%%MatrixMarket"):
            raise DMLRuntimeError("invalid MatrixMarket header")
        toks = header.lower().split()
        layout = toks[2] if len(toks) > 2 else "coordinate"
        symmetric = "symmetric" in toks
        line = f.readline()
        while line.startswith("%"):
            line = f.readline()
        dims = [int(x) for x in line.split()]
        data = np.loadtxt(f, ndmin=2) if True else None
    if layout == "array":
        r, c = dims[0], dims[1]
        return data.reshape(-1)[: r * c].reshape(c, r).T.copy()
    r, c = dims[0], dims[1]
    out = np.zeros((r, c))
    if data.size:
        i = data[:, 0].astype(np.int64) - 1
        j = data[:, 1].astype(np.int64) - 1
        v = data[:, 2] if data.shape[1] > 2 else np.ones(len(i))
        out[i, j] = v
        if symmetric:
            out[j, i] = v
    return out


def read_csv_matrix(fname, header=False, sep=",", fill=True, fill_value=0.0, na=None):
    from ..ops import native
    parts = []
    for k, f in enumerate(_files(fname)):
        # native multi-threaded parser (ops/csrc/fastio.cpp) unless NA strings / a non-zero fill
        a = native.parse_csv(f, sep, header, threads=os.cpu_count() or 8) \
            if (na is None and fill and fill_value == 0.0) else None
        if a is None:
            rows = []
            with open(f) as fh:
                if header:
                    fh.readline()
                for line in fh:
                    line = line.rstrip("\n\r")
                    if not line:
                        continue
                    vals = []
                    for t in line.split(sep):
                        t = t.strip()
                        if t == "" or (na and t in na):
                            vals.append(fill_value if fill else float("nan"))
                        else:
                            vals.append(float(t))
                    rows.append(vals)
            a = np.array(rows, dtype=np.float64) if rows else np.zeros((0, 0))
        parts.append(a)
    return np.concatenate(parts) if len(parts) > 1 else parts[0]


def read_binary(fname):
    with open(fname, "rb") as f:
        head = f.read(32)
    if not head.startswith(BIN_MAGIC):
        raise DMLRuntimeError("not a systemml_amd binary matrix file")
    r, c = np.frombuffer(head[8:24], dtype=np.int64)
    code = int(np.frombuffer(head[24:28], dtype=np.int32)[0])
    dt = {0: np.float64, 1: np.float32, 2: np.uint16}[code]
    arr = np.memmap(fname, dtype=dt, mode="r", offset=32, shape=(int(r), int(c)))
    if code == 2:
        t = torch.from_numpy(np.array(arr)).view(torch.bfloat16)
        return t
    return torch.from_numpy(np.array(arr, dtype=np.float64))


def read_frame(fname, fmt, rows, cols, md, **kw):
    header = _b(kw.get("header", md.get("header", False)))
    sep = kw.get("sep", md.get("sep", ","))
    schema = kw.get("schema", md.get("schema", None))
    lines = []
    names = None
    for f in _files(fname):
        with open(f) as fh:
            if header:
                h = fh.readline().rstrip("\n\r")
                if names is None:
                    names = [x.strip() for x in h.split(sep)]
            for line in fh:
                line = line.rstrip("\n\r")
                if line:
                    lines.append(_split_csv(line, sep))
    if fmt in ("text", "ijv"):
        cells = {}
        mr = mc = 0
        for l in lines:
            toks = l[0].split() if len(l) == 1 else l
            i, j, v = int(toks[0]), int(toks[1]), " ".join(toks[2:])
            cells[(i, j)] = v
            mr, mc = max(mr, i), max(mc, j)
        r = rows if rows > 0 else mr
        c = cols if cols > 0 else mc
        columns = [[cells.get((i + 1, j + 1)) for i in range(r)] for j in range(c)]
    else:
        c = max((len(l) for l in lines), default=0)
        columns = [[(l[j] if j < len(l) else None) for l in lines] for j in range(c)]
    sch = None
    if schema:
        sch = [s.strip().upper() for s in (schema.split(",") if isinstance(schema, str) else schema)]
        for j, s in enumerate(sch):
            if s in ("DOUBLE", "FP64", "FP32"):
                columns[j] = [float(v) if v not in (None, "") else None for v in columns[j]]
            elif s in ("INT", "INT64", "INT32"):
                columns[j] = [int(float(v)) if v not in (None, "") else None for v in columns[j]]
            elif s == "BOOLEAN":
                columns[j] = [str(v).upper() == "TRUE" if v not in (None, "") else None for v in columns[j]]
    return FrameBlock(columns, sch, names)


def _split_csv(line, sep):
    if '"' not in line:
        return [t.strip() for t in line.split(sep)]
    out, cur, q = [], [], False
    for ch in line:
        if ch == '"':
            q = not q
        elif ch == sep and not q:
            out.append("".join(cur).strip())
            cur = []
        else:
            cur.append(ch)
    out.append("".join(cur).strip())
    return out
