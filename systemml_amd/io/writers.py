"""Matrix / frame / scalar writers (reference: runtime/io/{WriterTextCell,WriterTextCSV,
WriterMatrixMarket,WriterBinaryBlock,FrameWriterTextCSV}.java).  Writes the data
file plus a `.mtd` JSON metadata file; only rank 0 writes in SPMD mode."""
from __future__ import annotations

import os

import numpy as np
import torch

from ..parser.errors import DMLRuntimeError
from ..runtime import scalars as S
from ..runtime.data import FrameBlock, ListObject
from . import mtd as M
from .readers import BIN_MAGIC


def _np(x):
    from ..ops import core as C
    if C.is_dist(x):
        x = C._dist().gather(x)
    if isinstance(x, torch.Tensor):
        return x.detach().to("cpu").double().numpy()
    if isinstance(x, np.ndarray) and x.ndim == 2:
        return x.astype(np.float64, copy=False)
    raise DMLRuntimeError("write: expected a matrix")


def write_matrix(x, fname, format="binary", **kw):
    """Write a matrix (tensor / numpy) with its .mtd file, outside of a DML program."""
    return write(None, x, fname, format=format, **kw)


def write(ctx, x, fname, format="text", **kw):
    fmt = str(format).lower()
    from ..ops import core as C
    if C.is_dist(x):
        x = C._dist().gather(x)
    if ctx is not None and ctx.dist is not None and ctx.dist.rank != 0:
        return
    d = os.path.dirname(fname)
    if d:
        os.makedirs(d, exist_ok=True)
    if isinstance(x, (bool, int, float, str)):
        with open(fname, "w") as f:
            f.write(S.to_str(x))
        M.write_mtd(fname, "scalar", S.vtype_of(x).lower(), 0, 0, fmt="text")
        return
    if isinstance(x, FrameBlock):
        return write_frame(x, fname, fmt, **kw)
    if isinstance(x, ListObject):
        raise DMLRuntimeError("write of lists is not supported")
    if fmt in ("binary", "native") and isinstance(x, torch.Tensor) and x.dtype == torch.bfloat16:
        # bf16 storage has no binary-block encoding: this framework's raw format (mmap-able)
        _write_binary_raw(x, fname, 2)
        M.write_mtd(fname, "matrix", "double", x.shape[0], x.shape[1], fmt=fmt)
        return
    a = _np(x)
    r, c = a.shape
    nnz = int(np.count_nonzero(a))
    from ..ops import native as NAT
    if fmt in ("text", "ijv"):
        open(fname, "w").close()
        if not NAT.write_cells(fname, a, 1, append=True):
            i, j = np.nonzero(a)
            with open(fname, "w") as f:
                for ii, jj in zip(i, j):
                    f.write(f"{ii + 1} {jj + 1} {S.java_double_str(float(a[ii, jj]))}\n")
    elif fmt == "csv":
        sep = kw.get("sep", ",")
        header = str(kw.get("header", False)).upper() == "TRUE"
        with open(fname, "w") as f:
            if header:
                f.write(sep.join(f"C{k + 1}" for k in range(c)) + "\n")
        if len(sep) != 1 or not NAT.write_cells(fname, a, 0, sep=sep, append=True):
            with open(fname, "a") as f:
                for row in a:
                    f.write(sep.join(S.java_double_str(float(v)) for v in row) + "\n")
    elif fmt == "mm":
        i, j = np.nonzero(a)
        with open(fname, "w") as f:
            f.write("%%MatrixMarket matrix coordinate real general\n")
            f.write(f"{r} {c} {len(i)}\n")
        if not NAT.write_cells(fname, a, 1, append=True):
            with open(fname, "a") as f:
                for ii, jj in zip(i, j):
                    f.write(f"{ii + 1} {jj + 1} {S.java_double_str(float(a[ii, jj]))}\n")
    elif fmt == "binary":
        # the reference's binary-block SequenceFile (io/binaryblock.py): loads in SystemML
        from .binaryblock import write_binary_block
        brlen = int(kw.get("rows_in_block", 1000))
        write_binary_block(fname, a, brlen, brlen)
        M.write_mtd(fname, "matrix", "double", r, c, nnz, fmt=fmt, rows_in_block=brlen, cols_in_block=brlen)
        return
    elif fmt == "native":
        _write_binary_raw(torch.from_numpy(a), fname, 0)
    else:
        raise DMLRuntimeError(f"write: unsupported format '{fmt}'")
    M.write_mtd(fname, "matrix", "double", r, c, nnz, fmt=fmt)


def _write_binary_raw(t, fname, code):
    r, c = t.shape
    with open(fname, "wb") as f:
        f.write(BIN_MAGIC)
        f.write(np.array([r, c], dtype=np.int64).tobytes())
        f.write(np.array([code, 0], dtype=np.int32).tobytes())
        if code == 2:
            f.write(t.detach().cpu().contiguous().view(torch.int16).numpy().tobytes())
        else:
            f.write(t.detach().cpu().contiguous().numpy().astype(np.float64 if code == 0 else np.float32).tobytes())


def write_frame(fr: FrameBlock, fname, fmt="csv", **kw):
    sep = kw.get("sep", ",")
    header = str(kw.get("header", False)).upper() == "TRUE"
    r, c = fr.shape
    with open(fname, "w") as f:
        if fmt == "csv":
            if header:
                f.write(sep.join(fr.names) + "\n")
            for i in range(r):
                f.write(sep.join("" if v is None else S.to_str(v) for v in fr.row(i)) + "\n")
        else:
            for i in range(r):
                for j in range(c):
                    v = fr.columns[j][i]
                    if v is not None and v != "":
                        f.write(f"{i + 1} {j + 1} {S.to_str(v)}\n")
    M.write_mtd(fname, "frame", "string", r, c, fmt=fmt, schema=",".join(fr.schema))
