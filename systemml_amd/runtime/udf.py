"""External functions (reference: udf/PackageFunction.java, udf/lib/*.java,
runtime/controlprogram/ExternalFunctionProgramBlock*.java).

`externalFunction(...) implemented in (classname="...")` binds a DML function
signature to native code.  The reference loads Java classes; we bind the
reference's class names to Python implementations of the same semantics
(org.apache.sysml.udf.lib.*), and user code can register its own:

    from systemml_amd.runtime.udf import register_udf
    register_udf("my.pkg.Scale", lambda ctx, X, s: (X * s,))
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from ..parser.errors import DMLRuntimeError
from ..ops.backend import place
from . import scalars as S

UDFS = {}


def register_udf(classname, fn):
    UDFS[classname] = fn


def call_external(ctx, fb, args, given):
    cls = fb.ext_params.get("classname")
    fn = UDFS.get(cls) or UDFS.get(cls.split(".")[-1] if cls else None)
    if fn is None:
        raise DMLRuntimeError(f"external function class '{cls}' is not available")
    vals = dict(zip(given, args))
    ordered = [vals.get(p.name) for p in fb.inputs]
    out = fn(ctx, *ordered)
    if not isinstance(out, tuple):
        out = (out,)
    return tuple(out)


def _np(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().double().numpy()
    from ..ops import core as C
    if C.is_dist(x):
        return C._dist().gather(x).cpu().double().numpy()
    return np.asarray(x, dtype=float)


def _t(a):
    return place(torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(
        np.asarray(a).shape[0], -1))))


def binning(ctx, A, binsize, numbins):
    """BinningWrapper: equi-height bin boundaries of a sorted column (duplicates extend a bin)."""
    col = _np(A).reshape(-1)
    n = col.shape[0]
    binsize, numbins = int(binsize), int(numbins)
    bins = np.zeros(numbins + 1)
    pos, bid = 0, 0
    bins[0] = col[0]
    while pos < n - 1 and bid < numbins:
        pos = n - 1 if pos + binsize >= n else pos + binsize
        end = col[pos]
        bins[bid + 1] = end
        while pos < n - 1 and col[pos + 1] == end:
            pos += 1
        bid += 1
    for i in range(bid):
        bins[i] = (bins[i] + bins[i + 1]) / 2
    return _t(bins.reshape(-1, 1)), bid


def order(ctx, A, col, desc=False):
    """OrderWrapper: sort rows by a column."""
    a = _np(A)
    idx = np.argsort(a[:, int(col) - 1], kind="stable")
    if S.as_bool(desc):
        idx = idx[::-1]
    return (_t(a[idx]),)


def cumsumprod(ctx, X, C, start):
    """CumSumProd: Y[i] = X[i] + C[i] * Y[i-1] (Y[0] from `start`)."""
    # Hillis-Steele scan of the affine maps y -> b + a * y: after the step of width k, (a[i], b[i])
    # maps y[i - 2k] to y[i]; log2(n) vectorised steps instead of an n-step loop
    b = _np(X).reshape(-1).astype(np.float64)
    a = _np(C).reshape(-1).astype(np.float64)
    k = 1
    while k < len(b):
        b[k:] = b[k:] + a[k:] * b[:-k]
        a[k:] = a[k:] * a[:-k]
        k *= 2
    return (_t((b + a * float(start)).reshape(-1, 1)),)


def multi_input_cbind(ctx, *args):
    return (torch.cat([a for a in args if isinstance(a, torch.Tensor)], 1),)


def remove_empty_rows(ctx, X):
    x = _np(X)
    keep = np.any(x != 0, axis=1)
    return (_t(x[keep] if keep.any() else np.zeros((1, x.shape[1]))),)


def time_wrapper(ctx, *a):
    return (float(time.time() * 1000.0),)


def dynamic_read_matrix(ctx, fname, rows, cols, fmt):
    from ..io import readers
    return (readers.read(ctx, S.to_str(fname), rows=int(rows), cols=int(cols), format=S.to_str(fmt)),)


def dynamic_write_matrix(ctx, X, fname, fmt):
    from ..io import writers
    writers.write(ctx, X, S.to_str(fname), format=S.to_str(fmt))
    return (True,)


def dynamic_project(ctx, X, c, r=None):
    x = _np(X)
    ci = _np(c).reshape(-1).astype(int) - 1
    if r is None:
        return (_t(x[np.ix_(ci, ci)]),)
    ri = _np(r).reshape(-1).astype(int) - 1
    return (_t(x[np.ix_(ri, ci)]),)


def gather(ctx, X, I):
    x = _np(X).reshape(-1)
    i = _np(I).reshape(-1).astype(int) - 1
    return (_t(x[i].reshape(-1, 1)),)


def row_class_meet(ctx, A, B):
    """RowClassMeet: for label vectors A, B counts class co-occurrence per row-pair class."""
    a = _np(A).reshape(-1).astype(int)
    b = _np(B).reshape(-1).astype(int)
    ka, kb = a.max(), b.max()
    out = np.zeros((ka, kb))
    np.add.at(out, (a - 1, b - 1), 1)
    return (_t(out),)


def sgd_nesterov(ctx, X, dX, lr, mu, v):
    x, dx, vv = _np(X), _np(dX), _np(v)
    v_prev = vv
    vv = float(mu) * vv - float(lr) * dx
    x = x - float(mu) * v_prev + (1 + float(mu)) * vv
    return _t(x), _t(vv)


for _cls, _fn in {
    "org.apache.sysml.udf.lib.BinningWrapper": binning,
    "org.apache.sysml.udf.lib.OrderWrapper": order,
    "org.apache.sysml.udf.lib.CumSumProd": cumsumprod,
    "org.apache.sysml.udf.lib.MultiInputCbind": multi_input_cbind,
    "org.apache.sysml.udf.lib.RemoveEmptyRows": remove_empty_rows,
    "org.apache.sysml.udf.lib.TimeWrapper": time_wrapper,
    "org.apache.sysml.udf.lib.DynamicReadMatrixCP": dynamic_read_matrix,
    "org.apache.sysml.udf.lib.DynamicWriteMatrixCP": dynamic_write_matrix,
    "org.apache.sysml.udf.lib.DynamicProjectMatrixCP": dynamic_project,
    "org.apache.sysml.udf.lib.GatherWrapper": gather,
    "org.apache.sysml.udf.lib.RowClassMeet": row_class_meet,
    "org.apache.sysml.udf.lib.SGDNesterovUpdate": sgd_nesterov,
}.items():
    register_udf(_cls, _fn)
    register_udf(_cls.split(".")[-1], _fn)
