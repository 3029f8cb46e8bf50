"""Host-side native helpers (C++, `ops/csrc/fastio.cpp` → `libsysml_native.so`):
multi-threaded CSV / ijv text parsing for the readers (reference: the parallel
readers runtime/io/ReaderTextCSVParallel.java, ReaderTextCellParallel.java).
Returns None when the library is not built so callers fall back to Python."""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_TRIED = False


def lib():
    global _LIB, _TRIED
    if _TRIED:
        return _LIB
    _TRIED = True
    path = os.path.join(_HERE, "lib", "libsysml_native.so")
    if os.path.exists(path):
        try:
            L = ctypes.CDLL(path)
            L.sysml_parse_csv.restype = ctypes.c_int64
            L.sysml_parse_csv.argtypes = [ctypes.c_char_p, ctypes.c_char, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                          ctypes.POINTER(ctypes.POINTER(ctypes.c_double)), ctypes.c_int]
            L.sysml_parse_csv_rows.restype = ctypes.c_int64
            L.sysml_parse_csv_rows.argtypes = [ctypes.c_char_p, ctypes.c_char, ctypes.c_int, ctypes.c_int64,
                                               ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                                               ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                               ctypes.POINTER(ctypes.POINTER(ctypes.c_double)), ctypes.c_int]
            L.sysml_parse_ijv.restype = ctypes.c_int64
            L.sysml_parse_ijv.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.POINTER(ctypes.c_double)),
                                          ctypes.c_int]
            L.sysml_free.argtypes = [ctypes.c_void_p]
            _LIB = L
        except OSError:
            _LIB = None
    return _LIB


def parse_csv(path, sep=",", header=False, threads=8):
    L = lib()
    if L is None or len(sep) != 1:
        return None
    rows = ctypes.c_int64()
    cols = ctypes.c_int64()
    buf = ctypes.POINTER(ctypes.c_double)()
    rc = L.sysml_parse_csv(path.encode(), sep.encode(), int(bool(header)), ctypes.byref(rows),
                           ctypes.byref(cols), ctypes.byref(buf), threads)
    if rc < 0:
        return None
    n = rows.value * cols.value
    arr = np.ctypeslib.as_array(buf, shape=(max(n, 1),))[:n].copy().reshape(rows.value, cols.value)
    L.sysml_free(buf)
    return arr


def parse_csv_rows(path, row_lo, row_hi, sep=",", header=False, threads=8):
    """Data rows [row_lo, row_hi) of a CSV file and the file's total row count (only the
    byte ranges holding those rows are parsed)."""
    L = lib()
    if L is None or len(sep) != 1:
        return None
    rows, cols, total = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    buf = ctypes.POINTER(ctypes.c_double)()
    rc = L.sysml_parse_csv_rows(path.encode(), sep.encode(), int(bool(header)), int(row_lo), int(row_hi),
                                ctypes.byref(rows), ctypes.byref(cols), ctypes.byref(total), ctypes.byref(buf),
                                threads)
    if rc < 0:
        return None
    n = rows.value * cols.value
    arr = np.ctypeslib.as_array(buf, shape=(max(n, 1),))[:n].copy().reshape(rows.value, cols.value)
    L.sysml_free(buf)
    return arr, total.value


def parse_ijv(path, threads=8):
    L = lib()
    if L is None:
        return None
    buf = ctypes.POINTER(ctypes.c_double)()
    n = L.sysml_parse_ijv(path.encode(), ctypes.byref(buf), threads)
    if n < 0:
        return None
    arr = np.ctypeslib.as_array(buf, shape=(max(n * 3, 1),))[: n * 3].copy().reshape(n, 3)
    L.sysml_free(buf)
    return arr
