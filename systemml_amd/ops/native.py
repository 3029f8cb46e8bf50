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
            L.sysml_write_cells.restype = ctypes.c_int64
            L.sysml_write_cells.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                            ctypes.c_int, ctypes.c_char, ctypes.c_int, ctypes.c_int]
            L.sysml_java_double.restype = ctypes.c_int
            L.sysml_java_double.argtypes = [ctypes.c_double, ctypes.c_char_p]
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


def write_cells(path, a, mode, sep=",", append=False, threads=8):
    """Write a dense fp64 matrix as csv rows (mode 0) or 'i j v' non-zero lines (mode 1)
    with java.lang.Double.toString formatting; False when the library is unavailable."""
    L = lib()
    if L is None:
        return False
    a = np.ascontiguousarray(a, dtype=np.float64)
    r, c = a.shape
    rc = L.sysml_write_cells(str(path).encode(), a.ctypes.data, r, c, mode, sep.encode()[:1], int(append), threads)
    if rc != 0:
        raise OSError(f"native writer failed ({rc}) for {path}")
    return True


def java_double(d):
    L = lib()
    buf = ctypes.create_string_buffer(64)
    n = L.sysml_java_double(float(d), buf)
    return buf.raw[:n].decode()
