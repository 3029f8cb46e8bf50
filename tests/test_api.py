"""API tests: MLContext, JMLC, CLI, PyDML (reference: test/integration/mlcontext/*,
functions/jmlc/*, python/tests/test_mlcontext.py)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from systemml_amd import MLContext, dml, pydml, DMLConfig
from systemml_amd.api.jmlc import Connection

CFG = DMLConfig(gpu=False)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_mlcontext_roundtrip():
    ml = MLContext(config=CFG)
    out = []
    ml.setOutput(out.append)
    X = np.arange(6, dtype=float).reshape(3, 2)
    s = dml("Y = X %*% t(X); s = sum(Y); print('s=' + s)").input(X=X).output("Y", "s")
    r = ml.execute(s)
    np.testing.assert_allclose(r.get("Y").toNumPy(), X @ X.T)
    assert r.getDouble("s") == (X @ X.T).sum()
    assert out == ["s=" + str(float((X @ X.T).sum()))]


def test_mlcontext_stats_and_explain():
    ml = MLContext(config=CFG).setStatistics(True).setExplain(True)
    out = []
    ml.setOutput(out.append)
    ml.execute(dml("x = rand(rows=10, cols=10, seed=1); print(sum(x))"))
    txt = "\n".join(out)
    assert "EXPLAIN" in txt and "Heavy hitter" in txt


def test_pydml_script():
    ml = MLContext(config=CFG)
    X = np.arange(12, dtype=float).reshape(4, 3)
    src = """
def scale(M: matrix[float], f: float) -> (R: matrix[float]):
    R = M * f

A = X[0:2, ]
B = scale(X[1:3, 1:3], 2.0)
s = sum(X, axis=0)
r = sum(X, axis=1)
t = 0
for i in range(1, 4):  # PyDML range bounds are inclusive (reference semantics)
    if i == 2:
        t = t + 10
    elif i == 3:
        t = t + 100
    else:
        t = t + 1
n = X.shape(0)
P = dot(X, transpose(X))
q = 2 ** 3 + 7 // 2 + 7 % 4
"""
    r = ml.execute(pydml(src).input(X=X).output("A", "B", "s", "r", "t", "n", "P", "q"))
    np.testing.assert_allclose(r.get("A").toNumPy(), X[0:2])
    np.testing.assert_allclose(r.get("B").toNumPy(), X[1:3, 1:3] * 2)
    np.testing.assert_allclose(r.get("s").toNumPy(), X.sum(0, keepdims=True))
    np.testing.assert_allclose(r.get("r").toNumPy(), X.sum(1, keepdims=True))
    assert r.get("t") == 112 and r.get("n") == 4 and r.get("q") == 8.0 + 3 + 3
    np.testing.assert_allclose(r.get("P").toNumPy(), X @ X.T)


def test_jmlc_prepared_script_reuse():
    conn = Connection(CFG)
    ps = conn.prepareScript("W = read($W); X = read($X); Y = X %*% W; write(Y, $Y)",
                            args={"$W": "w", "$X": "x", "$Y": "y"}, inputs=["X", "W"], outputs=["Y"])
    W = np.random.rand(4, 2)
    ps.setMatrix("W", W, reuse=True)
    for _ in range(3):
        X = np.random.rand(5, 4)
        ps.setMatrix("X", X)
        np.testing.assert_allclose(ps.executeScript().getMatrix("Y"), X @ W)


def test_cli_file_and_io(tmp_path):
    script = tmp_path / "s.dml"
    script.write_text("X = rand(rows=$r, cols=3, seed=5); write(X, $out, format=$fmt); "
                      "Y = read($out); print('S ' + sum(abs(X - Y)))\n")
    for fmt in ("text", "csv", "mm", "binary"):
        out = tmp_path / f"x_{fmt}"
        p = subprocess.run([sys.executable, "-m", "systemml_amd", "-f", str(script), "-cpu", "-nvargs", "r=7",
                            f"out={out}", f"fmt={fmt}"], capture_output=True, text=True, cwd=ROOT,
                           env={**os.environ, "PYTHONPATH": ROOT})
        assert p.returncode == 0, p.stderr
        assert "S 0.0" in p.stdout, p.stdout
        assert os.path.exists(str(out) + ".mtd")


def test_cli_stop_returns_error(tmp_path):
    p = subprocess.run([sys.executable, "-m", "systemml_amd", "-s", "stop('boom')", "-cpu"], capture_output=True,
                       text=True, cwd=ROOT, env={**os.environ, "PYTHONPATH": ROOT})
    assert p.returncode == 1 and "boom" in p.stderr


def test_native_csv_and_ijv_parsers(tmp_path):
    import numpy as np
    from systemml_amd.ops import native
    if native.lib() is None:
        pytest.skip("libsysml_native.so not built")
    rng = np.random.default_rng(0)
    A = rng.standard_normal((40000, 7))
    A[3, 2] = 0.0
    f = tmp_path / "a.csv"
    with open(f, "w") as fh:
        fh.write("h1,h2,h3,h4,h5,h6,h7\n")
        for row in A:
            fh.write(",".join(repr(float(v)) for v in row) + "\n")
    B = native.parse_csv(str(f), ",", True, threads=8)     # > 1 MB: multi-threaded path
    np.testing.assert_array_equal(A, B)
    g = tmp_path / "b.ijv"
    g.write_text("1 1 2.5\n3 2 -1e-3\n\n2 3 Infinity\n")
    C = native.parse_ijv(str(g))
    assert C.shape == (3, 3) and C[1, 2] == -1e-3 and np.isinf(C[2, 2])
    h = tmp_path / "c.csv"
    h.write_text("1,,3\n4,5\n")
    np.testing.assert_array_equal(native.parse_csv(str(h), ",", False), [[1, 0, 3], [4, 5, 0]])


def test_debugger_breakpoints_step_and_print():
    import io
    from systemml_amd.api.executor import compile_script
    from systemml_amd.conf import DMLConfig
    from systemml_amd.utils.debugger import Debugger
    src = "A = rand(rows=3, cols=2, seed=1)\nB = A * 2\nC = B + 1\ns = sum(C)\nprint(s)\n"
    cs = compile_script(src, config=DMLConfig(gpu=False))
    inp = io.StringIO("b 3\ni\nr\nw B\nl\ns\nc\n")
    out = io.StringIO()
    ctx = Debugger(cs, inp=inp, out=out).run()
    log = out.getvalue()
    assert "Breakpoint set at line 3" in log and "Breakpoint at line 3" in log
    assert "Program finished." in log
    assert "=>   3  C = B + 1" in log
    assert "matrix[torch.float64] 3x2" in log        # whatis B inside the running block


def test_binary_block_sequencefile_roundtrip(tmp_path):
    """format="binary" is the reference's binary-block SequenceFile (MatrixIndexes ->
    MatrixBlock records): dense, sparse, ultra-sparse and empty blocks, several blocks per
    dimension, sync markers.  A record laid out by hand per MatrixBlock.write decodes too
    (no SystemML-written fixture exists in the reference tree: parity unpinned beyond that)."""
    import struct
    import torch
    from systemml_amd.io import binaryblock as BB, writers, readers
    rng = np.random.default_rng(0)
    A = rng.standard_normal((2500, 1300))
    A[:, 1000:] = 0
    A[1000:2000, :1000] *= rng.random((1000, 1000)) < 0.1        # sparse block row
    A[2000:, :1000] = 0
    A[2100, 7] = 3.5                                              # ultra-sparse block
    p = str(tmp_path / "A")
    writers.write(None, torch.from_numpy(A), p, format="binary")
    assert BB.is_sequence_file(p)
    kinds = {bi * 10 + bj: (payload is None, isinstance(payload, np.ndarray))
             for bi, bj, _, _, payload in BB.iter_blocks(p)}
    assert len(kinds) == 6 and kinds[12] == (True, False) and kinds[11] == (False, True)
    from systemml_amd.ops.sparse import densify
    np.testing.assert_array_equal(densify(readers.read(None, p)).numpy(), A)
    # hand-built file: one 2x3 dense block and one 2x2 sparse block
    def text(s):
        return bytes([len(s)]) + s.encode()
    def rec(bi, bj, val):
        key = struct.pack(">qq", bi, bj)
        return struct.pack(">ii", len(key) + len(val), len(key)) + key + val
    dense = struct.pack(">iib", 2, 3, 3) + struct.pack(">6d", 1, 2, 3, 4, 5, 6)
    sparse = struct.pack(">iib", 2, 2, 2) + struct.pack(">i", 1) + struct.pack(">i", 0) + \
        struct.pack(">i", 1) + struct.pack(">id", 1, 9.0)
    body = b"SEQ\x06" + text(BB.KEY_CLASS) + text(BB.VALUE_CLASS) + b"\x00\x00" + struct.pack(">i", 0) + \
        b"S" * 16 + rec(1, 1, dense) + struct.pack(">i", -1) + b"S" * 16 + rec(1, 2, sparse)
    q = tmp_path / "B"
    q.write_bytes(body)
    got = BB.read_binary_block(str(q), 2, 5, brlen=2, bclen=3)
    np.testing.assert_array_equal(got, [[1, 2, 3, 0, 0], [4, 5, 6, 0, 9]])


def test_native_text_writers_match_java_formatting(tmp_path):
    """Native csv / ijv writers (ops/csrc/fastio.cpp) format cells exactly like
    java.lang.Double.toString (runtime/scalars.java_double_str), special values included."""
    from systemml_amd.ops import native
    from systemml_amd.runtime.scalars import java_double_str
    if native.lib() is None:
        pytest.skip("native library not built")
    rng = np.random.default_rng(8)
    a = rng.standard_normal((700, 9)) * 10.0 ** rng.integers(-15, 15, (700, 9))
    a[rng.random(a.shape) < 0.3] = 0.0
    a[0, :6] = [np.nan, np.inf, -np.inf, -0.0, 1e7, 1e-3]
    a[1, :4] = [9999999.0, 0.00099999, 5e-324, 1.7976931348623157e308]
    native.write_cells(tmp_path / "a.csv", a, 0)
    rows = (tmp_path / "a.csv").read_text().splitlines()
    assert rows == [",".join(java_double_str(float(v)) for v in r) for r in a]
    native.write_cells(tmp_path / "a.txt", a, 1)
    i, j = np.nonzero(a)
    want = [f"{ii + 1} {jj + 1} {java_double_str(float(a[ii, jj]))}" for ii, jj in zip(i, j)]
    assert (tmp_path / "a.txt").read_text().splitlines() == want


def test_mlresults_frame_tuple_and_context_accessors():
    from systemml_amd.api.mlcontext import MLContext, Frame, Matrix, dml
    ml = MLContext(config=CFG)
    src = """
    X = matrix("1 2 3 4", rows=2, cols=2)
    F = as.frame(X)
    s = sum(X)
    name = "x"
    """
    r = ml.execute(dml(src).output("X", "F", "s", "name"))
    f = r.getFrame("F")
    assert isinstance(f, Frame) and f.shape == (2, 2)
    assert r.getFrameAs2DStringArray("F") == [["1.0", "2.0"], ["3.0", "4.0"]]
    X, F, s, name = r.getTuple("X", "F", "s", "name")
    assert isinstance(X, Matrix) and isinstance(F, Frame) and s == 10.0 and name == "x"
    np.testing.assert_array_equal(r.getMatrixAs2DDoubleArray("X"), [[1, 2], [3, 4]])
    (only,) = r.getTuple("s")
    assert only == 10.0
    with pytest.raises(TypeError):
        r.getFrame("X")
    ml.setStatisticsMaxHeavyHitters(7)
    assert ml.getStatisticsMaxHeavyHitters() == 7
    ml.resetConfig()
    assert ml.getStatisticsMaxHeavyHitters() == MLContext().getStatisticsMaxHeavyHitters()
    info = ml.info()
    assert info.property("Version") == ml.version()
    assert not ml.isStatistics() and not ml.isExplain()
