"""External functions bound to the reference's udf.lib class names (runtime/udf.py), called
from DML through `externalFunction ... implemented in (classname=...)`.  Reference tests:
test/integration/functions/external/{OrderTest, DynProjectTest, ...}; CumSumProd's semantics
from udf/lib/CumSumProd.java (Y[i] = X[i] + C[i] * Y[i-1])."""
import numpy as np

from systemml_amd.api.executor import run
from systemml_amd.conf import DMLConfig

DECL = """
cumsumprod = externalFunction(Matrix[Double] X, Matrix[Double] C, Double start) return (Matrix[Double] Y)
  implemented in (classname="org.apache.sysml.udf.lib.CumSumProd", execlocation="master")
orderExt = externalFunction(Matrix[Double] A, Integer col, Boolean desc) return (Matrix[Double] B)
  implemented in (classname="org.apache.sysml.udf.lib.OrderWrapper")
"""


def _run(src, ins, outs):
    return run(DECL + src, inputs=ins, outputs=outs, config=DMLConfig(gpu=False), out=lambda s: None)


def test_cumsumprod_matches_the_recurrence():
    rng = np.random.default_rng(4)
    for n in (1, 2, 5, 1000, 4097):
        x, c = rng.standard_normal((n, 1)), rng.random((n, 1))
        res = _run("Y = cumsumprod(X, C, 0.25)", {"X": x, "C": c}, ["Y"])
        y, prev = np.zeros(n), 0.25
        for i in range(n):
            prev = x[i, 0] + c[i, 0] * prev
            y[i] = prev
        np.testing.assert_allclose(np.asarray(res["Y"]).reshape(-1), y, rtol=1e-12, atol=1e-12)


def test_order_wrapper_sorts_rows_by_column():
    A = np.array([[3.0, 1], [1, 2], [2, 3], [1, 4]])
    res = _run("B = orderExt(A, 1, FALSE)\nD = orderExt(A, 2, TRUE)", {"A": A}, ["B", "D"])
    np.testing.assert_array_equal(np.asarray(res["B"]), A[np.argsort(A[:, 0], kind="stable")])
    np.testing.assert_array_equal(np.asarray(res["D"]), A[::-1])
