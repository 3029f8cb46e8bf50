"""Lazy numpy-like DML DSL (reference: src/main/python/tests/test_matrix_*.py compare
defmatrix results with numpy)."""
import numpy as np

import systemml_amd.api.defmatrix as sml
from systemml_amd.conf import DMLConfig

sml.set_config(DMLConfig(gpu=False))


def test_arithmetic_and_aggregates_match_numpy():
    rng = np.random.default_rng(0)
    A = rng.random((5, 4))
    B = rng.random((4, 3))
    m = sml.matrix(A)
    expr = ((m @ B) * 2 + 1).sum(axis=1)
    np.testing.assert_allclose(expr.toNumPy().ravel(), ((A @ B) * 2 + 1).sum(1))
    np.testing.assert_allclose(float(m.sum()), A.sum())
    np.testing.assert_allclose(m.mean(axis=0).toNumPy().ravel(), A.mean(0))
    np.testing.assert_allclose((1 - m).exp().toNumPy(), np.exp(1 - A))
    np.testing.assert_allclose(m.T.toNumPy(), A.T)
    np.testing.assert_allclose(m[1:3, 0:2].toNumPy(), A[1:3, 0:2])
    np.testing.assert_allclose((m > 0.5).toNumPy(), (A > 0.5).astype(float))
    np.testing.assert_allclose(np.asarray(sml.hstack(m, m)), np.hstack([A, A]))
    np.testing.assert_allclose(m.argmax().toNumPy().ravel(), A.argmax(1) + 1)


def test_solve_seq_full_and_setitem():
    rng = np.random.default_rng(1)
    A = rng.random((4, 4)) + 4 * np.eye(4)
    b = rng.random((4, 1))
    x = sml.solve(sml.matrix(A), sml.matrix(b))
    np.testing.assert_allclose(x.toNumPy(), np.linalg.solve(A, b))
    np.testing.assert_allclose(sml.seq(5).toNumPy().ravel(), np.arange(6))      # stop included (reference)
    z = sml.full((2, 3), 7)
    z[0, 1] = 0
    np.testing.assert_allclose(z.toNumPy(), [[7, 0, 7], [7, 7, 7]])
