"""The reference's own Python API tests, unmodified, against the `systemml` package here.

src/main/python/tests/test_matrix_agg_fn.py, test_matrix_binary_op.py and test_mlcontext.py
(the lazy `matrix` DSL's aggregates / binary operators against numpy, and the MLContext
script / input / output API) import pyspark only to create a SparkContext and to turn lists of
CSV lines into RDDs.  pyspark is not installed here, so a stand-in module provides those two
handles (`parallelize` returns the lines, which MLContext accepts as the no-Spark form of an
RDD<String> CSV input); everything else is the reference test code as shipped.

Not covered (parity unpinned): test_matrix_toDF compares the repr of a *Spark* DataFrame;
test_mllearn_*.py need pyspark.ml and test_nn_numpy.py needs keras (neither installed) --
tests/test_mllearn.py covers the estimators against the same sklearn references instead.
"""
import importlib.util
import os
import sys
import types
import unittest

import pytest

REF = "/root/reference/src/main/python/tests"
SKIP = {"test_mlcontext.TestAPI.test_matrix_toDF"}


class _RDDContext:
    @staticmethod
    def getOrCreate(*a, **k):
        return _RDDContext()

    def parallelize(self, lines, *a, **k):
        return list(lines)


def _stand_in():
    ps = types.ModuleType("pyspark")
    ctx = types.ModuleType("pyspark.context")
    ctx.SparkContext = _RDDContext
    ps.SparkContext = _RDDContext
    ps.context = ctx
    return {"pyspark": ps, "pyspark.context": ctx}


@pytest.mark.parametrize("name", ["test_matrix_agg_fn", "test_matrix_binary_op", "test_mlcontext"])
def test_reference_python_api_suite(name, monkeypatch):
    path = os.path.join(REF, name + ".py")
    if not os.path.exists(path):
        pytest.skip("reference sources not mounted")
    for k, v in _stand_in().items():
        monkeypatch.setitem(sys.modules, k, v)
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    monkeypatch.syspath_prepend(here)
    # the reference test puts ITS package directory first on sys.path: bind `systemml` (and its
    # submodules) to this repository's package before the module executes
    import systemml
    assert os.path.dirname(os.path.dirname(os.path.abspath(systemml.__file__))) == here
    for k in [m for m in sys.modules if m == "systemml" or m.startswith("systemml.")]:
        monkeypatch.setitem(sys.modules, k, sys.modules[k])
    monkeypatch.setattr(sys, "path", list(sys.path))      # the module's own sys.path insert is undone
    spec = importlib.util.spec_from_file_location("ref_" + name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    suite = unittest.TestSuite()
    for t in unittest.defaultTestLoader.loadTestsFromModule(mod):
        for case in (t if isinstance(t, unittest.TestSuite) else [t]):
            if case.id().split(".", 1)[1] not in SKIP and not case.id().endswith(tuple(SKIP)):
                suite.addTest(case)
    res = unittest.TextTestRunner(verbosity=0, stream=open(os.devnull, "w")).run(suite)
    bad = [(t.id(), tb.strip().splitlines()[-1]) for t, tb in res.failures + res.errors]
    assert res.testsRun > 0 and not bad, bad
