"""`import systemml as sml` compatibility package: the Python API names of the reference
(src/main/python/systemml/__init__.py — mlcontext, defmatrix, converters, random, mllearn)
served by systemml_amd.  No Spark is needed: the `sc` / `sparkSession` arguments of the
reference signatures are accepted and ignored."""
from systemml_amd.api.mlcontext import (MLContext, MLResults, Script, Matrix, dml, pydml,  # noqa: F401
                                        dmlFromFile, pydmlFromFile, dmlFromResource)
from systemml_amd.api.mlcontext import getHopDAG, pydmlFromResource  # noqa: F401
from systemml_amd.api.defmatrix import matrix, eval, solve, full, seq, load, set_lazy, reset  # noqa: F401
from systemml_amd.api.converters import *  # noqa: F401,F403
from systemml_amd.api import converters as _conv
from . import random, mllearn  # noqa: F401


def setSparkContext(sc):
    """Accepted for source compatibility; execution does not use Spark."""
    return None


def debug_array_conversion(throwError):
    return None


__all__ = (["MLResults", "MLContext", "Script", "Matrix", "dml", "pydml", "dmlFromFile", "pydmlFromFile",
            "dmlFromResource", "pydmlFromResource", "getHopDAG", "matrix", "eval", "solve", "full", "seq",
            "load", "set_lazy", "reset", "setSparkContext", "debug_array_conversion"] + list(_conv.__all__))
