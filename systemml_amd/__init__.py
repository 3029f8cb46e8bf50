"""systemml_amd — an MI355X-native declarative machine learning engine with the
language, APIs and algorithm library of Apache SystemML (nakul02/systemml).

DML/PyDML scripts are parsed, compiled through a HOP/LOP-style optimizer
(rewrites, operator fusion, liveness) and executed on host (CP), on a single
MI355X (HBM-resident matrices + hand-written HIP kernels) or SPMD across the
GPUs of a node (row-partitioned matrices + RCCL collectives).
"""
__version__ = "0.1.0"

from .api.mlcontext import MLContext, Script, dml, pydml, dmlFromFile, pydmlFromFile, dmlFromResource  # noqa: E402,F401
from .conf import DMLConfig  # noqa: E402,F401
