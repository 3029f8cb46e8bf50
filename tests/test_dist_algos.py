"""Algorithm scripts SPMD over 2 and 4 `gloo` ranks (CPU) against one process: ALS-CG
(sparse ratings, weighted quaternary ops), Kmeans, GLM (Poisson/log), L2SVM and
MultiLogReg with icpt=2 (scale & shift) must produce the single-process outputs while no
operator all-gathers a row-partitioned operand (fallback_gathers == 0).  Unseeded rand /
sample draw from the run's agreed seed sequence (sysml.random.seed), so both executions
see the same initialisation.  Reference analogue: the HYBRID_SPARK runs of
test/integration/applications/{als,kmeans,glm,l2svm,multilogreg}."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ALGOS = ["ALS-CG", "Kmeans", "GLM", "l2-svm", "MultiLogReg"]


@pytest.mark.parametrize("world", [2, 4])
def test_algorithms_spmd_match_single_process(world, tmp_path):
    from tools.dist_probe import probe
    ref, got, res, errs1 = probe(ALGOS, world=world, minrows=50, d=str(tmp_path), n=600)
    assert not errs1, errs1
    for rank, per, errs in res:
        assert not errs, errs
        for name, (st, sites) in per.items():
            assert st["fallback_gathers"] == 0, (rank, name, sites)
            assert st["allreduce"] > 0, (rank, name)
    assert set(ref) == set(got) and len(ref) >= 5, (sorted(ref), sorted(got))
    for k in ref:
        np.testing.assert_allclose(got[k], ref[k], rtol=1e-8, atol=1e-9, err_msg=k)
