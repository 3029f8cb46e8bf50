"""The algorithm library on the GPU backend against the CP backend (reference analogue: the
GPU variants of test/integration/applications/*, which compare the GPU run of a script with
its CP run): every output matrix of the deterministic algorithms must match the host fp64
results when the GPU backend computes in fp64 (HBM-resident operands, HIP kernels, hybrid
placement of small operands)."""
import glob
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OURS = os.path.join(HERE, "systemml_amd", "scripts", "algorithms")
ALGOS = ["LinearRegCG", "LinearRegDS", "GLM", "GLM-predict", "MultiLogReg", "l2-svm", "l2-svm-predict", "m-svm",
         "m-svm-predict", "naive-bayes", "naive-bayes-predict", "PCA", "Univar-Stats", "bivar-stats", "stratstats",
         "KM", "Cox", "CsplineCG", "CsplineDS", "StepLinearRegDS"]
# ALS-CG is left out: its unseeded random initialisation is drawn on the device by the GPU
# backend, so the two runs start from different factors (tests/test_quaternary.py covers its
# fused operators on both backends)


def _read(path):
    from systemml_amd.io import readers
    v = readers.read(None, path)
    if hasattr(v, "to_matrix"):
        v = v.to_matrix()
    return np.asarray(v.cpu().double().numpy() if hasattr(v, "cpu") else v, dtype=float)


@pytest.mark.gpu
def test_algorithm_library_gpu_matches_cp(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sys.path.insert(0, os.path.join(HERE, "tools"))
    import run_algos as RA
    from systemml_amd.conf import DMLConfig
    from systemml_amd.ops import kernels
    d = str(tmp_path)
    RA.make_data(d, n=400)
    cp = RA.run_suite(OURS, d, out_dir=d + "/out_cp", only=ALGOS)
    k0 = sum(kernels.counters.values())
    gpu = RA.run_suite(OURS, d, out_dir=d + "/out_gpu", only=ALGOS,
                       config=DMLConfig(gpu=True, precision="double", gpu_min_cells=0))
    failed = {k: f"{type(e).__name__}: {e}" for k, e in gpu.items() if e is not None}
    assert not failed, failed
    assert not {k: e for k, e in cp.items() if e is not None}
    assert sum(kernels.counters.values()) > k0          # HIP kernels ran
    mism, compared = [], 0
    for mtd in sorted(glob.glob(d + "/out_cp/**/*.mtd", recursive=True)):
        f = mtd[:-4]
        rel = os.path.relpath(f, d + "/out_cp")
        other = os.path.join(d + "/out_gpu", rel)
        try:
            a, b = _read(f), _read(other)
        except Exception:   # noqa: BLE001 -- string frames
            continue
        compared += 1
        if rel.startswith("pca"):
            a, b = np.abs(a), np.abs(b)        # eigenvectors (and projections) up to sign
        if a.shape != b.shape:
            mism.append(f"{rel}: shape {a.shape} vs {b.shape}")
        elif not np.allclose(a, b, rtol=1e-6, atol=1e-8 * (np.nanmax(np.abs(a)) + 1), equal_nan=True):
            mism.append(f"{rel}: max |diff| {np.nanmax(np.abs(a - b)):.3g}")
    assert compared >= 15, compared
    assert not mism, "\n".join(mism)
