"""Utility scripts (scripts/utils, reference scripts/utils/*.dml) checked against numpy."""
import os

import numpy as np
import pandas as pd
import torch

from systemml_amd.api.executor import run
from systemml_amd.api.mlcontext import SCRIPTS_DIR
from systemml_amd.conf import DMLConfig
from systemml_amd.io.readers import read_matrix
from systemml_amd.io.writers import write_matrix

CFG = DMLConfig(gpu=False)
UT = os.path.join(SCRIPTS_DIR, "utils")


def util(name, args=None, src=None, inputs=None, outputs=()):
    path = os.path.join(UT, name if src is None else "_inline.dml")
    out = []
    res = run(src if src is not None else open(path).read(), args=args or {}, inputs=inputs or {}, outputs=outputs,
              config=CFG, out=out.append, filename=path)
    return {k: (v.numpy() if hasattr(v, "numpy") else v) for k, v in res.items()}, out


def wr(p, a):
    write_matrix(torch.from_numpy(np.asarray(a, dtype=np.float64)), str(p), "csv")
    return str(p)


def rd(p):
    return read_matrix(str(p)).numpy()


X = np.arange(1, 31, dtype=float).reshape(6, 5)


def test_format_head_rowindexmax_generate(tmp_path):
    t = tmp_path
    util("csv2bin.dml", dict(csv=wr(t / "X", X), bin=str(t / "B")))
    np.testing.assert_array_equal(rd(t / "B"), X)
    util("write.dml", dict(I=str(t / "B"), O=str(t / "W"), ofmt="csv", sep="|", header=True))
    assert open(t / "W").readline().strip().startswith("C1|")
    util("head.dml", dict(x=str(t / "X"), n=2, o=str(t / "H")))
    np.testing.assert_array_equal(rd(t / "H"), X[:2])
    M = np.array([[1, 5, 2], [7, 7, 0.0]])
    util("rowIndexMax.dml", dict(I=wr(t / "M", M), O=str(t / "R")))
    assert rd(t / "R")[0, 0] == 2
    util("generateData.dml", dict(R=50, C=4, S=0.5, Min=1, Max=3, Path=str(t / "G")))
    G = rd(t / "G")
    assert G.shape == (50, 4) and G[G != 0].min() >= 1 and G.max() <= 3


def test_shuffle_project_split(tmp_path):
    t = tmp_path
    util("shuffle.dml", dict(x=wr(t / "X", X), o=str(t / "S")))
    S = rd(t / "S")
    assert sorted(map(tuple, S)) == sorted(map(tuple, X))
    util("project.dml", dict(X=str(t / "X"), P=wr(t / "P", [[4], [2]]), o=str(t / "PX"), ofmt="csv"))
    np.testing.assert_array_equal(rd(t / "PX"), X[:, [3, 1]])
    util("project.dml", dict(X=str(t / "X"), P=str(t / "P"), o=str(t / "EX"), exclude=True, ofmt="csv"))
    np.testing.assert_array_equal(rd(t / "EX"), X[:, [0, 2, 4]])
    util("splitXY.dml", dict(X=str(t / "X"), y=3, OX=str(t / "OX"), OY=str(t / "OY"), ofmt="csv"))
    np.testing.assert_array_equal(rd(t / "OX"), X[:, [0, 1, 3, 4]])
    np.testing.assert_array_equal(rd(t / "OY"), X[:, [2]])
    util("splitXY-dummy.dml", dict(X=str(t / "X"), S=2, N=2, OX=str(t / "DX"), OY=str(t / "DY"), ofmt="csv"))
    np.testing.assert_array_equal(rd(t / "DX"), X[:, [0, 3, 4]])
    np.testing.assert_array_equal(rd(t / "DY"), X[:, [1, 2]])


def test_sample_disjoint_subsets(tmp_path):
    t = tmp_path
    Y = np.arange(1, 201, dtype=float)[:, None]
    util("sample.dml", dict(X=wr(t / "Y", Y), sv=wr(t / "sv", [[0.5], [0.3], [0.2]]), O=str(t / "out"), ofmt="csv"))
    parts = [rd(t / "out" / str(i)).ravel() for i in (1, 2, 3)]
    allv = np.concatenate(parts)
    assert len(allv) == 200 and len(np.unique(allv)) == 200
    assert 70 < len(parts[0]) < 130


def test_metrics_image_and_dataprep():
    yt = np.array([[1, 2, 2, 3, 3, 3.0]]).T
    yp = np.array([[1, 2, 3, 3, 3, 1.0]]).T
    src = 'source("metrics.dml") as M\nout = M::classification_report(yt, yp, seq(1, 3))\nC = M::confusion_matrix(yt, yp, 3)\n'
    r, _ = util("metrics.dml", src=src, inputs=dict(yt=yt, yp=yp), outputs=("out", "C"))
    rows = [list(map(float, l.split())) for l in r["out"].strip().split("\n")[1:]]
    np.testing.assert_allclose(rows[0], [1, 0.5, 1.0, 2 / 3, 1], atol=1e-6)
    np.testing.assert_allclose(rows[2], [3, 2 / 3, 2 / 3, 2 / 3, 3], atol=1e-6)
    np.testing.assert_array_equal(r["C"], [[1, 0, 0], [0, 1, 1], [1, 0, 2]])
    img = np.arange(2 * 3 * 6 * 6, dtype=float).reshape(2, 3 * 36)
    src = 'source("image_utils.dml") as I\nG = I::crop_grayscale(Xg, 6, 6, 4, 2)\nR = I::crop_rgb(X, 6, 6, 2, 2)\n'
    r, _ = util("image_utils.dml", src=src, inputs=dict(X=img, Xg=img[:, :36]), outputs=("G", "R"))
    # the reference's crop window starts at 1-based ceil((Hin-Hout)/2) (kept for parity)
    np.testing.assert_array_equal(r["G"], img[:, :36].reshape(2, 6, 6)[:, 0:4, 1:3].reshape(2, -1))
    np.testing.assert_array_equal(r["R"], img.reshape(2, 3, 6, 6)[:, :, 1:3, 1:3].reshape(2, -1))
    F = pd.DataFrame({"u": ["a", "b", "a", "c", "a"], "p": ["x", "x", "y", "y", "z"], "r": [5, 3, 4, 2, 1]})
    src = 'source("dataprep.dml") as D\n[X, M] = D::convertToRatingsMatrix(F, 2, 0)\n'
    r, _ = util("dataprep.dml", src=src, inputs=dict(F=F), outputs=("X",))
    assert r["X"].shape[0] == 1 and sorted(r["X"].ravel()) == [1, 4, 5]
