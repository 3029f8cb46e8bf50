"""Staging scripts (scripts/staging, reference scripts/staging/*): each runs at a small
size on the CP backend and is checked against a numpy/scipy reference of the same
computation (the reference ships no expected outputs for these)."""
import os

import numpy as np
import pytest
import torch

from systemml_amd.api.executor import run
from systemml_amd.api.mlcontext import SCRIPTS_DIR
from systemml_amd.conf import DMLConfig
from systemml_amd.io.readers import read_matrix
from systemml_amd.io.writers import write_matrix

CFG = DMLConfig(gpu=False)
ST = os.path.join(SCRIPTS_DIR, "staging")


def staging(name, args=None, src=None, outputs=(), inputs=None):
    path = os.path.join(ST, name if src is None else "_inline.dml")
    out = []
    res = run(src if src is not None else open(path).read(), args=args or {}, inputs=inputs or {}, outputs=outputs,
              config=CFG, out=out.append, filename=path)
    return {k: (v.numpy() if hasattr(v, "numpy") else v) for k, v in res.items()}, out


def wr(path, a):
    write_matrix(torch.from_numpy(np.asarray(a, dtype=np.float64)), str(path), "csv")
    return str(path)


def rd(p):
    return read_matrix(str(p)).numpy()


def test_scalable_linalg_decompositions():
    rng = np.random.default_rng(0)
    A = rng.standard_normal((13, 13))
    S = A @ A.T + 13 * np.eye(13)
    b = rng.standard_normal((13, 2))
    src = ('source("scalable_linalg/linalg_decomp.dml") as D\n'
           "L = D::Cholesky(S, 3)\n[P, Lu, U] = D::LU(A, 4)\n[Q, R] = D::QR(T, 3)\n"
           "Ai = D::Inverse(A, 4)\nx = D::Solve(A, b, 4)\nLi = D::L_triangular_inv(L)\n")
    T = rng.standard_normal((20, 9))
    r, _ = staging("scalable_linalg/linalg_decomp.dml", src=src, inputs=dict(S=S, A=A, b=b, T=T),
                   outputs=("L", "P", "Lu", "U", "Q", "R", "Ai", "x", "Li"))
    np.testing.assert_allclose(r["L"], np.linalg.cholesky(S), atol=1e-10)
    np.testing.assert_allclose(r["P"] @ A, r["Lu"] @ r["U"], atol=1e-9)
    assert np.allclose(np.tril(r["Lu"]), r["Lu"]) and np.allclose(np.triu(r["U"]), r["U"])
    np.testing.assert_allclose(r["Q"] @ r["R"], T, atol=1e-10)
    np.testing.assert_allclose(r["Q"].T @ r["Q"], np.eye(9), atol=1e-10)
    np.testing.assert_allclose(r["Ai"], np.linalg.inv(A), atol=1e-8)
    np.testing.assert_allclose(r["x"], np.linalg.solve(A, b), atol=1e-8)
    np.testing.assert_allclose(r["Li"], np.linalg.inv(np.linalg.cholesky(S)), atol=1e-10)


def test_qr_recursive_and_lanczos(tmp_path):
    rng = np.random.default_rng(1)
    X = rng.standard_normal((30, 7))
    staging("QR_recursive.dml", dict(X=wr(tmp_path / "X", X), k=2, OUTDIR=str(tmp_path) + "/", OFMT="csv"))
    Q, R = rd(tmp_path / "Q.csv"), rd(tmp_path / "R.csv")
    np.testing.assert_allclose(Q @ R, X, atol=1e-10)
    B = rng.standard_normal((12, 12))
    A = B + B.T
    staging("Lanczos.dml", {"1": wr(tmp_path / "A", A), "2": str(tmp_path / "ev"), "3": str(tmp_path / "V")})
    ev, V = rd(tmp_path / "ev").ravel(), rd(tmp_path / "V")
    np.testing.assert_allclose(np.sort(ev), np.linalg.eigvalsh(A), atol=1e-8)
    np.testing.assert_allclose(A @ V, V * ev, atol=1e-7)


def test_pnmf_decreases_objective(tmp_path):
    rng = np.random.default_rng(2)
    X = rng.poisson(3, (25, 15)).astype(float)
    W0, H0 = rng.random((25, 3)) + 0.1, rng.random((3, 15)) + 0.1
    _, out = staging("PNMF.dml", {"1": wr(tmp_path / "X", X), "2": wr(tmp_path / "W", W0), "3": wr(tmp_path / "H", H0),
                                  "4": 3, "5": 1e-8, "6": 30, "7": str(tmp_path / "Wo"), "8": str(tmp_path / "Ho")})
    objs = [float(s.split("obj=")[1]) for s in out if "obj=" in s]
    assert len(objs) == 29 and all(b <= a + 1e-9 for a, b in zip(objs, objs[1:]))
    assert (rd(tmp_path / "Wo") >= 0).all()


def test_ppca_and_pca(tmp_path):
    rng = np.random.default_rng(3)
    Z = rng.standard_normal((300, 2))
    X = Z @ rng.standard_normal((2, 6)) * 3 + 0.1 * rng.standard_normal((300, 6))
    staging("PPCA.dml", dict(X=wr(tmp_path / "X", X), C=str(tmp_path / "C"), V=str(tmp_path / "V"), k=2, iter=50,
                             tolrecerr=0.0, tolobj=1e-12))
    C = rd(tmp_path / "C")
    # the PPCA loadings span the principal subspace
    U = np.linalg.svd(X - X.mean(0), full_matrices=False)[2][:2].T
    Qc = np.linalg.qr(C)[0]
    assert np.linalg.norm(Qc - U @ (U.T @ Qc)) < 0.05
    V = rd(tmp_path / "V").ravel()
    assert V[0] >= V[1]
    staging("PCA.dml", dict(INPUT=str(tmp_path / "X"), K=2, CENTER=1, OUTPUT=str(tmp_path), OFMT="csv", PROJDATA=1))
    ev = rd(tmp_path / "dominant.eigen.values").ravel()
    np.testing.assert_allclose(ev, np.sort(np.linalg.eigvalsh(np.cov(X.T)))[::-1][:2], rtol=1e-8)
    assert rd(tmp_path / "projected.data").shape == (300, 2)


def test_rbm_train_and_predict(tmp_path):
    rng = np.random.default_rng(4)
    X = (rng.random((200, 8)) < 0.3).astype(float)
    _, out = staging("rbm_minibatch.dml", dict(X=wr(tmp_path / "X", X), W=str(tmp_path / "W"), A=str(tmp_path / "A"),
                                               B=str(tmp_path / "B"), hid=3, epochs=5, batchsize=50))
    errs = [float(s.split("is ")[1]) for s in out if "Cumulative error" in s]
    assert len(errs) == 5 and errs[-1] < errs[0]
    staging("rbm_predict.dml", dict(X=str(tmp_path / "X"), W=str(tmp_path / "W"), A=str(tmp_path / "A"),
                                    B=str(tmp_path / "B"), O=str(tmp_path / "H")))
    H = rd(tmp_path / "H")
    assert H.shape == (200, 3) and set(np.unique(H)) <= {0, 1}


def test_knn_search_prediction_and_selection(tmp_path):
    rng = np.random.default_rng(5)
    P = np.vstack([rng.normal(0, 1, (40, 3)), rng.normal(6, 1, (40, 3))])
    y = np.repeat([1.0, 2.0], 40)[:, None]
    Q = np.vstack([rng.normal(0, 1, (5, 3)), rng.normal(6, 1, (5, 3))])
    a = dict(X=wr(tmp_path / "P", P), T=wr(tmp_path / "Q", Q), Y=wr(tmp_path / "y", y), Y_T=wr(tmp_path / "yt", [[2]]),
             NNR=str(tmp_path / "NNR"), PR=str(tmp_path / "PR"), k_value=4)
    staging("knn.dml", a)
    NNR = rd(tmp_path / "NNR")
    D = ((Q[:, None, :] - P[None]) ** 2).sum(-1)
    np.testing.assert_array_equal(NNR, np.argsort(D, axis=1)[:, :4] + 1)
    np.testing.assert_array_equal(rd(tmp_path / "PR").ravel(), np.repeat([1, 2], 5))
    _, out = staging("knn.dml", dict(a, select_k=1, k_min=1, k_max=6, select_feature=1, feature_max=2,
                                     FEATURE_SELECTED=str(tmp_path / "fs")))
    assert any("LOOCV" in s for s in out) and rd(tmp_path / "fs").sum() >= 1


def test_lasso_matches_coordinate_descent(tmp_path):
    rng = np.random.default_rng(6)
    X = rng.standard_normal((60, 8))
    w_true = np.array([3, 0, 0, -2, 0, 0, 1, 0.0])
    y = X @ w_true + 0.1 * rng.standard_normal(60)
    staging("regression/lasso/lasso.dml", dict(X=wr(tmp_path / "X", X), Y=wr(tmp_path / "y", y[:, None]),
                                               model=str(tmp_path / "w"), tau=5.0, maxi=500))
    w = rd(tmp_path / "w").ravel()
    # coordinate-descent optimum of 0.5||Xw-y||^2 + 5||w||_1
    v = np.zeros(8)
    for _ in range(2000):
        for j in range(8):
            r = y - X @ v + X[:, j] * v[j]
            rho = X[:, j] @ r
            v[j] = np.sign(rho) * max(abs(rho) - 5.0, 0) / (X[:, j] @ X[:, j])
    np.testing.assert_allclose(w, v, atol=1e-5)


def test_gaussian_process_mode_and_covariance():
    r, out = staging("gaussian_process/mode.dml", outputs=("f",))
    f = r["f"].ravel()
    K = np.array([[9.9090, 4.3453, -2.0279, 2.0109, 4.3453], [4.3453, 9.6392, 0.8006, 4.6520, 9.6392],
                  [-2.0279, 0.8006, 4.6162, 0.7838, 0.8006], [2.0109, 4.6520, 0.7838, 6.4825, 4.6520],
                  [4.3453, 9.6392, 0.8006, 4.6520, 9.6392]])
    y = np.array([-1, 1, 1, -1, -1.0])
    # stationarity of the Laplace mode: f = K grad log p(y|f)
    np.testing.assert_allclose(f, K @ ((y + 1) / 2 - 1 / (1 + np.exp(-f))), atol=1e-8)
    X = np.random.default_rng(7).standard_normal((6, 3))
    r, _ = staging("gaussian_process/covariance.dml", src='source("gaussian_process/covariance.dml") as G\nK = G::cov(X)',
                   inputs=dict(X=X), outputs=("K",))
    np.testing.assert_allclose(r["K"], np.exp(-0.5 * ((X[:, None] - X[None]) ** 2).sum(-1)), atol=1e-12)


def test_autoencoder_reduces_reconstruction(tmp_path):
    X = np.random.default_rng(8).standard_normal((64, 6))
    a = dict(X=wr(tmp_path / "X", X), H1=4, H2=2, EPOCH=6, BATCH=16, STEP=0.05, OBJ=True, HIDDEN=str(tmp_path / "H"),
             fmt="csv")
    for i in range(1, 5):
        a[f"W{i}_out"], a[f"b{i}_out"] = str(tmp_path / f"W{i}"), str(tmp_path / f"b{i}")
    _, out = staging("autoencoder-2layer.dml", a)
    full = [float(s.split("=")[-1]) for s in out if "FULL DATA" in s]
    assert len(full) == 6 and full[-1] < full[0]
    assert rd(tmp_path / "H").shape == (64, 2) and rd(tmp_path / "W1").shape == (4, 6)


@pytest.mark.parametrize("kind", ["binclass", "regression"])
def test_factorization_machines(kind):
    rng = np.random.default_rng(9)
    X = rng.random((100, 5))
    y = X @ np.array([[1.0], [-2], [0.5], [0], [1]])
    if kind == "binclass":
        y = (y > np.median(y)).astype(float)
    src = (f'source("fm-{kind}.dml") as M\n'
           + ("[w0, W, V, loss] = M::train(X, y, X, y)\n" if kind == "binclass" else "[w0, W, V] = M::train(X, y, X, y)\n")
           + "p = M::predict(X, w0, W, V)\n")
    r, _ = staging(f"fm-{kind}.dml", src=src, inputs=dict(X=X, y=y), outputs=("p",))
    p = r["p"]
    if kind == "binclass":
        assert ((p > 0.5) == (y > 0.5)).mean() > 0.8
    else:
        assert np.mean((p - y) ** 2) < 0.5 * np.var(y)


def test_lenet_train_staging(tmp_path):
    rng = np.random.default_rng(10)
    n, nt = 40, 10
    y = rng.integers(0, 3, (n + nt, 1)).astype(float)
    X = np.zeros((n + nt, 64))
    X[np.arange(n + nt), (y[:, 0] * 20 + 3).astype(int)] = 255       # class-dependent bright pixel
    _, out = staging("lenet-train.dml", dict(X=wr(tmp_path / "X", X[:n]), Y=wr(tmp_path / "y", y[:n]),
                                             Xt=wr(tmp_path / "Xt", X[n:]), Yt=wr(tmp_path / "yt", y[n:]),
                                             FMAPS1=2, FMAPS2=2, NODES=8, lambda_=0, epochs=1, batch=10,
                                             validation=10, Hin=8, Win=8, classes=3, step=0.05)
                     | {"lambda": 0})
    assert any("Final accuracy on test set" in s for s in out)
