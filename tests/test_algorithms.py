"""Algorithm library tests on the CP backend (reference: test/integration/applications/*Test
which compare DML results against R; here against numpy/scipy/sklearn references)."""
import os

import numpy as np
import pytest

from systemml_amd.api.executor import run
from systemml_amd.api.mlcontext import SCRIPTS_DIR
from systemml_amd.conf import DMLConfig

CFG = DMLConfig(gpu=False, seed=5)   # unseeded rand() in the scripts (ALS inits) draws from this


def algo(name, args, inputs, outputs):
    path = os.path.join(SCRIPTS_DIR, "algorithms", name + ".dml")
    with open(path) as f:
        src = f.read()
    out = []
    res = run(src, args=args, inputs=inputs, outputs=outputs, config=CFG, out=out.append, filename=path)
    return {k: (v.numpy() if hasattr(v, "numpy") else v) for k, v in res.items()}, out


@pytest.fixture(scope="module")
def reg_data():
    rng = np.random.default_rng(0)
    X = rng.standard_normal((300, 6)) * 2 + 1
    y = X @ rng.standard_normal((6, 1)) + 0.5 + 0.05 * rng.standard_normal((300, 1))
    return X, y


@pytest.mark.parametrize("icpt", [0, 1, 2])
@pytest.mark.parametrize("name", ["LinearRegCG", "LinearRegDS"])
def test_linear_regression(reg_data, name, icpt):
    X, y = reg_data
    r, out = algo(name, dict(X="X", Y="y", B="B", icpt=icpt, reg=1e-9, tol=1e-12, maxi=200),
                  {"X": X, "y": y}, ["beta"])
    Xi = X if icpt == 0 else np.hstack([X, np.ones((300, 1))])
    np.testing.assert_allclose(r["beta"], np.linalg.lstsq(Xi, y, rcond=None)[0], atol=1e-7)
    assert any(s.startswith("AVG_TOT_Y") for s in "\n".join(out).split("\n"))


def test_multilogreg_matches_scipy_optimum():
    from scipy.optimize import minimize
    rng = np.random.default_rng(1)
    N, D, K = 500, 5, 3
    X = rng.standard_normal((N, D))
    y = (np.argmax(X @ rng.standard_normal((D, K)) + rng.standard_normal((N, K)), 1) + 1).reshape(-1, 1)
    r, _ = algo("MultiLogReg", dict(X="X", Y="Y", B="B", icpt=0, reg=0.1, tol=1e-12, moi=100, mii=0),
                {"X": X, "Y_vec": y.astype(float)}, ["B_out"])
    Y = np.eye(K)[y.ravel() - 1]

    def obj(b):
        B = b.reshape(D, K - 1)
        LT = np.hstack([X @ B, np.zeros((N, 1))])
        m = LT.max(1, keepdims=True)
        return -np.sum(Y * LT) + np.sum(m.ravel() + np.log(np.exp(LT - m).sum(1))) + 0.05 * np.sum(B ** 2)
    ref = minimize(obj, np.zeros(D * (K - 1)), method="BFGS", options=dict(gtol=1e-10, maxiter=5000))
    np.testing.assert_allclose(obj(r["B_out"].ravel()), ref.fun, rtol=1e-8)
    np.testing.assert_allclose(r["B_out"].ravel(), ref.x, atol=1e-4)


def test_l2svm_and_predict(tmp_path):
    rng = np.random.default_rng(2)
    X = rng.standard_normal((400, 4))
    y = np.where(X @ np.array([[1.0], [-2.0], [0.5], [0.0]]) > 0.2, 1.0, -1.0)
    r, _ = algo("l2-svm", dict(X="X", Y="Y", model="m", icpt=1, tol=1e-9, reg=0.01, maxiter=100),
                {"X": X, "Y": y}, ["model"])
    w = r["model"]
    assert w.shape == (4 + 1 + 4, 1)
    scores = X @ w[:4] + w[4]
    assert ((scores >= 0) == (y > 0)).mean() > 0.97


def test_msvm_matches_independent_l2svm():
    rng = np.random.default_rng(3)
    X = rng.standard_normal((300, 4))
    y = (np.argmax(X[:, :3], 1) + 1).reshape(-1, 1).astype(float)
    r, _ = algo("m-svm", dict(X="X", Y="Y", model="m", icpt=0, tol=1e-12, reg=0.1, maxiter=200),
                {"X": X, "Y": y}, ["W"])
    W = r["W"]
    for c in range(3):
        yc = np.where(y == c + 1, 1.0, -1.0)
        rb, _ = algo("l2-svm", dict(X="X", Y="Y", model="m", icpt=0, tol=1e-12, reg=0.1, maxiter=200),
                     {"X": X, "Y": yc}, ["w"])
        np.testing.assert_allclose(W[:, c:c + 1], rb["w"], rtol=1e-4, atol=1e-6)


def test_naive_bayes():
    rng = np.random.default_rng(4)
    X = rng.integers(0, 5, (200, 6)).astype(float)
    y = rng.integers(1, 4, (200, 1)).astype(float)
    r, _ = algo("naive-bayes", dict(X="X", Y="Y", prior="p", conditionals="c", laplace=1),
                {"X": X, "y": y}, ["prior", "cond"])
    for k in range(3):
        cnt = X[y.ravel() == k + 1].sum(0)
        np.testing.assert_allclose(r["cond"][k], (cnt + 1) / (cnt.sum() + 6))
        np.testing.assert_allclose(r["prior"][k, 0], (y == k + 1).mean())


def test_kmeans_finds_separated_clusters():
    rng = np.random.default_rng(5)
    centers = np.array([[0, 0], [10, 10], [-10, 10]])
    X = np.vstack([c + rng.standard_normal((100, 2)) for c in centers])
    r, _ = algo("Kmeans", dict(X="X", k=3, runs=3, maxi=50, C="C"), {"X": X}, ["best_C"])
    C = r["best_C"]
    for c in centers:
        assert np.min(np.linalg.norm(C - c, axis=1)) < 0.5


def test_pca_eigenvalues():
    rng = np.random.default_rng(6)
    A = rng.standard_normal((200, 5)) @ rng.standard_normal((5, 5))
    r, _ = algo("PCA", dict(INPUT="A", K=2, CENTER=1, OUTPUT="/tmp/_pca_test", PROJDATA=0), {"A": A}, ["lam"])
    w = np.sort(np.linalg.eigvalsh(np.cov(A.T)))[::-1]
    np.testing.assert_allclose(r["lam"].ravel(), w[:2], rtol=1e-10)


# ---------------------------------------------------------------------------
# GLM (reference: test/integration/applications/GLMTest compares against R's glm();
# here against a direct scipy minimisation of the same penalised deviance)
# ---------------------------------------------------------------------------
def _glm_data(kind, n=1500, m=4, seed=11):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, m))
    beta = rng.standard_normal((m, 1)) * 0.3
    eta = X @ beta + 0.5
    if kind == "gauss":
        y = eta + 0.1 * rng.standard_normal((n, 1))
    elif kind == "poisson":
        y = rng.poisson(np.exp(eta)).astype(float)
    elif kind == "gamma":
        y = rng.gamma(2.0, np.exp(eta) / 2.0)
    else:
        y = (rng.random((n, 1)) < 1 / (1 + np.exp(-eta))).astype(float)
    return X, y


def _glm_objective(kind, link, X, y, reg):
    from scipy.special import ndtr
    Xi = np.hstack([X, np.ones((X.shape[0], 1))])
    yv = y.ravel()

    def f(b):
        eta = Xi @ b
        if link == "log":
            mu = np.exp(eta)
        elif link == "id":
            mu = eta
        elif link == "logit":
            mu = 1 / (1 + np.exp(-eta))
        else:
            mu = ndtr(eta)
        if kind == "gauss":
            dev = np.sum((yv - mu) ** 2)
        elif kind == "poisson":
            dev = 2 * np.sum(np.where(yv > 0, yv * np.log(np.where(yv > 0, yv, 1) / mu), 0) - (yv - mu))
        elif kind == "gamma":
            dev = 2 * np.sum(-np.log(yv / mu) + (yv - mu) / mu)
        else:
            mu = np.clip(mu, 1e-300, 1 - 1e-16)
            dev = -2 * np.sum(yv * np.log(mu) + (1 - yv) * np.log(1 - mu))
        return 0.5 * dev + 0.5 * reg * np.sum(b[:-1] ** 2)
    return f


@pytest.mark.parametrize("kind,args,link", [
    ("gauss", dict(dfam=1, vpow=0.0), "id"),
    ("poisson", dict(dfam=1, vpow=1.0), "log"),
    ("gamma", dict(dfam=1, vpow=2.0, link=1, lpow=0.0), "log"),
    ("binom", dict(dfam=2, link=2), "logit"),
    ("binom", dict(dfam=2, link=3), "probit"),
])
def test_glm_matches_direct_minimisation(kind, args, link):
    from scipy.optimize import minimize
    X, y = _glm_data(kind)
    reg = 0.5
    r, out = algo("GLM", dict(X="X", Y="Y", B="B", icpt=1, reg=reg, tol=1e-12, moi=200, **args),
                  {"X": X, "Y": y}, ["B"])
    b = r["B"].ravel()
    f = _glm_objective(kind, link, X, y, reg)
    ref = minimize(f, np.zeros(X.shape[1] + 1), method="BFGS", options=dict(gtol=1e-9, maxiter=10000))
    assert f(b) <= ref.fun * (1 + 1e-9) + 1e-9
    np.testing.assert_allclose(b, ref.x, atol=2e-4)
    assert "TERMINATION_CODE,1" in "\n".join(out)


def test_glm_standardized_intercept_and_binomial_counts():
    X, y = _glm_data("binom", seed=3)
    r1, _ = algo("GLM", dict(X="X", Y="Y", B="B", icpt=1, dfam=2, link=2, tol=1e-12), {"X": X, "Y": y}, ["B"])
    r2, _ = algo("GLM", dict(X="X", Y="Y", B="B", icpt=2, dfam=2, link=2, tol=1e-12), {"X": X, "Y": y}, ["B"])
    assert r2["B"].shape == (X.shape[1] + 1, 2)
    np.testing.assert_allclose(r2["B"][:, 0], r1["B"].ravel(), atol=1e-6)
    # the same data as (#pos, #neg) counts, with yneg=-1 labels for the one-column form
    Y2 = np.hstack([y, 1 - y])
    r3, _ = algo("GLM", dict(X="X", Y="Y", B="B", icpt=1, dfam=2, link=2, tol=1e-12), {"X": X, "Y": Y2}, ["B"])
    np.testing.assert_allclose(r3["B"], r1["B"], atol=1e-6)
    r4, _ = algo("GLM", dict(X="X", Y="Y", B="B", icpt=1, dfam=2, link=2, yneg=-1.0, tol=1e-12),
                 {"X": X, "Y": 2 * y - 1}, ["B"])
    np.testing.assert_allclose(r4["B"], r1["B"], atol=1e-6)


def test_glm_predict_means_and_r2():
    X, y = _glm_data("poisson", seed=5)
    r, _ = algo("GLM", dict(X="X", Y="Y", B="B", icpt=1, dfam=1, vpow=1.0, tol=1e-12), {"X": X, "Y": y}, ["B"])
    B = r["B"]
    p, out = algo("GLM-predict", dict(X="X", B="B", M="M", Y="Y", dfam=1, vpow=1.0, link=1, lpow=0.0),
                  {"X": X, "B": B, "Y": y}, ["M"])
    mu = np.exp(X @ B[:-1] + B[-1])
    np.testing.assert_allclose(p["M"], mu, rtol=1e-12)
    stats = dict((l.split(",")[0] + l.split(",")[1], float(l.split(",")[-1]))
                 for l in "\n".join(out).split("\n") if l.count(",") == 3)
    r2 = 1 - np.sum((y - mu) ** 2) / np.sum((y - y.mean()) ** 2)
    np.testing.assert_allclose(stats["R21"], r2, rtol=1e-10)
    np.testing.assert_allclose(stats["PEARSON_X2"], np.sum((y - mu) ** 2 / mu), rtol=1e-10)


def test_univar_stats():
    rng = np.random.default_rng(8)
    n = 501
    X = np.hstack([rng.gamma(2.0, 1.5, (n, 1)), rng.integers(1, 5, (n, 1)).astype(float),
                   rng.standard_normal((n, 1)) * 3 + 1, rng.integers(1, 3, (n, 1)).astype(float)])
    types = np.array([[1, 2, 1, 3]], dtype=float)
    r, _ = algo("Univar-Stats", dict(X="X", TYPES="T", STATS="/tmp/_univar_stats"), {"X": X, "K": types}, ["S"])
    S = r["S"]
    for j in (0, 2):
        x = X[:, j]
        mu, sd = x.mean(), x.std(ddof=1)
        m2, m3, m4 = [np.mean((x - mu) ** k) for k in (2, 3, 4)]
        exp = [x.min(), x.max(), np.ptp(x), mu, sd ** 2, sd, sd / np.sqrt(n), sd / mu, m3 / sd ** 3, m4 / sd ** 4 - 3]
        np.testing.assert_allclose(S[:10, j], exp, rtol=1e-10)
        np.testing.assert_allclose(S[12, j], np.median(x), rtol=1e-12)
        xs = np.sort(x)   # inter-quartile mean of the middle half
        assert np.quantile(x, 0.25) <= S[13, j] <= np.quantile(x, 0.75)
    for j in (1, 3):
        cnt = np.bincount(X[:, j].astype(int))[1:]
        assert S[14, j] == len(cnt) and S[15, j] == np.argmax(cnt) + 1 and S[16, j] == np.sum(cnt == cnt.max())
        assert np.all(S[:12, j] == 0)


def test_bivar_stats(tmp_path):
    from scipy import stats as st
    from systemml_amd.io.readers import read_matrix
    rng = np.random.default_rng(9)
    n = 400
    s1 = rng.standard_normal(n)
    s2 = 0.6 * s1 + rng.standard_normal(n)
    c1 = rng.integers(1, 4, n).astype(float)
    o1 = np.clip(np.round(s1 + 2.5), 1, 5)
    o2 = np.clip(np.round(s2 + 2.5), 1, 5)
    X = np.column_stack([s1, s2, c1, o1, o2])
    idx1, idx2 = np.array([[1, 3, 4]]), np.array([[2, 5]])
    t1, t2 = np.array([[1, 2, 3]]), np.array([[1, 3]])
    algo("bivar-stats", dict(X="X", index1="i1", index2="i2", types1="t1", types2="t2", OUTDIR=str(tmp_path)),
         {"D": X, "S1": idx1, "S2": idx2, "K1": t1, "K2": t2}, [])
    ss = read_matrix(str(tmp_path / "bivar.scale.scale.stats")).numpy()
    r, _ = st.pearsonr(s1, s2)
    np.testing.assert_allclose(ss[:, 0], [1, 2, r, np.cov(s1, s2)[0, 1], s1.std(ddof=1), s2.std(ddof=1)], rtol=1e-10)
    nn = read_matrix(str(tmp_path / "bivar.nominal.nominal.stats")).numpy()
    for col, (a, b) in enumerate([(c1, o2), (o1, o2)]):
        tab = np.array([[np.sum((a == u) & (b == v)) for v in np.unique(b)] for u in np.unique(a)])
        chi2, p, dof, _ = st.chi2_contingency(tab, correction=False)
        np.testing.assert_allclose(nn[2:5, col], [chi2, dof, p], rtol=1e-8)
    oo = read_matrix(str(tmp_path / "bivar.ordinal.ordinal.stats")).numpy()
    np.testing.assert_allclose(oo[2, 0], st.spearmanr(o1, o2)[0], rtol=1e-10)
    ns = read_matrix(str(tmp_path / "bivar.nominal.scale.stats")).numpy()
    # scale column s1 against nominal c1 (ordinal o1 vs scale s2 handled the same way)
    f, p = st.f_oneway(*[s2[c1 == u] for u in np.unique(c1)])
    k = [i for i in range(ns.shape[1]) if ns[0, i] == 3 and ns[1, i] == 2][0]
    np.testing.assert_allclose(ns[3:5, k], [f, p], rtol=1e-8)


def _tree_data(n=800, seed=12):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, 3))
    cat = rng.integers(1, 4, n)
    Xd = np.hstack([X, np.eye(3)[cat - 1]])
    y = ((X[:, 0] > 0.3) & (cat != 2)).astype(int) + 1 + (X[:, 1] > 1).astype(int)
    R = np.array([[1, 1, 1], [2, 2, 2], [3, 3, 3], [4, 4, 6]], dtype=float)
    return Xd, np.eye(3)[y - 1], y, R


def test_decision_tree_fit_and_predict():
    Xd, Y, y, R = _tree_data()
    r, out = algo("decision-tree", dict(X="X", Y="Y", R="R", M="M", bins=20, depth=8, num_leaf=5),
                  {"X": Xd, "Y": Y, "R": R}, ["M"])
    M = r["M"]
    assert M.shape[0] == 6 and M[0, 0] == 1
    # model consistency: children of internal node j sit at j + offset and j + offset + 1
    for j in range(M.shape[1]):
        if M[2, j] > 0:
            lc = j + int(M[1, j])
            assert M[0, lc] == 2 * M[0, j] and M[0, lc + 1] == 2 * M[0, j] + 1
    p, pout = algo("decision-tree-predict", dict(X="X", Y="Y", R="R", M="M", P="P"),
                   {"X": Xd, "Y": Y, "R": R, "M": M}, ["P"])
    acc = (p["P"].ravel() == y).mean()
    assert acc > 0.97
    train_acc = float([l for l in out if "accuracy" in l][0].split(":")[1])
    np.testing.assert_allclose(train_acc, 100 * acc)      # leaves' error counts match the replay


def test_random_forest_votes():
    Xd, Y, y, R = _tree_data(seed=13)
    r, _ = algo("random-forest", dict(X="X", Y="Y", R="R", M="M", C="C", bins=16, depth=8, num_leaf=5,
                                      num_trees=5, feature_subset=1.0), {"X": Xd, "Y": Y, "R": R}, ["M", "Cnt"])
    M = r["M"]
    assert M.shape[0] == 7 and set(np.unique(M[1])) == {1, 2, 3, 4, 5}
    p, out = algo("random-forest-predict", dict(X="X", Y="Y", R="R", M="M", C="C", P="P"),
                  {"X": Xd, "Y": Y, "R": R, "M": M, "Cnt": r["Cnt"]}, ["P"])
    assert (p["P"].ravel() == y).mean() > 0.95
    assert any(l.startswith("Out-Of-Bag error") for l in out)


@pytest.mark.parametrize("name,a,b", [("ALS-CG", "U", "V"), ("ALS-DS", "L", "R")])
@pytest.mark.parametrize("reg", ["L2", "wL2"])
def test_als_recovers_low_rank(name, a, b, reg):
    rng = np.random.default_rng(14)
    m, n, k = 60, 40, 3
    full = rng.standard_normal((m, k)) @ rng.standard_normal((k, n))
    mask = rng.random((m, n)) < 0.6
    X = np.where(mask, full, 0.0)
    inp = "X" if name == "ALS-CG" else "Vm"
    r, _ = algo(name, {"X" if name == "ALS-CG" else "V": "X", a: a, b: b, "rank": k, "reg": reg,
                       "lambda": 1e-6, "maxi": 60, "check": False, "thr": 1e-12},
                {inp: X}, [a, b])
    P = r[a] @ r[b]
    err = np.abs(P - full)[mask].max()
    assert err < 1e-3, err
    # held-out entries are recovered too (rank-3 structure)
    assert np.abs(P - full)[~mask].max() < 1e-2


def test_als_predict_and_topk(tmp_path):
    rng = np.random.default_rng(15)
    L = rng.standard_normal((6, 2))
    R = rng.standard_normal((2, 5))
    pairs = np.array([[1, 1], [6, 5], [3, 2]], dtype=float)
    r, _ = algo("ALS_predict", dict(X="X", Y="Y", L="L", R="R", Vrows=6, Vcols=5),
                {"X": pairs, "L": L, "R": R}, ["Y"])
    S = L @ R
    np.testing.assert_allclose(r["Y"][:, 2], [S[0, 0], S[5, 4], S[2, 1]])
    V = np.zeros((6, 5))
    V[1, np.argmax(S[1])] = 1          # user 2 already rated its best item
    users = np.array([[2], [4]], dtype=float)
    t, _ = algo("ALS_topk_predict", dict(X="X", Y=str(tmp_path / "Y"), L="L", R="R", V="V", K=2),
                {"X": users, "L": L, "R": R, "V": V}, ["IDS", "SC"])
    s2 = np.where(V[1] != 0, -np.inf, S[1])
    np.testing.assert_array_equal(t["IDS"][0], np.argsort(-s2)[:2] + 1)
    np.testing.assert_array_equal(t["IDS"][1], np.argsort(-S[3])[:2] + 1)


def test_step_linear_regression_selects_true_features():
    rng = np.random.default_rng(16)
    n, m = 500, 8
    X = rng.standard_normal((n, m))
    y = 3 * X[:, [2]] - 2 * X[:, [5]] + 0.5 * X[:, [0]] + 1.0 + 0.1 * rng.standard_normal((n, 1))
    r, _ = algo("StepLinearRegDS", dict(X="X", Y="y", B="B", S="S", icpt=1, thr=0.001),
                {"X": X, "y": y}, ["S", "Bfull"])
    assert list(r["S"].ravel()[:3]) == [3, 6, 1]
    B = r["Bfull"].ravel()
    sel = [int(s) - 1 for s in r["S"].ravel()]
    Xi = np.hstack([X[:, sel], np.ones((n, 1))])
    ref = np.linalg.lstsq(Xi, y, rcond=None)[0].ravel()
    np.testing.assert_allclose(B[sel], ref[:-1], atol=1e-8)
    np.testing.assert_allclose(B[-1], ref[-1], atol=1e-8)
    assert np.all(np.delete(B[:-1], sel) == 0)


@pytest.mark.parametrize("name", ["CsplineDS", "CsplineCG"])
def test_cubic_spline_matches_scipy(name):
    from scipy.interpolate import CubicSpline
    x = np.array([0.0, 0.7, 1.5, 2.0, 3.2, 4.0, 5.5])
    y = np.sin(x) + 0.1 * x
    cs = CubicSpline(x, y, bc_type="natural")
    for xq in (0.3, 2.6, 5.0):
        r, _ = algo(name, dict(X="X", Y="Y", K="K", O="O", inp_x=xq), {"X": x.reshape(-1, 1), "Y": y.reshape(-1, 1)},
                    ["K", "q"])
        np.testing.assert_allclose(r["K"].ravel(), cs(x, 1), rtol=1e-6, atol=1e-8)
        np.testing.assert_allclose(r["q"], cs(xq), rtol=1e-6)


def test_stratstats_against_numpy():
    from scipy import stats as st
    rng = np.random.default_rng(21)
    n = 600
    s = rng.integers(1, 5, n).astype(float)
    x = rng.standard_normal(n) + s
    y = 0.7 * x + 0.5 * s + rng.standard_normal(n)
    x[5] = np.nan
    y[9] = np.nan
    X = np.column_stack([s, x, y])
    r, _ = algo("stratstats", dict(X="X", O="O", Xcid="xc", Ycid="yc", Scid=1),
                {"X": X, "Xcid": np.array([[2]]), "Ycid": np.array([[3]])}, ["OUT"])
    row = r["OUT"][0]
    ok = ~np.isnan(x) & ~np.isnan(y)
    xs, ys, ss = x[ok], y[ok], s[ok]
    res = st.linregress(xs, ys)
    np.testing.assert_allclose(row[[20, 21, 23, 25, 27]], [ok.sum(), res.slope, res.rvalue, res.rvalue ** 2,
                                                          res.pvalue], rtol=1e-9)
    np.testing.assert_allclose(row[22], res.stderr, rtol=1e-9)
    # stratified slope = within-stratum (fixed effects) regression
    xd = xs - np.array([xs[ss == k].mean() for k in ss])
    yd = ys - np.array([ys[ss == k].mean() for k in ss])
    np.testing.assert_allclose(row[31], (xd @ yd) / (xd @ xd), rtol=1e-9)
    # covariate x vs strata: one-way ANOVA
    xv = x[~np.isnan(x)]
    f, p = st.f_oneway(*[xv[s[~np.isnan(x)] == k] for k in (1, 2, 3, 4)])
    np.testing.assert_allclose(row[7], p, rtol=1e-6)
    assert row[0] == 2 and row[10] == 3 and row[38] == 4


def _km_ref(t, e):
    """KM table at the event times (rows with at least one event: the reference's layout)."""
    ut = np.unique(t)
    n_risk = np.array([(t >= u).sum() for u in ut], float)
    d = np.array([e[t == u].sum() for u in ut], float)
    s = np.cumprod(1 - d / n_risk)
    gw = np.cumsum(d / np.maximum(n_risk * (n_risk - d), 1e-300) * (n_risk > d))
    k = d > 0
    return ut[k], n_risk[k], d[k], s[k], (s * np.sqrt(gw))[k]


def test_kaplan_meier_and_logrank():
    from scipy.stats import CensoredData, ecdf, logrank
    rng = np.random.default_rng(5)
    n = 120
    g = rng.integers(1, 3, n)
    t = np.round(rng.exponential(np.where(g == 1, 5.0, 9.0)), 1) + 0.1
    e = (rng.random(n) < 0.75).astype(float)
    X = np.column_stack([t, e, g])
    TE = np.array([[1.0, 2.0]])
    r, out = algo("KM", dict(X="X", TE="TE", GI="GI", O="O", M="M", T="T", ttype="log-rank",
                             etype="greenwood", ctype="log"),
                  {"X": X, "TE": TE, "GI": np.array([[3.0]])}, ["KM", "Mout", "Tout"])
    KM, M, T = r["KM"], r["Mout"], r["Tout"]
    for gi in (1, 2):
        sel = g == gi
        ut, nr, d, s, se = _km_ref(t[sel], e[sel])
        blk = KM[:len(ut), 7 * (gi - 1):7 * gi]
        np.testing.assert_allclose(blk[:, 0], ut)
        np.testing.assert_allclose(blk[:, 1], nr)
        np.testing.assert_allclose(blk[:, 2], d)
        np.testing.assert_allclose(blk[:, 3], s, atol=1e-12)
        np.testing.assert_allclose(blk[:, 4], se, atol=1e-12)
        # survival also matches scipy's KM estimator
        cd = CensoredData(uncensored=t[sel][e[sel] == 1], right=t[sel][e[sel] == 0])
        np.testing.assert_allclose(blk[:, 3], ecdf(cd).sf.evaluate(ut), atol=1e-12)
        med = ut[np.argmax(s <= 0.5)] if (s <= 0.5).any() else np.nan
        assert M[gi - 1, 0] == gi and M[gi - 1, 1] == sel.sum() and M[gi - 1, 2] == e[sel].sum()
        np.testing.assert_allclose(M[gi - 1, 3], med)
    c1 = CensoredData(uncensored=t[(g == 1) & (e == 1)], right=t[(g == 1) & (e == 0)])
    c2 = CensoredData(uncensored=t[(g == 2) & (e == 1)], right=t[(g == 2) & (e == 0)])
    lr = logrank(c1, c2)
    np.testing.assert_allclose(T[0, 2], lr.statistic ** 2, rtol=1e-10)
    np.testing.assert_allclose(T[0, 3], lr.pvalue, rtol=1e-8)
    assert T[0, 0] == 2 and T[0, 1] == 1


def test_kaplan_meier_strata_wilcoxon():
    rng = np.random.default_rng(6)
    n = 90
    g = rng.integers(1, 4, n)
    s = rng.integers(1, 3, n)
    t = rng.integers(1, 30, n).astype(float)
    e = (rng.random(n) < 0.8).astype(float)
    X = np.column_stack([t, e, g, s])
    r, _ = algo("KM", dict(X="X", TE="TE", GI="GI", SI="SI", O="O", M="M", T="T", ttype="wilcoxon"),
                {"X": X, "TE": np.array([[1.0, 2.0]]), "GI": np.array([[3.0]]), "SI": np.array([[4.0]])},
                ["KM", "Mout", "Tout"])
    KM, M, T = r["KM"], r["Mout"], r["Tout"]
    assert KM.shape[1] == 7 * 6 and M.shape == (6, 2 + 5)
    for gi in (1, 2, 3):
        for si in (1, 2):
            c = (gi - 1) * 2 + si
            sel = (g == gi) & (s == si)
            ut, nr, d, sv, _ = _km_ref(t[sel], e[sel])
            np.testing.assert_allclose(KM[:len(ut), 7 * (c - 1) + 3], sv, atol=1e-12)
            assert M[c - 1, 0] == gi and M[c - 1, 1] == si
    # stratified Gehan-Wilcoxon reference
    O = np.zeros(3); E = np.zeros(3); V = np.zeros((3, 3))
    for si in (1, 2):
        ms = s == si
        for u in np.unique(t[ms]):
            risk = np.array([((t >= u) & ms & (g == k)).sum() for k in (1, 2, 3)], float)
            dk = np.array([(e * ((t == u) & ms & (g == k))).sum() for k in (1, 2, 3)])
            N, D = risk.sum(), dk.sum()
            if D == 0:
                continue
            w = N
            O += w * dk
            E += w * risk * D / N
            f = w ** 2 * D * (N - D) / max(N - 1, 1) / N ** 2
            V += f * (np.diag(risk * N) - np.outer(risk, risk))
    oe = (O - E)[:2]
    stat = oe @ np.linalg.solve(V[:2, :2], oe)
    np.testing.assert_allclose(T[0, 2], stat, rtol=1e-9)


def _cox_ref(t, e, Z, b):
    """Breslow partial likelihood, score and information by explicit risk-set loops."""
    l, g, I = 0.0, np.zeros(Z.shape[1]), np.zeros((Z.shape[1],) * 2)
    w = np.exp(Z @ b)
    for u in np.unique(t[e == 1]):
        R = t >= u
        D = (t == u) & (e == 1)
        s0 = w[R].sum()
        s1 = (w[R, None] * Z[R]).sum(0)
        s2 = (w[R, None, None] * Z[R, :, None] * Z[R, None, :]).sum(0)
        dk = D.sum()
        l += (Z[D] @ b).sum() - dk * np.log(s0)
        g += Z[D].sum(0) - dk * s1 / s0
        I += dk * (s2 / s0 - np.outer(s1, s1) / s0 ** 2)
    return l, g, I


def test_cox_regression_and_predict():
    from scipy.optimize import minimize
    from scipy.stats import chi2
    rng = np.random.default_rng(7)
    n = 150
    Z = rng.standard_normal((n, 3))
    fac = rng.integers(0, 3, n)
    F = np.eye(3)[fac]                                   # one factor, 3 levels
    beta = np.array([0.6, -0.4, 0.2, 0.5, -0.3])
    full = np.hstack([Z, F[:, 1:]])
    t = np.round(rng.exponential(1.0 / np.exp(full @ beta)), 2) + 0.01
    e = (rng.random(n) < 0.8).astype(float)
    X = np.column_stack([t, e, Z, F])                    # cols 1,2 | 3..5 | 6..8
    r, _ = algo("Cox", dict(X="X", TE="TE", R="R", M="M", S="S", T="T", COV="COV", RT="RT",
                            XO="XO", MF="MF", tol=1e-12),
                {"X": X, "TE": np.array([[1.0], [2.0]]), "R": np.array([[6.0, 8.0]])},
                ["M", "St", "Tst", "COV", "XO", "RT", "MF"])
    M, St, Tst, COV, MF = r["M"], r["St"], r["Tst"], r["COV"], r["MF"]
    # the most frequent factor level is the baseline
    base = 6 + int(np.argmax(np.bincount(fac, minlength=3)[::-1]) * -1 + 2)
    kept = [c for c in (6, 7, 8) if c != base]
    np.testing.assert_array_equal(MF.ravel(), [1, 2, 3, 4, 5] + kept)
    Zk = X[:, [c - 1 for c in MF.ravel()[2:].astype(int)]]
    Zk = Zk - Zk.mean(0)
    ref = minimize(lambda b: -_cox_ref(t, e, Zk, b)[0], np.zeros(5),
                   jac=lambda b: -_cox_ref(t, e, Zk, b)[1], method="BFGS",
                   options=dict(gtol=1e-10))
    np.testing.assert_allclose(M[:, 0], ref.x, atol=1e-6)
    l, g, I = _cox_ref(t, e, Zk, M[:, 0])
    np.testing.assert_allclose(COV, np.linalg.inv(I), rtol=1e-8)
    np.testing.assert_allclose(M[:, 2], np.sqrt(np.diag(np.linalg.inv(I))), rtol=1e-8)
    l0, g0, I0 = _cox_ref(t, e, Zk, np.zeros(5))
    np.testing.assert_allclose(St.ravel()[:4], [n, e.sum(), l, -2 * l + 10], rtol=1e-10)
    # rows in the reference's order (Cox.dml:423-440): Wald, likelihood ratio, score
    np.testing.assert_allclose(Tst[:, 0], [M[:, 0] @ I @ M[:, 0], 2 * (l - l0),
                                           g0 @ np.linalg.solve(I0, g0)], rtol=1e-8)
    np.testing.assert_allclose(Tst[1, 2], chi2.sf(2 * (l - l0), 5), rtol=1e-8)

    # prediction on new records (original column layout)
    Y = X[:7].copy()
    Y[:, 0] = [0.001, 0.05, 0.3, 1.0, 2.5, t.max() + 1, np.median(t)]
    p, _ = algo("Cox-predict", dict(X="XO", RT="RT", M="M", Y="Y", COV="COV", MF="MF", P="P"),
                {"X": r["XO"], "RT": r["RT"], "M": M, "Y": Y, "COV": COV, "MF": MF}, ["P"])
    P = p["P"]
    cols = MF.ravel()[2:].astype(int) - 1
    mu = X[:, cols].mean(0)
    b = M[:, 0]
    Zc = X[:, cols] - mu
    w = np.exp(Zc @ b)
    for i in range(7):
        z = Y[i, cols] - mu
        lp = z @ b
        H0 = VH = 0.0
        Qv = np.zeros(5)
        for u in np.unique(t[e == 1]):
            if u > Y[i, 0]:
                continue
            R = t >= u
            dk = ((t == u) & (e == 1)).sum()
            s0 = w[R].sum()
            H0 += dk / s0
            VH += dk / s0 ** 2
            Qv += dk * (w[R, None] * Zc[R]).sum(0) / s0 ** 2
        dq = z * H0 - Qv
        exp_row = [lp, np.sqrt(z @ COV @ z), np.exp(lp), np.exp(lp) * np.sqrt(z @ COV @ z),
                   H0 * np.exp(lp), np.exp(lp) * np.sqrt(VH + dq @ COV @ dq)]
        np.testing.assert_allclose(P[i], exp_row, rtol=1e-8, atol=1e-12)


@pytest.mark.parametrize("link,icpt", [(2, 1), (3, 2), (4, 0)])
def test_step_glm_bernoulli(link, icpt):
    from scipy.optimize import minimize
    from scipy.stats import norm
    rng = np.random.default_rng(11)
    n, m = 600, 6
    X = rng.standard_normal((n, m)) + 0.3
    eta = 1.4 * X[:, 1] - 1.1 * X[:, 4] + (0.3 if icpt else 0.0)
    inv = {2: lambda e: 1 / (1 + np.exp(-e)), 3: norm.cdf, 4: lambda e: 1 - np.exp(-np.exp(e))}[link]
    y = (rng.random(n) < inv(eta)).astype(float) * 2 - 1       # labels -1 / 1
    r, out = algo("StepGLM", dict(X="X", Y="Y", B="B", S="S", link=link, yneg=-1.0, icpt=icpt,
                                  tol=1e-12, thr=0.001),
                  {"X": X, "Y": y.reshape(-1, 1)}, ["Bout", "S", "dev"])
    S = r["S"].ravel().astype(int)
    assert set(S[:2]) == {2, 5}
    cols = S - 1
    A = X[:, cols]
    if icpt:
        A = np.hstack([A, np.ones((n, 1))])
    y01 = (y > 0).astype(float)

    def nll(b):
        mu = np.clip(inv(A @ b), 1e-12, 1 - 1e-12)
        return -np.sum(y01 * np.log(mu) + (1 - y01) * np.log(1 - mu))
    ref = minimize(nll, np.zeros(A.shape[1]), method="BFGS", options=dict(gtol=1e-9))
    B = r["Bout"]
    got = B[cols, 0]
    if icpt:
        got = np.append(got, B[m, 0])
    np.testing.assert_allclose(got, ref.x, atol=2e-4)
    np.testing.assert_allclose(r["dev"], 2 * ref.fun, rtol=1e-6)
    assert np.all(B[[c for c in range(m) if c not in cols], 0] == 0)


@pytest.mark.parametrize("icpt", [1, 2])
def test_intercept_column_is_a_view_and_matches_materialised(icpt):
    """icpt = 1 | 2 append a ones column; the compiler turns it into a constant-column view
    (ops/augmented.py) so X is never copied.  LinearRegCG and MultiLogReg produce the same
    coefficients as with the materialised cbind (rewrites off)."""
    import os
    from systemml_amd.api.executor import compile_script, execute, explain
    from systemml_amd.api.mlcontext import SCRIPTS_DIR
    from systemml_amd.conf import DMLConfig
    rng = np.random.default_rng(icpt)
    X = rng.standard_normal((20000, 60)) + 0.5
    y = X @ rng.standard_normal((60, 1)) + 1.0 + 0.1 * rng.standard_normal((20000, 1))
    lab = (np.argmax(X[:, :3], 1) + 1).reshape(-1, 1).astype(float)
    cases = [("LinearRegCG", {"X": X, "y": y}, dict(X="X", Y="y", B="B", icpt=icpt, maxi=20, tol=1e-12, reg=1e-3)),
             ("MultiLogReg", {"X": X, "Y_vec": lab}, dict(X="X", Y="Y", B="B", icpt=icpt, moi=5, mii=5, reg=0.01))]
    for name, ins, args in cases:
        src = open(os.path.join(SCRIPTS_DIR, "algorithms", name + ".dml")).read()
        outs = {}
        for rw in (True, False):
            cfg = DMLConfig(gpu=False, rewrites=rw)
            cs = compile_script(src, args, inputs=ins, outputs=["B_out"], config=cfg)
            if rw:
                assert "_cbind_const" in explain(cs.cp, "hops"), name
            res, _ = execute(cs, ins, out=lambda s: None)
            outs[rw] = np.asarray(res["B_out"].double().numpy() if hasattr(res["B_out"], "numpy") else res["B_out"])
        np.testing.assert_allclose(outs[True], outs[False], rtol=1e-7, atol=1e-9, err_msg=name)
