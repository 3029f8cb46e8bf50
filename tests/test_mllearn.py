"""mllearn estimators (reference: src/main/python/tests/test_mllearn_numpy.py compares
against scikit-learn on the same data)."""
import numpy as np
import pytest

from systemml_amd.models.mllearn import LinearRegression, LogisticRegression, NaiveBayes, SVM


@pytest.fixture(scope="module")
def cls_data():
    rng = np.random.default_rng(0)
    X = rng.standard_normal((600, 5))
    W = rng.standard_normal((5, 3))
    y = np.array(["a", "b", "c"])[np.argmax(X @ W + 0.3 * rng.standard_normal((600, 3)), 1)]
    return X, y


def test_logistic_regression_vs_sklearn(cls_data):
    from sklearn.linear_model import LogisticRegression as SkLR
    X, y = cls_data
    clf = LogisticRegression(C=10.0, max_iter=100, tol=1e-10).fit(X, y)
    sk = SkLR(C=10.0, max_iter=2000, tol=1e-10).fit(X, y)
    assert np.mean(clf.predict(X) == sk.predict(X)) > 0.97
    P = clf.predict_proba(X)
    np.testing.assert_allclose(P.sum(1), 1.0)
    assert clf.score(X, y) > 0.85


def test_linear_regression_solvers():
    rng = np.random.default_rng(1)
    X = rng.standard_normal((400, 6))
    y = X @ rng.standard_normal(6) + 2.0
    for solver in ("newton-cg", "direct-solve"):
        m = LinearRegression(solver=solver, tol=1e-12, max_iter=200).fit(X, y)
        np.testing.assert_allclose(m.predict(X), y, atol=1e-5)
        assert m.score(X, y) > 0.999999


def test_svm_binary_and_multiclass(cls_data):
    X, y = cls_data
    m = SVM(is_multi_class=True, C=10.0).fit(X, y)
    assert m.score(X, y) > 0.8
    yb = np.where(y == "a", "pos", "neg")
    b = SVM(C=10.0).fit(X, yb)
    assert b.score(X, yb) > 0.85 and set(b.predict(X)) <= {"pos", "neg"}


def test_naive_bayes_vs_sklearn(tmp_path):
    from sklearn.naive_bayes import MultinomialNB
    rng = np.random.default_rng(2)
    X = rng.integers(0, 6, (300, 8)).astype(float)
    y = rng.integers(1, 4, 300)
    X[y == 2, 0] += 5
    nb = NaiveBayes(laplace=1.0).fit(X, y)
    sk = MultinomialNB(alpha=1.0).fit(X, y)
    np.testing.assert_allclose(nb.predict_proba(X), sk.predict_proba(X), rtol=1e-8)
    nb.save(str(tmp_path / "nb"))
    nb2 = NaiveBayes().load(str(tmp_path / "nb"))
    np.testing.assert_array_equal(nb2.predict(X), nb.predict(X))
