"""scikit-learn style estimators over the DML algorithm library (reference:
src/main/python/systemml/mllearn/estimators.py and the Scala api/ml wrappers
LogisticRegression, LinearRegression, SVM, NaiveBayes).

    from systemml_amd.models.mllearn import LogisticRegression
    clf = LogisticRegression(C=1.0, max_iter=100).fit(X, y)
    clf.predict(X_test); clf.predict_proba(X_test); clf.score(X_test, y_test)

Inputs may be numpy arrays, scipy sparse matrices, pandas DataFrames/Series or torch
tensors.  Training runs the library script (scripts/algorithms/*.dml) through the
executor with in-memory bindings (no files); prediction is a short DML snippet over the
learned model.  Labels are recoded to 1..k internally and decoded on the way out, as the
reference's encode/decode do.  `sparkSession` arguments of the reference API are
accepted and ignored (there is no Spark here: the engine is the MI355X backend).
"""
from __future__ import annotations

import os

import numpy as np

from ..api.executor import run
from ..api.mlcontext import SCRIPTS_DIR
from ..conf import DMLConfig


def _np(x):
    if hasattr(x, "toarray") and not isinstance(x, np.ndarray):
        return x
    if hasattr(x, "to_numpy"):
        x = x.to_numpy()
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    x = np.asarray(x, dtype=np.float64)
    return x.reshape(-1, 1) if x.ndim == 1 else x


def _raw(y):
    """Labels as a flat numpy array, any dtype (strings allowed)."""
    if hasattr(y, "to_numpy"):
        y = y.to_numpy()
    if hasattr(y, "detach"):
        y = y.detach().cpu().numpy()
    return np.asarray(y).ravel()


def _out(v):
    if hasattr(v, "to_dense") and getattr(v, "layout", None) is not None and "sparse" in str(v.layout):
        v = v.to_dense()
    if hasattr(v, "detach"):
        return v.detach().double().cpu().numpy()
    return v


class BaseSystemMLEstimator:
    script = None

    def __init__(self, sparkSession=None, **params):
        self.config = DMLConfig()
        self._explain = ""
        self._stats = False
        self.params = params
        self.model_ = None

    # ---------------------------------------------------------------- config
    def setGPU(self, enable):
        self.config.gpu = bool(enable)
        return self

    def setForceGPU(self, enable):
        self.config.gpu = bool(enable)
        return self

    def setExplain(self, explain):
        self.config.explain = "hops" if explain else ""
        return self

    def setExplainLevel(self, level):
        self.config.explain = str(level)
        return self

    def setStatistics(self, statistics):
        self.config.stats = bool(statistics)
        return self

    def setStatisticsMaxHeavyHitters(self, k):
        self.config.stats_count = int(k)
        return self

    def setConfigProperty(self, name, value):
        self.config.set(name, value)
        return self

    def get_params(self, deep=True):
        return dict(self.params)

    def set_params(self, **params):
        self.params.update(params)
        return self

    # ---------------------------------------------------------------- helpers
    def _run_script(self, args, inputs, outputs):
        path = os.path.join(SCRIPTS_DIR, "algorithms", self.script + ".dml")
        with open(path) as f:
            src = f.read()
        out = []
        res = run(src, args=args, inputs=inputs, outputs=outputs, config=self.config, out=out.append,
                  filename=path)
        self.log_ = out
        return {k: _out(v) for k, v in res.items()}

    def _snippet(self, src, inputs, outputs):
        res = run(src, inputs=inputs, outputs=outputs, config=self.config, out=lambda s: None)
        return {k: _out(v) for k, v in res.items()}

    def fit_numpy(self, X, y):
        return self.fit(X, y)

    def fit_file(self, X_file, y_file):
        from ..io.readers import read_matrix
        return self.fit(read_matrix(X_file).numpy(), read_matrix(y_file).numpy())

    def transform(self, X):
        return self.predict(X)

    # ---------------------------------------------------------------- persistence
    def save(self, outputDir, format="binary", sep="/"):
        from ..io.writers import write_matrix
        import torch
        os.makedirs(outputDir, exist_ok=True)
        for k, v in self.model_.items():
            write_matrix(torch.as_tensor(np.asarray(v, dtype=np.float64).reshape(np.shape(v) or (1, 1))),
                         outputDir + sep + k, format)
        if getattr(self, "labels_", None) is not None:
            import json
            with open(outputDir + sep + "labels.json", "w") as f:
                json.dump([x.item() if hasattr(x, "item") else x for x in self.labels_], f)
        return self

    def load(self, weights, sep="/", eager=False):
        from ..io.readers import read_matrix
        self.model_ = {}
        for k in self.model_keys:
            self.model_[k] = read_matrix(weights + sep + k).numpy()
        lab = weights + sep + "labels.json"
        if os.path.exists(lab):
            import json
            with open(lab) as f:
                self.labels_ = np.asarray(json.load(f))
        return self


class BaseSystemMLClassifier(BaseSystemMLEstimator):
    def encode(self, y):
        y = _raw(y)
        self.labels_ = np.unique(y)
        return (np.searchsorted(self.labels_, y) + 1).astype(np.float64).reshape(-1, 1)

    def decode(self, idx):
        idx = np.asarray(idx).ravel().astype(int) - 1
        return self.labels_[np.clip(idx, 0, len(self.labels_) - 1)]

    def predict(self, X):
        P = self.predict_proba(X)
        return self.decode(np.argmax(P, axis=1) + 1)

    def score(self, X, y):
        return float(np.mean(self.predict(X) == _raw(y)))


class BaseSystemMLRegressor(BaseSystemMLEstimator):
    def score(self, X, y):
        y = _np(y).ravel()
        p = np.asarray(self.predict(X)).ravel()
        return float(1 - np.sum((y - p) ** 2) / np.sum((y - y.mean()) ** 2))


# ============================================================================
class LogisticRegression(BaseSystemMLClassifier):
    """Multinomial logistic regression (MultiLogReg.dml: trust-region Newton)."""
    script = "MultiLogReg"
    model_keys = ("B",)

    def __init__(self, sparkSession=None, penalty="l2", fit_intercept=True, normalize=False, max_iter=100,
                 max_inner_iter=0, tol=0.000001, C=1.0, solver="newton-cg", transferUsingDF=False):
        super().__init__(sparkSession, penalty=penalty, fit_intercept=fit_intercept, normalize=normalize,
                         max_iter=max_iter, max_inner_iter=max_inner_iter, tol=tol, C=C, solver=solver)
        if penalty != "l2" or solver != "newton-cg":
            raise ValueError("only penalty='l2' with solver='newton-cg' is supported")

    def fit(self, X, y, params=None):
        p = self.params
        icpt = (2 if p["normalize"] else 1) if p["fit_intercept"] else 0
        yk = self.encode(y)
        r = self._run_script(dict(X="X", Y="Y", B="B", icpt=icpt, reg=1.0 / p["C"], tol=p["tol"],
                                  moi=p["max_iter"], mii=p["max_inner_iter"]),
                             {"X": _np(X), "Y_vec": yk}, ["B_out"])
        self.model_ = {"B": r["B_out"]}       # original-scale betas (intercept last)
        return self

    def predict_proba(self, X):
        B = self.model_["B"]
        r = self._snippet('''
m = ncol(X)
LT = X %*% B[1:m, ]
if (nrow(B) > m) {
  LT = LT + B[m + 1, ]
}
LT = cbind(LT, matrix(0, rows = nrow(X), cols = 1))
E = exp(LT - rowMaxs(LT))
P = E / rowSums(E)
''', {"X": _np(X), "B": B}, ["P"])
        return r["P"]


class LinearRegression(BaseSystemMLRegressor):
    """Linear regression: solver 'newton-cg' -> LinearRegCG.dml, 'direct-solve' -> LinearRegDS.dml."""
    model_keys = ("B",)

    def __init__(self, sparkSession=None, fit_intercept=True, normalize=False, max_iter=100, tol=0.000001,
                 C=float("inf"), solver="newton-cg", transferUsingDF=False):
        super().__init__(sparkSession, fit_intercept=fit_intercept, normalize=normalize, max_iter=max_iter,
                         tol=tol, C=C, solver=solver)
        if solver not in ("newton-cg", "direct-solve"):
            raise ValueError("solver must be 'newton-cg' or 'direct-solve'")
        self.script = "LinearRegCG" if solver == "newton-cg" else "LinearRegDS"

    def fit(self, X, y, params=None):
        p = self.params
        icpt = (2 if p["normalize"] else 1) if p["fit_intercept"] else 0
        reg = 0.0 if p["C"] == float("inf") else 1.0 / p["C"]
        args = dict(X="X", Y="y", B="B", icpt=icpt, reg=max(reg, 1e-12), tol=p["tol"], maxi=p["max_iter"])
        r = self._run_script(args, {"X": _np(X), "y": _np(y)}, ["B_out"])
        self.model_ = {"B": r["B_out"][:, :1]}
        return self

    def predict(self, X):
        B = self.model_["B"]
        X = _np(X)
        m = X.shape[1]
        out = X @ B[:m] if not hasattr(X, "toarray") else X.toarray() @ B[:m]
        if B.shape[0] > m:
            out = out + B[m]
        return out.ravel()


class SVM(BaseSystemMLClassifier):
    """Linear SVM: binary l2-svm.dml or one-vs-rest m-svm.dml (is_multi_class=True)."""
    model_keys = ("W",)

    def __init__(self, sparkSession=None, fit_intercept=True, normalize=False, max_iter=100, tol=0.000001,
                 C=1.0, is_multi_class=False, transferUsingDF=False):
        super().__init__(sparkSession, fit_intercept=fit_intercept, normalize=normalize, max_iter=max_iter,
                         tol=tol, C=C, is_multi_class=is_multi_class)
        self.script = "m-svm" if is_multi_class else "l2-svm"

    def fit(self, X, y, params=None):
        p = self.params
        X = _np(X)
        yk = self.encode(y)
        icpt = 1 if p["fit_intercept"] else 0
        args = dict(X="X", Y="Y", model="model", icpt=icpt, tol=p["tol"], reg=1.0 / p["C"], maxiter=p["max_iter"])
        if p["is_multi_class"]:
            r = self._run_script(args, {"X": X, "Y": yk}, ["W"])
            self.model_ = {"W": r["W"]}
        else:
            if len(self.labels_) != 2:
                raise ValueError("binary SVM needs exactly two classes (use is_multi_class=True)")
            r = self._run_script(args, {"X": X, "Y": 2 * yk - 3}, ["w"])    # labels -> -1 / +1
            w = r["w"]
            self.model_ = {"W": np.hstack([-w, w])}                        # scores for class 1 / 2
        return self

    def predict_proba(self, X):
        X = _np(X)
        X = X.toarray() if hasattr(X, "toarray") else X
        W = self.model_["W"]
        m = X.shape[1]
        S = X @ W[:m]
        if W.shape[0] > m:
            S = S + W[m]
        return S                     # decision scores (argmax = predicted class), as the reference


class NaiveBayes(BaseSystemMLClassifier):
    """Multinomial naive Bayes (naive-bayes.dml)."""
    script = "naive-bayes"
    model_keys = ("prior", "cond")

    def __init__(self, sparkSession=None, laplace=1.0, transferUsingDF=False):
        super().__init__(sparkSession, laplace=laplace)

    def fit(self, X, y, params=None):
        yk = self.encode(y)
        r = self._run_script(dict(X="X", Y="Y", prior="p", conditionals="c", laplace=self.params["laplace"]),
                             {"X": _np(X), "y": yk}, ["prior", "cond"])
        self.model_ = {"prior": r["prior"], "cond": r["cond"]}
        return self

    def predict_proba(self, X):
        r = self._snippet('''
logp = X %*% t(log(cond)) + t(log(prior))
P = exp(logp - rowMaxs(logp))
P = P / rowSums(P)
''', {"X": _np(X), "cond": self.model_["cond"], "prior": self.model_["prior"]}, ["P"])
        return r["P"]
