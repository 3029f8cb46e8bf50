"""Performance test suite: the reference's scripts/perftest drivers (runAll.sh and its
runAll{Binomial,Multinomial,Regression,Stats,Clustering,DimensionReduction,Trees}.sh,
gen*Data.sh, run<Algorithm>.sh) as one driver.

    python -m systemml_amd.perftest [--dir DIR] [--sizes 10k_1k,100k_1k] [--families ...]
                                    [--sparsity dense,sparse] [--cpu] [--maxiter 20]
                                    [--out times.jsonl]

Like the shell suite, every family first generates its data with the datagen scripts
(scripts/datagen/*.dml, positional / named arguments as in gen*Data.sh, binary format),
splits off the held-out "_test" rows (scripts/perftest/extractTestData.dml), and then runs
each training script with the perftest settings (intercept variants icpt = 0, 1, 2 for the
regression family, 0 / 1 for the SVMs, max. iterations MAXITR = 20) followed by its predict
script.  One run = compile + execute of one script including its reads and writes, timed
end to end (the reference times each `systemml -f` invocation); results are appended to a
JSON-lines file (the reference's times.txt) and printed.

Sizes are "<rows>_<cols>" with k / M suffixes; the reference ships 10k_1k enabled and
100k .. 100M commented out.  The families and their runs:

  binomial        MultiLogReg (k=2), l2-svm, m-svm (k=2)              on X<size>_{dense,sparse}
  multinomial     naive-bayes, MultiLogReg, m-svm (k=5)               on X<size>_{dense,sparse}_k5
  regression      LinearRegDS, LinearRegCG, GLM poisson/log, gamma/log, binomial/probit
  stats           Univar-Stats, bivar-stats (A_<rows> descriptive data), stratstats
  clustering      Kmeans (k=5) + Kmeans-predict                       (dense only)
  dimreduction    PCA (SCALE=1 PROJDATA=1) on <rows/2>_<2*cols>       (dense only)
  trees           decision-tree, random-forest + predict scripts
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
SCRIPTS = os.path.join(HERE, "scripts")
FAMILIES = ("binomial", "multinomial", "regression", "stats", "clustering", "dimreduction", "trees")
SPARSITY = {"dense": 0.9, "sparse": 0.01}       # gen*Data.sh DENSE_SP / SPARSE_SP
FORMAT = "binary"


def parse_size(s):
    """'10k_1k' -> (10000, 1000)."""
    def num(t):
        mult = {"k": 1_000, "M": 1_000_000}.get(t[-1], 1)
        return int(float(t[:-1] if mult > 1 else t) * mult)
    r, c = s.split("_")
    return num(r), num(c)


class Suite:
    def __init__(self, root, gpu=None, maxiter=20, out=None, echo=print, stats=False):
        from .conf import get_default_config
        self.root = root
        self.maxiter = maxiter
        self.cfg = get_default_config().copy()
        if gpu is not None:
            self.cfg.gpu = gpu
        self.out = out
        self.echo = echo
        self.stats = stats
        self.results = []

    # ------------------------------------------------------------------ one script run
    def run(self, script, args, family="", data="", tag=None, record=True):
        """Compile + execute one DML script with -nvargs / -args (positional keys '1', '2', ..)."""
        from .api import executor as EX
        path = os.path.join(SCRIPTS, script)
        with open(path) as f:
            src = f.read()
        args = {str(k): str(v) for k, v in args.items()}
        printed = []
        t0 = time.perf_counter()
        ok, err = True, None
        try:
            cs = EX.compile_script(src, args, config=self.cfg, filename=path)
            EX.execute(cs, {}, out=printed.append)
            _sync()
        except Exception as e:   # noqa: BLE001 -- a failing run is recorded, the suite goes on
            ok, err = False, f"{type(e).__name__}: {e}"
            if os.environ.get("SYSML_PERFTEST_TRACE"):
                traceback.print_exc()
        sec = time.perf_counter() - t0
        if record:
            rec = {"family": family, "script": os.path.basename(script), "data": data, "seconds": round(sec, 4),
                   "ok": ok}
            if tag:
                rec.update(tag)
            if err:
                rec["error"] = err[:500]
            self.results.append(rec)
            self.echo(json.dumps(rec))
            if self.out:
                with open(self.out, "a") as f:
                    f.write(json.dumps(rec) + "\n")
        elif not ok:
            raise RuntimeError(f"{script}: {err}")
        return ok

    def gen(self, script, args):
        """Data generation / preparation step (not timed into the results)."""
        self.run(script, args, record=False)

    def p(self, *parts):
        d = os.path.join(self.root, *parts[:-1])
        os.makedirs(d, exist_ok=True)
        return os.path.join(d, parts[-1])

    # ------------------------------------------------------------------ families
    def binomial_data(self, size, kind):
        n, m = parse_size(size)
        X, y = self.p("binomial", f"X{size}_{kind}"), self.p("binomial", f"y{size}_{kind}")
        if not os.path.exists(X + ".mtd"):
            self.gen("datagen/genRandData4LogisticRegression.dml",
                     {1: n, 2: m, 3: 5, 4: 5, 5: self.p("binomial", f"w{size}_{kind}"), 6: X, 7: y, 8: 1, 9: 0,
                      10: SPARSITY[kind], 11: FORMAT, 12: 1})
            self.gen("perftest/extractTestData.dml", {1: X, 2: y, 3: X + "_test", 4: y + "_test", 5: FORMAT})
        return X, y

    def multinomial_data(self, size, kind, k=5):
        n, m = parse_size(size)
        X, y = self.p("multinomial", f"X{size}_{kind}_k{k}"), self.p("multinomial", f"y{size}_{kind}_k{k}")
        if not os.path.exists(X + ".mtd"):
            self.gen("datagen/genRandData4Multinomial.dml",
                     {1: n, 2: m, 3: SPARSITY[kind], 4: k, 5: 0, 6: X, 7: y, 8: FORMAT})
            self.gen("perftest/extractTestData.dml", {1: X, 2: y, 3: X + "_test", 4: y + "_test", 5: FORMAT})
        return X, y

    def fam_binomial(self, size, kind):
        X, y = self.binomial_data(size, kind)
        base, d = os.path.dirname(X), f"{size}_{kind}"
        self._mlogreg(X, y, 2, base, "binomial", d)
        self._svms(X, y, 2, base, "binomial", d, msvm_only=False)

    def fam_multinomial(self, size, kind):
        X, y = self.multinomial_data(size, kind)
        base, d = os.path.dirname(X), f"{size}_{kind}_k5"
        self.run("algorithms/naive-bayes.dml",
                 dict(X=X, Y=y, classes=5, prior=f"{base}/prior", conditionals=f"{base}/conditionals",
                      accuracy=f"{base}/debug_output", fmt="csv"), "multinomial", d)
        self.run("algorithms/naive-bayes-predict.dml",
                 dict(X=X + "_test", Y=y + "_test", prior=f"{base}/prior", conditionals=f"{base}/conditionals",
                      fmt="csv", probabilities=f"{base}/probabilities"), "multinomial", d)
        self._mlogreg(X, y, 5, base, "multinomial", d)
        self._svms(X, y, 5, base, "multinomial", d, msvm_only=True)

    def _mlogreg(self, X, y, k, base, fam, d):
        dfam = 3 if k > 2 else 2                     # runMultiLogReg.sh DFAM
        for icpt in (0, 1, 2):
            self.run("algorithms/MultiLogReg.dml",
                     dict(icpt=icpt, reg=0.01, tol=0.0001, moi=self.maxiter, mii=5, X=X, Y=y, B=f"{base}/b"),
                     fam, d, {"icpt": icpt})
            self.run("algorithms/GLM-predict.dml",
                     dict(dfam=dfam, vpow=-1, link=2, lpow=-1, fmt="csv", X=X + "_test", B=f"{base}/b",
                          Y=y + "_test", M=f"{base}/m", O=f"{base}/out.csv"), fam, d, {"icpt": icpt})

    def _svms(self, X, y, k, base, fam, d, msvm_only):
        for icpt in (0, 1):
            if not msvm_only:
                self.run("algorithms/l2-svm.dml",
                         dict(X=X, Y=y, icpt=icpt, tol=0.0001, reg=0.01, maxiter=self.maxiter, model=f"{base}/b",
                              Log=f"{base}/debug_output", fmt="csv"), fam, d, {"icpt": icpt})
                self.run("algorithms/l2-svm-predict.dml",
                         dict(X=X + "_test", Y=y + "_test", icpt=icpt, model=f"{base}/b", fmt="csv"),
                         fam, d, {"icpt": icpt})
            self.run("algorithms/m-svm.dml",
                     dict(X=X, Y=y, icpt=icpt, classes=k, tol=0.0001, reg=0.01, maxiter=self.maxiter,
                          model=f"{base}/w", Log=f"{base}/debug_output", fmt="csv"), fam, d, {"icpt": icpt})
            self.run("algorithms/m-svm-predict.dml",
                     dict(X=X + "_test", Y=y + "_test", icpt=icpt, model=f"{base}/w", fmt="csv"),
                     fam, d, {"icpt": icpt})

    def fam_regression(self, size, kind):
        X, y = self.binomial_data(size, kind)
        base, d = os.path.dirname(X), f"{size}_{kind}"
        lin_pred = dict(dfam=1, link=1, vpow=0.0, lpow=1.0)
        for icpt in (0, 1, 2):
            self.run("algorithms/LinearRegDS.dml", dict(X=X, Y=y, B=f"{base}/b", icpt=icpt, fmt="csv", reg=0.01),
                     "regression", d, {"icpt": icpt})
            self._glm_predict(X, y, base, lin_pred, d, icpt)
        for icpt in (0, 1, 2):
            self.run("algorithms/LinearRegCG.dml",
                     dict(X=X, Y=y, B=f"{base}/b", icpt=icpt, fmt="csv", maxi=self.maxiter, tol=0.0001, reg=0.01),
                     "regression", d, {"icpt": icpt})
            self._glm_predict(X, y, base, lin_pred, d, icpt)
        glms = (("poisson_log", dict(dfam=1, vpow=1.0, link=1, lpow=0.0)),
                ("gamma_log", dict(dfam=1, vpow=2.0, link=1, lpow=0.0)),
                ("binomial_probit", dict(dfam=2, link=3, yneg=2)))
        for name, fam in glms:
            for icpt in (0, 1, 2):
                self.run("algorithms/GLM.dml",
                         dict(X=X, Y=y, B=f"{base}/b", icpt=icpt, fmt="csv", moi=self.maxiter, mii=5, tol=0.0001,
                              reg=0.01, **fam), "regression", d, {"icpt": icpt, "glm": name})
                pf = {k: v for k, v in fam.items() if k != "yneg"}
                self._glm_predict(X, y, base, pf, d, icpt, {"glm": name})

    def _glm_predict(self, X, y, base, fam, d, icpt, extra=None):
        self.run("algorithms/GLM-predict.dml",
                 dict(fmt="csv", X=X + "_test", B=f"{base}/b", Y=y + "_test", M=f"{base}/m", O=f"{base}/out.csv",
                      **fam), "regression", d, dict({"icpt": icpt}, **(extra or {})))

    def fam_stats(self, size, kind):
        n, _ = parse_size(size)
        tag = f"A_{size.split('_')[0]}"
        b = self.p("bivar", tag, "data")
        bd = os.path.dirname(b)
        if not os.path.exists(b + ".mtd"):
            self.gen("datagen/genRandData4DescriptiveStats.dml",
                     dict(R=n, C=1000, NC=100, MAXDOMAIN=1100, DATA=b, TYPES=f"{bd}/types", SETSIZE=20,
                          LABELSETSIZE=10, TYPES1=f"{bd}/set1.types", TYPES2=f"{bd}/set2.types",
                          INDEX1=f"{bd}/set1.indices", INDEX2=f"{bd}/set2.indices", FMT=FORMAT))
        s = self.p("stratstats", tag, "data")
        sd = os.path.dirname(s)
        if not os.path.exists(s + ".mtd"):
            self.gen("datagen/genRandData4StratStats.dml",
                     dict(nr=n, nf=100, D=s, Xcid=f"{sd}/Xcid", Ycid=f"{sd}/Ycid", A=f"{sd}/A", fmt=FORMAT))
        self.run("algorithms/Univar-Stats.dml", dict(X=b, TYPES=f"{bd}/types", STATS=f"{bd}/stats/u"),
                 "stats", tag)
        self.run("algorithms/bivar-stats.dml",
                 dict(X=b, index1=f"{bd}/set1.indices", index2=f"{bd}/set2.indices", types1=f"{bd}/set1.types",
                      types2=f"{bd}/set2.types", OUTDIR=f"{bd}/stats/b"), "stats", tag)
        self.run("algorithms/stratstats.dml",
                 dict(X=s, Xcid=f"{sd}/Xcid", Ycid=f"{sd}/Ycid", O=f"{sd}/STATS/s", fmt="csv"), "stats", tag)

    def fam_clustering(self, size, kind):
        n, m = parse_size(size)
        X = self.p("clustering", f"X{size}_dense")
        base = os.path.dirname(X)
        if not os.path.exists(X + ".mtd"):
            self.gen("datagen/genRandData4Kmeans.dml",
                     dict(nr=n, nf=m, nc=5, dc=10.0, dr=1.0, fbf=100.0, cbf=100.0, X=X, C=f"{base}/C{size}_dense",
                          Y=f"{base}/y{size}_dense", YbyC=f"{base}/YbyC{size}_dense", fmt=FORMAT))
        d = f"{size}_dense"
        self.run("algorithms/Kmeans.dml", dict(X=X, k=5, C=f"{base}/centroids.mtx", maxi=self.maxiter, tol=0.0001),
                 "clustering", d)
        self.run("algorithms/Kmeans-predict.dml", dict(X=X, C=f"{base}/centroids.mtx", prY=f"{base}/prY.mtx"),
                 "clustering", d)

    def fam_dimreduction(self, size, kind):
        n, m = parse_size(size)
        n, m = max(n // 2, 1), 2 * m                 # 10k_1k -> the suite's 5k_2k
        d = f"{n // 1000}k_{m // 1000}k_dense"
        X = self.p("dimensionreduction", f"pcaData{d}")
        base = os.path.dirname(X)
        if not os.path.exists(X + ".mtd"):
            self.gen("datagen/genRandData4PCA.dml", dict(R=n, C=m, OUT=X, FMT=FORMAT))
        self.run("algorithms/PCA.dml", dict(INPUT=X, SCALE=1, PROJDATA=1, OUTPUT=f"{base}/output"),
                 "dimreduction", d)

    def fam_trees(self, size, kind):
        X, y = self.binomial_data(size, kind)
        base, d = self.p("trees", "M"), f"{size}_{kind}"
        base = os.path.dirname(base)
        self.run("algorithms/decision-tree.dml", dict(X=X, Y=y, fmt="csv", M=f"{base}/M"), "trees", d)
        self.run("algorithms/decision-tree-predict.dml",
                 dict(M=f"{base}/M", X=X + "_test", Y=y + "_test", P=f"{base}/P"), "trees", d)
        self.run("algorithms/random-forest.dml", dict(X=X, Y=y, fmt="csv", M=f"{base}/MRF"), "trees", d)
        self.run("algorithms/random-forest-predict.dml",
                 dict(M=f"{base}/MRF", X=X + "_test", Y=y + "_test", P=f"{base}/PRF"), "trees", d)

    def run_all(self, sizes, families, kinds):
        for fam in families:
            for size in sizes:
                for kind in kinds:
                    if fam in ("clustering", "dimreduction", "stats") and kind != kinds[0]:
                        continue                     # dense-only families run once per size
                    getattr(self, "fam_" + fam)(size, kind)
        return self.results


def _sync():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except Exception:   # noqa: BLE001
        pass


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--dir", default=os.path.join(os.getcwd(), "perftest_data"))
    ap.add_argument("--sizes", default="10k_1k")
    ap.add_argument("--families", default=",".join(FAMILIES))
    ap.add_argument("--sparsity", default="dense,sparse")
    ap.add_argument("--maxiter", type=int, default=20)
    ap.add_argument("--cpu", action="store_true", help="CP (host) execution only")
    ap.add_argument("--out", default=None, help="JSON-lines result file (appended)")
    a = ap.parse_args(argv)
    fams = [f for f in a.families.split(",") if f]
    bad = set(fams) - set(FAMILIES)
    if bad:
        raise SystemExit(f"unknown families {sorted(bad)}; choose from {FAMILIES}")
    suite = Suite(a.dir, gpu=False if a.cpu else None, maxiter=a.maxiter, out=a.out)
    res = suite.run_all(a.sizes.split(","), fams, a.sparsity.split(","))
    failed = [r for r in res if not r["ok"]]
    total = sum(r["seconds"] for r in res)
    print(json.dumps({"runs": len(res), "failed": len(failed), "total_seconds": round(total, 3)}))
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
