"""Run the DML algorithm library (ours, or the reference's scripts for language-coverage
checks) on small synthetic inputs through the CP backend.

    python tools/run_algos.py [--dir systemml_amd/scripts/algorithms] [--only NAME ...]

Writes inputs as CSV + .mtd into a temp dir, executes each script with its
command-line contract and reports OK / FAIL with the error message.
"""
import argparse
import os
import sys
import tempfile
import time
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def write(path, a, fmt="csv"):
    import torch
    from systemml_amd.io import writers
    writers.write(None, torch.from_numpy(np.asarray(a, dtype=float)), path, format=fmt)


def make_data(d, n=200, m=8, seed=3):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, m))
    beta = rng.standard_normal((m, 1))
    y = X @ beta + 0.1 * rng.standard_normal((n, 1))
    ybin = np.where(X @ beta > 0, 1.0, -1.0)
    ycls = (np.argmax(X[:, :3] + 0.3 * rng.standard_normal((n, 3)), 1) + 1).reshape(-1, 1)
    counts = rng.poisson(np.exp(0.3 * X[:, :1]))
    Xpos = np.abs(X)
    Xint = np.floor(np.abs(X) * 2) + 1          # categorical-ish (1..k)
    R = (rng.random((60, 40)) < 0.2) * rng.integers(1, 6, (60, 40))
    types = np.ones((1, m))
    types[0, -2:] = 2                            # last two attrs categorical
    Xuni = np.hstack([X[:, :-2], Xint[:, -2:]])
    write(f"{d}/X", X)
    write(f"{d}/y", y)
    write(f"{d}/ybin", ybin)
    write(f"{d}/ycls", ycls)
    write(f"{d}/ydummy", np.eye(3)[ycls[:, 0] - 1])        # recoded + dummy-coded labels (tree scripts)
    write(f"{d}/y01", ((X @ beta + 1.5 * rng.standard_normal((n, 1))) > 0) * 1.0)   # noisy: finite MLE
    write(f"{d}/counts", counts)
    write(f"{d}/Xpos", Xpos + 0.1)
    write(f"{d}/Xint", Xint)
    write(f"{d}/R", R)
    write(f"{d}/types", types)
    write(f"{d}/Xuni", Xuni)
    write(f"{d}/S1", np.array([[1, 2]]))
    write(f"{d}/S2", np.array([[3, 4]]))
    write(f"{d}/K1", np.array([[1, 1]]))
    write(f"{d}/K2", np.array([[1, 1]]))
    # survival: time, event, features
    T = np.hstack([np.abs(rng.standard_normal((n, 1))) * 10 + 1, (rng.random((n, 1)) < 0.7) * 1.0,
                   rng.integers(1, 3, (n, 1)) * 1.0, X[:, :3]])
    write(f"{d}/surv", T)
    write(f"{d}/te", np.array([[1], [2]]))
    write(f"{d}/gi", np.array([[3]]))
    write(f"{d}/si", np.array([[3]]))
    write(f"{d}/F", np.array([[4], [5], [6]]))
    # unit-spaced knots: the reference Cspline scripts build the right-hand side with dy * h^2
    # where the spline equations need dy / h^2 (CsplineCG.dml calcKnotsDerivKs); the two agree
    # for h = 1, so their outputs are comparable with ours there
    xk = np.arange(1.0, 31.0).reshape(-1, 1)
    write(f"{d}/Xcs", xk)
    write(f"{d}/ycs", np.sin(xk * 0.3))


def cases(d):
    o = f"{d}/out"
    return {
        "LinearRegCG": dict(X=f"{d}/X", Y=f"{d}/y", B=f"{o}/B", icpt=1, maxi=50, tol=1e-9, reg=1e-4),
        "LinearRegDS": dict(X=f"{d}/X", Y=f"{d}/y", B=f"{o}/B", icpt=2, reg=1e-4),
        "MultiLogReg": dict(X=f"{d}/X", Y=f"{d}/ycls", B=f"{o}/B", icpt=2, reg=0.01, moi=10, mii=5),
        "l2-svm": dict(X=f"{d}/X", Y=f"{d}/ybin", model=f"{o}/w", icpt=1, tol=0.001, reg=1.0, maxiter=20,
                       Log=f"{o}/log"),
        "l2-svm-predict": dict(X=f"{d}/X", Y=f"{d}/ybin", model=f"{o}/w", icpt=1, scores=f"{o}/s",
                               accuracy=f"{o}/acc", confusion=f"{o}/conf"),
        "m-svm": dict(X=f"{d}/X", Y=f"{d}/ycls", model=f"{o}/mw", icpt=1, tol=0.001, reg=1.0, maxiter=20,
                      Log=f"{o}/log2"),
        "m-svm-predict": dict(X=f"{d}/X", Y=f"{d}/ycls", model=f"{o}/mw", icpt=1, scores=f"{o}/ms",
                              accuracy=f"{o}/macc", confusion=f"{o}/mconf"),
        "naive-bayes": dict(X=f"{d}/Xint", Y=f"{d}/ycls", prior=f"{o}/prior", conditionals=f"{o}/cond",
                            accuracy=f"{o}/nbacc", laplace=1),
        "naive-bayes-predict": dict(X=f"{d}/Xint", Y=f"{d}/ycls", prior=f"{o}/prior", conditionals=f"{o}/cond",
                                    accuracy=f"{o}/nbacc2", confusion=f"{o}/nbconf", probabilities=f"{o}/nbp"),
        "Kmeans": dict(X=f"{d}/X", k=3, C=f"{o}/C", runs=2, maxi=20, isY=1, Y=f"{o}/Y"),
        "Kmeans-predict": dict(X=f"{d}/X", C=f"{o}/C", prY=f"{o}/prY", O=f"{o}/kmstats"),
        "PCA": dict(INPUT=f"{d}/X", K=3, CENTER=1, SCALE=1, PROJDATA=1, OUTPUT=f"{o}/pca"),
        "GLM": dict(X=f"{d}/X", Y=f"{d}/counts", B=f"{o}/glmB", dfam=1, vpow=1.0, link=1, lpow=0.0, icpt=1,
                    moi=20, mii=10),
        "GLM-predict": dict(X=f"{d}/X", Y=f"{d}/counts", B=f"{o}/glmB", M=f"{o}/glmM", dfam=1, vpow=1.0,
                            link=1, lpow=0.0, O=f"{o}/glmO"),
        "Univar-Stats": dict(X=f"{d}/Xuni", TYPES=f"{d}/types", STATS=f"{o}/ustats"),
        "bivar-stats": dict(X=f"{d}/X", index1=f"{d}/S1", index2=f"{d}/S2", types1=f"{d}/K1",
                            types2=f"{d}/K2", OUTDIR=f"{o}/bivar"),
        "ALS-CG": dict(X=f"{d}/R", U=f"{o}/U", V=f"{o}/V", rank=4, reg="L2", lambda_=0.01, maxi=10),
        "ALS-DS": dict(V=f"{d}/R", L=f"{o}/L", R=f"{o}/Rf", rank=4, reg="L2", lambda_=0.01, maxi=10),
        "decision-tree": dict(X=f"{d}/X", Y=f"{d}/ydummy", M=f"{o}/tree", bins=5, depth=4, num_leaf=5),
        "decision-tree-predict": dict(X=f"{d}/X", Y=f"{d}/ycls", M=f"{o}/tree", P=f"{o}/treeP",
                                      A=f"{o}/treeA", CM=f"{o}/treeCM"),
        "random-forest": dict(X=f"{d}/X", Y=f"{d}/ydummy", M=f"{o}/rf", bins=5, depth=4, num_leaf=5, num_trees=3),
        "random-forest-predict": dict(X=f"{d}/X", Y=f"{d}/ycls", M=f"{o}/rf", P=f"{o}/rfP", A=f"{o}/rfA",
                                      CM=f"{o}/rfCM"),
        "KM": dict(X=f"{d}/surv", TE=f"{d}/te", GI=f"{d}/gi", SI=f"{d}/si", O=f"{o}/km", M=f"{o}/kmM",
                   T=f"{o}/kmT"),
        "Cox": dict(X=f"{d}/surv", TE=f"{d}/te", F=f"{d}/F", M=f"{o}/coxM", S=f"{o}/coxS", T=f"{o}/coxT",
                    COV=f"{o}/coxCOV", RT=f"{o}/coxRT", XO=f"{o}/coxXO", MF=f"{o}/coxMF"),
        "CsplineCG": dict(X=f"{d}/Xcs", Y=f"{d}/ycs", K=f"{o}/csK", O=f"{o}/csO", inp_x=4.5, maxi=100,
                          tol=1e-12),
        "CsplineDS": dict(X=f"{d}/Xcs", Y=f"{d}/ycs", K=f"{o}/csK2", O=f"{o}/csO2", inp_x=4.5),
        "StepLinearRegDS": dict(X=f"{d}/X", Y=f"{d}/y", B=f"{o}/stepB", S=f"{o}/stepS", icpt=1, thr=0.01),
        "StepGLM": dict(X=f"{d}/X", Y=f"{d}/y01", B=f"{o}/sglmB", S=f"{o}/sglmS", link=2, yneg=0.0, icpt=1,
                        thr=0.01, tol=1e-9),
        "stratstats": dict(X=f"{d}/Xint", Xcid=f"{d}/S1", Ycid=f"{d}/S2", Scid=3, O=f"{o}/strat"),
    }


def run_suite(script_dir, d, out_dir=None, only=None, out_lines=None, config=None):
    """Run every case whose script exists in `script_dir` on the data in `d` (make_data); the
    scripts' output files go to `out_dir` (default d/out).  Returns {name: None | exception}.
    `config`: DMLConfig of the runs (default: CP / host fp64)."""
    from systemml_amd.api import executor as EX
    from systemml_amd.conf import DMLConfig
    cfg = config or DMLConfig(gpu=False)
    o = out_dir or f"{d}/out"
    os.makedirs(o, exist_ok=True)
    res = {}
    for name, args in cases(d).items():
        if only and name not in only:
            continue
        path = os.path.join(script_dir, name + ".dml")
        if not os.path.exists(path):
            continue
        args = {k.rstrip("_"): (str(v).replace(f"{d}/out", o)) for k, v in args.items()}
        out = [] if out_lines is None else out_lines.setdefault(name, [])
        try:
            with open(path) as f:
                src = f.read()
            cs = EX.compile_script(src, args, config=cfg, filename=path)
            EX.execute(cs, {}, out=out.append)
            res[name] = None
        except Exception as e:  # noqa: BLE001
            res[name] = e
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                   "systemml_amd", "scripts", "algorithms"))
    ap.add_argument("--only", nargs="*")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    d = tempfile.mkdtemp()
    os.makedirs(d + "/out", exist_ok=True)
    make_data(d)
    ok = fail = 0
    for name in cases(d):
        if a.only and name not in a.only:
            continue
        if not os.path.exists(os.path.join(a.dir, name + ".dml")):
            print(f"SKIP {name} (no script)")
            continue
        t = time.time()
        lines = {}
        r = run_suite(a.dir, d, only=[name], out_lines=lines)[name]
        if r is None:
            print(f"OK   {name:24s} {time.time() - t:6.2f}s")
            ok += 1
        else:
            print(f"FAIL {name:24s} {type(r).__name__}: {str(r)[:300]}")
            if a.verbose:
                traceback.print_exception(type(r), r, r.__traceback__)
            fail += 1
        if a.verbose:
            print("\n".join(lines.get(name, [])[-int(os.environ.get("RUN_ALGOS_TAIL", "5")):]))
    print(f"{ok} ok, {fail} failed")
    return 0 if fail == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
