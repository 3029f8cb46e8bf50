"""Run algorithm scripts SPMD over `gloo` ranks on the CPU and compare with one process.

    python tools/dist_probe.py [--world 2] [--only ALS-CG Kmeans ...] [--minrows 50]

For every case of tools/run_algos.py it prints whether the distributed outputs match the
single-process ones and which operators had to all-gather a row-partitioned operand
(parallel/dist.fallback_sites).  tests/test_dist_algos.py runs the same harness.
"""
import argparse
import os
import socket
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

ALGOS = ["LinearRegCG", "MultiLogReg", "l2-svm", "m-svm", "Kmeans", "GLM", "ALS-CG", "PCA", "LinearRegDS",
         "naive-bayes"]


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def read_outputs(o):
    """All matrices the scripts wrote under o/<case>/ as numpy arrays keyed 'case/file'."""
    from systemml_amd.io import readers
    res = {}
    for case in sorted(os.listdir(o)):
        cd = os.path.join(o, case)
        if not os.path.isdir(cd):
            continue
        for f in sorted(os.listdir(cd)):
            p = os.path.join(cd, f)
            if f.endswith(".mtd") or f.startswith(".") or f.startswith("log"):
                continue
            try:
                v = readers.read(None, p)
            except Exception:  # noqa: BLE001 - non-matrix outputs
                continue
            if hasattr(v, "numpy"):
                res[f"{case}/{f}"] = v.double().cpu().numpy()
    return res


def run_cases(d, names, out_dir, cfg, dist=None):
    from tools.run_algos import cases
    from systemml_amd.api import executor as EX
    from systemml_amd.api.mlcontext import SCRIPTS_DIR
    os.makedirs(out_dir, exist_ok=True)
    errs = {}
    for name in names:
        o = os.path.join(out_dir, name)
        os.makedirs(o, exist_ok=True)
        args = {k.rstrip("_"): str(v).replace(f"{d}/out", o) for k, v in cases(d)[name].items()}
        path = os.path.join(SCRIPTS_DIR, "algorithms", name + ".dml")
        try:
            with open(path) as f:
                cs = EX.compile_script(f.read(), args, config=cfg, filename=path)
            EX.execute(cs, {}, out=lambda s: None, dist=dist)
        except Exception as e:  # noqa: BLE001
            import traceback
            errs[name] = traceback.format_exc()
    return errs


def _worker(rank, world, port, d, names, minrows, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from systemml_amd.parallel import dist as D
        from systemml_amd.conf import DMLConfig
        ctx = D.init(backend="gloo")
        cfg = DMLConfig(gpu=False, dist_min_rows=minrows, seed=42)
        per = {}
        errs = {}
        for n in names:
            D.reset_stats()
            e = run_cases(d, [n], f"{d}/dist_out", cfg, ctx)
            errs.update(e)
            per[n] = (dict(D.stats), dict(D.fallback_sites))
        q.put((rank, per, errs))
        D.shutdown()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, None, {"init": traceback.format_exc()}))


def probe(names, world=2, minrows=50, d=None, n=600):
    """Returns (single-process outputs, distributed outputs, per-rank stats, errors)."""
    import torch.multiprocessing as mp
    from tools.run_algos import make_data
    from systemml_amd.conf import DMLConfig
    d = d or tempfile.mkdtemp()
    make_data(d, n=n)
    errs1 = run_cases(d, names, f"{d}/out", DMLConfig(gpu=False, seed=42))
    ref = read_outputs(f"{d}/out")
    port = free_port()
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    procs = [mctx.Process(target=_worker, args=(r, world, port, d, names, minrows, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=900) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    got = read_outputs(f"{d}/dist_out")
    return ref, got, sorted(res, key=lambda r: r[0]), errs1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--minrows", type=int, default=50)
    ap.add_argument("--only", nargs="*")
    a = ap.parse_args()
    names = a.only or ALGOS
    ref, got, res, errs1 = probe(names, a.world, a.minrows)
    for n, e in errs1.items():
        print(f"single-process FAIL {n}: {e.splitlines()[-1]}")
    for rank, per, errs in res:
        for n, e in errs.items():
            print(f"rank {rank} FAIL {n}:\n{e}")
        if rank == 0 and per:
            for n, (st, sites) in per.items():
                print(f"{n:14s} allreduce={st['allreduce']:4d} alltoall={st['alltoall']:3d} "
                      f"fallbacks={st['fallback_gathers']:3d} {sites}")
    for k in sorted(ref):
        if k not in got:
            print(f"MISSING {k}")
            continue
        a, b = ref[k], got[k]
        if a.shape != b.shape:
            print(f"SHAPE {k}: {a.shape} vs {b.shape}")
            continue
        err = float(np.max(np.abs(a - b) / (1 + np.abs(a)))) if a.size else 0.0
        print(f"{'OK  ' if err < 1e-6 else 'DIFF'} {k:24s} max rel err {err:.2e}")


if __name__ == "__main__":
    main()
