"""SPMD row-partitioned execution over `gloo` (world_size 2, CPU): results must match
single-process execution and the hot operators must stay distributed (no all-gather
fallbacks) — reference analogue: the Spark-vs-CP equivalence tests of
test/integration/applications/* run in HYBRID_SPARK mode."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    rng = np.random.default_rng(5)
    X = rng.standard_normal((600, 12))
    y = X @ rng.standard_normal((12, 1)) + 0.05 * rng.standard_normal((600, 1))
    lab = (np.argmax(X[:, :3] + 0.3 * rng.standard_normal((600, 3)), 1) + 1).reshape(-1, 1).astype(float)
    return X, y, lab


def _run_algos(cfg, dist=None):
    from systemml_amd.api import executor as EX
    from systemml_amd.api.mlcontext import SCRIPTS_DIR
    X, y, lab = _data()
    out = []
    src1 = open(os.path.join(SCRIPTS_DIR, "algorithms", "LinearRegCG.dml")).read()
    src2 = open(os.path.join(SCRIPTS_DIR, "algorithms", "MultiLogReg.dml")).read()
    cs1 = EX.compile_script(src1, dict(X="X", Y="y", B="B", icpt=1, maxi=30, tol=1e-10, reg=0.01),
                            inputs={"X": X, "y": y}, outputs=["B_out"], config=cfg)
    r1, _ = EX.execute(cs1, {"X": X, "y": y}, out=out.append, dist=dist)
    cs2 = EX.compile_script(src2, dict(X="X", Y="Y", B="B", icpt=0, moi=8, mii=5, reg=0.01, tol=1e-8),
                            inputs={"X": X, "Y_vec": lab}, outputs=["B_out"], config=cfg)
    r2, _ = EX.execute(cs2, {"X": X, "Y_vec": lab}, out=out.append, dist=dist)
    from systemml_amd.parallel import dist as D
    b1 = D.gather(r1["B_out"]) if isinstance(r1["B_out"], D.DistMatrix) else r1["B_out"]
    b2 = D.gather(r2["B_out"]) if isinstance(r2["B_out"], D.DistMatrix) else r2["B_out"]
    return b1.numpy(), b2.numpy(), out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from systemml_amd.parallel import dist as D
        from systemml_amd.conf import DMLConfig
        ctx = D.init(backend="gloo")
        cfg = DMLConfig(gpu=False, dist_min_rows=100)
        b1, b2, out = _run_algos(cfg, ctx)
        q.put((rank, b1, b2, dict(D.stats), len(out)))
        D.shutdown()
    except Exception as e:  # pragma: no cover - surfaced in the parent
        import traceback
        q.put((rank, "ERR", traceback.format_exc(), None, None))


def test_spmd_matches_single_process():
    from systemml_amd.conf import DMLConfig
    ref1, ref2, _ = _run_algos(DMLConfig(gpu=False))
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert not isinstance(r[1], str), r[2]
    for rank, b1, b2, stats, nout in res:
        np.testing.assert_allclose(b1, ref1, rtol=1e-7, atol=1e-9)
        np.testing.assert_allclose(b2, ref2, rtol=1e-6, atol=1e-8)
        assert stats["allreduce"] > 0
        assert stats["fallback_gathers"] == 0, stats
    # only rank 0 prints
    nouts = {rank: n for rank, _, _, _, n in res}
    assert nouts[0] > 0 and nouts[1] == 0
