"""Distributed (SPMD, row-partitioned) operators over `gloo` ranks on the CPU: every result
must equal single-process execution and no operator may fall back to all-gathering a
row-partitioned operand (parallel/dist.fallback_gathers).  World sizes 2 and 3 (uneven row
blocks).  Reference analogue: the Spark-vs-CP equivalence of test/integration/functions/*
run with ExecMode.SPARK (reorg/TransposeTest, append/RBindTest, indexing/*, cumsum,
quaternary/Weighted*Test, io/ReadCSVTest)."""
import os
import socket

import numpy as np
import pytest

SRC = """
X = rand(rows=90, cols=30, seed=1)
W = rand(rows=30, cols=40, seed=2)
A = X %*% W
T1 = t(X)
T2 = t(X[, 1:5])
G = X %*% t(X)
R1 = rbind(X, X[1:7, ])
R2 = rbind(X, A[, 1:30])
cs = cumsum(X)
cp = cumprod(X / 2 + 0.75)
cmn = cummin(X - 0.5)
cmx = cummax(X)
S1 = X[11:70, 3:9]
S2 = X[44:48, ]
X2 = X
X2[31:62, 2:4] = matrix(7, rows=32, cols=3)
X3 = X
X3[5:64, ] = A[1:60, 1:30]
E = removeEmpty(target = X * (X > 0.9), margin = "rows")
tr = trace(X[1:30, ])
Tb = table(round(X[, 1] * 3) + 1, round(X[, 2] * 2) + 1)
Z = rand(rows=400, cols=200, sparsity=0.1, seed=5)
U = rand(rows=400, cols=5, seed=6)
V = rand(rows=200, cols=5, seed=7)
ws = sum((Z != 0) * (Z - U %*% t(V))^2)
wd = ((Z != 0) * (U %*% t(V))) %*% V
wl = t(t(U) %*% ((Z != 0) * (U %*% t(V))))
zs = sum(Z)
zc = colSums(Z)
zt = t(Z) %*% U
"""
OUTS = ["A", "T1", "T2", "G", "R1", "R2", "cs", "cp", "cmn", "cmx", "S1", "S2", "X2", "X3", "E", "tr", "Tb",
        "ws", "wd", "wl", "zs", "zc", "zt"]


def _np(v):
    from systemml_amd.parallel import dist as D
    from systemml_amd.ops import sparse as SP
    if isinstance(v, D.DistMatrix):
        v = D.gather(v)
    if hasattr(v, "layout"):
        v = SP.densify(v)
        return v.double().cpu().numpy()
    return np.array(v, dtype=float)


def _run(cfg, dist=None):
    from systemml_amd.api import executor as EX
    from systemml_amd.parallel import dist as D
    cs = EX.compile_script(SRC, {}, outputs=OUTS, config=cfg)
    res, _ = EX.execute(cs, {}, out=lambda s: None, dist=dist)
    out = {}
    kinds = {}
    for k in OUTS:
        v = res[k]
        kinds[k] = "dist" if isinstance(v, D.DistMatrix) else type(v).__name__
        if isinstance(v, D.DistMatrix):
            from systemml_amd.ops import sparse as SP
            kinds[k] += "-csr" if SP.is_sparse(v.local) else ""
            v = D.gather(D.DistMatrix(SP.densify(v.local), v.nrows, v.ncols, v.start, v.ctx))
        out[k] = _np(v)
    return out, kinds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SRC_BAD_LIX = """
X = rand(rows=90, cols=30, seed=1)
X[1:10, 1:2] = matrix(1, rows=3, cols=2)
s = sum(X)
"""


def _worker(rank, world, port, q, mode="ops"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from systemml_amd.parallel import dist as D
        from systemml_amd.conf import DMLConfig
        ctx = D.init(backend="gloo")
        D.reset_stats()
        if mode == "badlix":
            from systemml_amd.api import executor as EX
            cs = EX.compile_script(SRC_BAD_LIX, {}, outputs=["s"], config=DMLConfig(gpu=False, dist_min_rows=20))
            try:
                EX.execute(cs, {}, out=lambda s: None, dist=ctx)
                q.put((rank, "no error", None, None, None))
            except Exception as e:  # noqa: BLE001
                q.put((rank, None, type(e).__name__ + ": " + str(e), None, None))
            return
        out, kinds = _run(DMLConfig(gpu=False, dist_min_rows=20, seed=3), ctx)
        q.put((rank, out, kinds, dict(D.stats), dict(D.fallback_sites)))
        D.shutdown()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc(), None, None, None))


def _spmd(world, mode="ops"):
    import torch.multiprocessing as mp
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    return sorted(res, key=lambda r: r[0])


@pytest.mark.parametrize("world", [2, 3])
def test_dist_operators_match_single_process(world):
    from systemml_amd.conf import DMLConfig
    ref, _ = _run(DMLConfig(gpu=False, seed=3))
    res = _spmd(world)
    for r in res:
        assert not isinstance(r[1], str), r[1]
    for rank, out, kinds, stats, sites in res:
        for k in OUTS:
            np.testing.assert_allclose(out[k], ref[k], rtol=1e-10, atol=1e-10, err_msg=f"{k} (rank {rank})")
        assert stats["fallback_gathers"] == 0, sites
        # the large results stay row-partitioned; small ones are replicated
        for k in ("A", "T1", "G", "R1", "R2", "cs", "S1", "X2", "X3", "E", "wd"):
            assert kinds[k].startswith("dist"), (k, kinds[k])
        for k in ("T2", "S2", "Tb", "wl"):
            assert not kinds[k].startswith("dist"), (k, kinds[k])
        assert stats["alltoall"] > 0


def test_dist_lix_shape_error_raises_on_every_rank():
    """A left-indexing source of the wrong shape into a row window only rank 0 owns: every
    rank reports the error (no rank moves on to the next collective and hangs)."""
    res = _spmd(2, "badlix")
    for rank, err_none, msg, _, _ in res:
        assert err_none is None, (rank, err_none)
        assert "dimension mismatch" in msg, (rank, msg)


def test_partitioned_reads(tmp_path):
    """CSV (native row-range parser) and binary (memory-mapped slice) reads: each rank only
    materialises its own rows."""
    import torch
    from systemml_amd.io import writers
    rng = np.random.default_rng(0)
    X = rng.standard_normal((101, 7))
    writers.write(None, torch.from_numpy(X), str(tmp_path / "X.csv"), format="csv")
    writers.write(None, torch.from_numpy(X), str(tmp_path / "X.bin"), format="binary")
    writers.write(None, torch.from_numpy(X), str(tmp_path / "X.nat"), format="native")
    from systemml_amd.ops import native
    if native.lib() is None:
        pytest.skip("native IO library not built")
    got, total = native.parse_csv_rows(str(tmp_path / "X.csv"), 30, 64)
    assert total == 101
    np.testing.assert_allclose(got, X[30:64])
    res = _spmd_read(str(tmp_path), 3)
    for rank, blocks in res:
        assert not isinstance(blocks, str), blocks
        for name, (start, loc, full) in blocks.items():
            np.testing.assert_allclose(loc, X[start:start + loc.shape[0]])
            np.testing.assert_allclose(full, X)


def _read_worker(rank, world, port, d, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from systemml_amd.parallel import dist as D
        from systemml_amd.conf import DMLConfig
        from systemml_amd.io import readers
        from systemml_amd.runtime.program import ExecutionContext
        ctx = D.init(backend="gloo")
        ectx = ExecutionContext(None, DMLConfig(gpu=False, dist_min_rows=50), dist=ctx)
        blocks = {}
        for f in ("X.csv", "X.bin", "X.nat"):
            m = readers.read(ectx, os.path.join(d, f))
            assert isinstance(m, D.DistMatrix), type(m)
            blocks[f] = (m.start, m.local.double().numpy(), D.gather(m).double().numpy())
        q.put((rank, blocks))
        D.shutdown()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


def _spmd_read(d, world):
    import torch.multiprocessing as mp
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_read_worker, args=(r, world, port, d, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    return sorted(res, key=lambda r: r[0])
