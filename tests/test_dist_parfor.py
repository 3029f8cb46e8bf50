"""SPMD ("remote") parfor: iterations are split across `gloo` ranks, each rank runs its range
with rank-local operators and the result variables are merged across ranks.  Results must
equal single-process execution -- including random numbers drawn inside the body (per-
iteration seed streams) -- and the data-parallel LeNet example (synchronous SGD with a parfor
over mini-batches) must train to the same weights on 2 ranks as on 1.  Reference analogue:
test/integration/functions/parfor/ParForRemoteSpark*Test and the nn distributed-SGD example."""
import os
import socket

import numpy as np

SRC_SIMPLE = """
R = matrix(0, rows=10, cols=4)
parfor (i in 1:10) {
  v = rand(rows=1, cols=4, seed=-1)
  R[i, ] = v * i
}
S = matrix(0, rows=1, cols=7)
parfor (j in 2:6, par=2) {
  S[1, j] = j * j
}
A = matrix(7, rows=3, cols=2)
acc = matrix(0, rows=1, cols=1)
parfor (i in 1:10) {
  A += matrix(i, rows=3, cols=2)
  acc += matrix(i, rows=1, cols=1)
}
C = matrix(0, rows=1, cols=2)
parfor (i in 1:4, check=0) {
  C[1, 1] = i
}
z = sum(R) + sum(S)
"""

SRC_LENET = """
source("nn/examples/mnist_lenet_distrib_sgd.dml") as dsgd
[X, Y] = dsgd::generate_dummy_data(48, 1, 12, 12, 4)
[W1, b1, W2, b2, W3, b3, W4, b4] = dsgd::train(X, Y, X[1:8, ], Y[1:8, ], 1, 12, 12, 6, 4, 1)
"""
SIMPLE_OUT = ["R", "S", "z", "A", "acc", "C"]
LENET_OUT = ["W1", "b1", "W2", "b2", "W3", "b3", "W4", "b4"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(src, outs, dist=None):
    from systemml_amd.api import executor as EX
    from systemml_amd.api.mlcontext import SCRIPTS_DIR
    from systemml_amd.conf import DMLConfig
    cfg = DMLConfig(gpu=False, seed=11, parallelism=1)
    cs = EX.compile_script(src, {}, outputs=outs, config=cfg, filename=os.path.join(SCRIPTS_DIR, "x.dml"))
    res, _ = EX.execute(cs, {}, out=lambda s: None, dist=dist)
    return {k: (res[k].double().numpy() if hasattr(res[k], "numpy") else np.array(res[k], dtype=float))
            for k in outs}


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from systemml_amd.parallel import dist as D
        ctx = D.init(backend="gloo")
        D.reset_stats()
        a = _run(SRC_SIMPLE, SIMPLE_OUT, ctx)
        b = _run(SRC_LENET, LENET_OUT, ctx)
        q.put((rank, a, b, dict(D.stats)))
        D.shutdown()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc(), None, None))


def test_spmd_parfor_matches_single_process():
    import torch.multiprocessing as mp
    ref_a = _run(SRC_SIMPLE, SIMPLE_OUT)
    assert ref_a["A"].min() == 62 and float(ref_a["acc"].sum()) == 55 and ref_a["C"][0, 0] == 4
    ref_b = _run(SRC_LENET, LENET_OUT)
    world = 2
    port = _free_port()
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    procs = [mctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, a, b, st in res:
        assert not isinstance(a, str), a
        for k in ref_a:
            np.testing.assert_allclose(a[k], ref_a[k], rtol=1e-12, err_msg=k)
        for k in ref_b:
            np.testing.assert_allclose(b[k], ref_b[k], rtol=1e-9, atol=1e-12, err_msg=k)
        assert st.get("parfor_remote", 0) >= 3          # 2 simple loops + the training parfor(s)
        assert st["fallback_gathers"] == 0
    np.testing.assert_array_equal(ref_a["S"].ravel(), [0, 4, 9, 16, 25, 36, 0])
