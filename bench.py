#!/usr/bin/env python
"""Headline benchmark (BASELINE.json): end-to-end seconds for LinregCG + MultiLogReg
on a 10M x 1K dense synthetic matrix (perftest settings), on N GPUs of one node.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = compile + execute scripts/algorithms/LinearRegCG.dml (icpt=0, maxi=20,
tol=1e-4, reg=0.01) followed by compile + execute scripts/algorithms/MultiLogReg.dml
(k=5 classes, icpt=0, moi=20, mii=5, tol=1e-4, reg=0.01) — the reference's
scripts/perftest/runLinearRegCG.sh / runMultiLogReg.sh settings.  Synthetic data is
generated directly in HBM (dense, sparsity 0.9 as genMultinomialData.sh), row-
partitioned across ranks (strong scaling: total work fixed), outside the timed region.
X is stored bf16 (fp32 accumulation in every kernel); all vectors/iterates are fp32.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

METRIC = "end-to-end sec for LinregCG + MLogReg on 10Mx1K dense (perftest) at 1/2/4/8 GPU"


def gen_data(ctx, rows, cols, classes, dtype, seed=7):
    """Dense synthetic X (90% non-zeros), regression target y and class labels, row-partitioned."""
    from systemml_amd.parallel import dist as D
    from systemml_amd.ops import core as C
    dev = torch.device("cuda", torch.cuda.current_device())
    if ctx is not None:
        s, e = ctx.partition(rows)
    else:
        s, e = 0, rows
    n = e - s
    g = torch.Generator(device=dev)
    g.manual_seed(seed + 7919 * s)
    X = torch.empty((n, cols), dtype=dtype, device=dev)
    step = 1 << 19
    for a in range(0, n, step):
        b = min(n, a + step)
        blk = torch.rand((b - a, cols), generator=g, device=dev)
        blk.mul_(torch.rand((b - a, cols), generator=g, device=dev) < 0.9)
        X[a:b] = blk.to(dtype)
        del blk
    gw = torch.Generator(device=dev)
    gw.manual_seed(seed)            # identical model weights on every rank
    w = torch.randn((cols, 1), generator=gw, device=dev)
    W = torch.randn((cols, classes), generator=gw, device=dev)
    y = C.mm(X, w) + 0.1 * torch.randn((n, 1), generator=g, device=dev)
    sc = C.mm(X, W)
    sc = sc - sc.mean(1, keepdim=True)
    gum = -torch.log(-torch.log(torch.rand((n, classes), generator=g, device=dev).clamp_min(1e-20)))
    lab = (torch.argmax(sc / sc.std() * 2.0 + gum, 1, keepdim=True) + 1).float()
    if ctx is not None:
        return (D.from_local(ctx, X, rows), D.from_local(ctx, y.contiguous(), rows),
                D.from_local(ctx, lab.contiguous(), rows))
    return X, y.contiguous(), lab.contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--cols", type=int, default=1000)
    ap.add_argument("--classes", type=int, default=5)
    ap.add_argument("--xdtype", default="bf16", choices=["bf16", "fp32", "fp64"])
    ap.add_argument("--maxi", type=int, default=20)
    ap.add_argument("--moi", type=int, default=20)
    ap.add_argument("--mii", type=int, default=5)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--stats", action="store_true")
    a = ap.parse_args()

    from systemml_amd.parallel import dist as D
    from systemml_amd.conf import DMLConfig
    from systemml_amd.api import executor as EX
    from systemml_amd.api.mlcontext import SCRIPTS_DIR
    from systemml_amd.ops import kernels
    from systemml_amd.utils.stats import Statistics

    world = int(os.environ.get("WORLD_SIZE", "1"))
    ctx = D.init() if world > 1 else None
    rank = ctx.rank if ctx else 0
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    if ctx is None:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))

    cfg = DMLConfig(precision="single", dist_min_rows=100_000)
    from systemml_amd.ops.backend import backend
    backend.configure(cfg)
    xdt = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp64": torch.float64}[a.xdtype]
    if a.xdtype == "fp64":
        cfg.precision = "double"
        backend.configure(cfg)

    t0 = time.perf_counter()
    X, y, lab = gen_data(ctx, a.rows, a.cols, a.classes, xdt)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0

    with open(os.path.join(SCRIPTS_DIR, "algorithms", "LinearRegCG.dml")) as f:
        src_lr = f.read()
    with open(os.path.join(SCRIPTS_DIR, "algorithms", "MultiLogReg.dml")) as f:
        src_mlr = f.read()
    args_lr = dict(X="X", Y="y", B="B", icpt=0, maxi=a.maxi, tol=0.0001, reg=0.01, fmt="csv")
    args_mlr = dict(X="X", Y="Y", B="B", icpt=0, reg=0.01, tol=0.0001, moi=a.moi, mii=a.mii)
    log = []
    out = (lambda s: log.append(s)) if not a.verbose else (lambda s: print(s, file=sys.stderr))

    def step(stats=None):
        cs1 = EX.compile_script(src_lr, args_lr, inputs={"X": X, "y": y}, outputs=["B_out"], config=cfg)
        r1, _ = EX.execute(cs1, {"X": X, "y": y}, out=out, dist=ctx, stats=stats)
        cs2 = EX.compile_script(src_mlr, args_mlr, inputs={"X": X, "Y_vec": lab}, outputs=["B_out"], config=cfg)
        r2, _ = EX.execute(cs2, {"X": X, "Y_vec": lab}, out=out, dist=ctx, stats=stats)
        return r1["B_out"], r2["B_out"]

    for _ in range(a.warmup):
        step()
    if ctx:
        ctx.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    st = Statistics(enabled=True) if a.stats else None
    for _ in range(a.steps):
        b1, b2 = step(st)
    torch.cuda.synchronize()
    if ctx:
        ctx.barrier()
    el = time.perf_counter() - t1
    if ctx:
        el = ctx.allreduce_scalar(el, "max")
    sec = el / a.steps
    if rank == 0:
        if st is not None:
            print(st.report(25), file=sys.stderr)
        if a.verbose:
            print(f"datagen {t_gen:.2f}s, kernels {kernels.counters}, dist {D.stats}", file=sys.stderr)
        res = {
            "metric": METRIC, "value": round(sec, 4), "unit": "s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(sec * 1000, 2), "higher_is_better": False,
            "scaling": "strong", "vs_baseline": None, "dtype": "bf16" if a.xdtype == "bf16" else a.xdtype,
            "data": "synthetic (in-HBM datagen, dense sparsity 0.9)",
            "config": {"model": "LinregCG+MultiLogReg (perftest: maxi=%d; k=%d moi=%d mii=%d)"
                                % (a.maxi, a.classes, a.moi, a.mii),
                       "global_batch": a.rows, "seq_len": a.cols, "rows": a.rows, "cols": a.cols,
                       "parallelism": f"dp{world}", "x_storage": a.xdtype, "accumulate": "fp32"},
        }
        print(json.dumps(res), flush=True)
    if ctx:
        D.shutdown()


if __name__ == "__main__":
    main()
