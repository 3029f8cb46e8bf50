#!/usr/bin/env python
"""Headline benchmark (BASELINE.json): end-to-end seconds for LinregCG + MultiLogReg
on a 10M x 1K dense synthetic matrix (perftest settings), on N GPUs of one node.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = compile + execute scripts/algorithms/LinearRegCG.dml (icpt=0, maxi=20,
tol=1e-4, reg=0.01) followed by compile + execute scripts/algorithms/MultiLogReg.dml
(k=5 classes, icpt=0, moi=20, mii=5, tol=1e-4, reg=0.01) — the reference's
scripts/perftest/runLinearRegCG.sh / runMultiLogReg.sh settings.  The inputs follow the
perftest data generators (gen_data below), are generated directly in HBM and row-
partitioned across ranks (strong scaling: total work fixed), outside the timed region.
X is stored bf16 (fp32 accumulation in every kernel); all vectors/iterates are fp32.
"""
from __future__ import annotations

import argparse
import gc
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

METRIC = "end-to-end sec for LinregCG + MLogReg on 10Mx1K dense (perftest) at 1/2/4/8 GPU"


def gen_data(ctx, rows, cols, classes, dtype, sparsity=0.9, seed=7):
    """The perftest inputs, generated directly in HBM and row-partitioned across ranks
    (each rank draws its rows from its own generator stream; model weights come from a
    shared seed so every rank uses the same ones):

    * LinregCG runs on the binomial data of scripts/perftest/genBinomialData.sh ->
      scripts/datagen/genRandData4LogisticRegression.dml (N 1000 maxFeature=5 maxWeight=5,
      addNoise=1, no intercept, sparsity 0.9, labels 1/2):
        X = 5 * U(-1, 1) with 90% non-zeros,  w = 5 * U(-1, 1),
        y = 1 + (sigmoid(X w) >= r),  r ~ U(0, 1)
    * MultiLogReg runs on the multinomial data of genMultinomialData.sh ->
      scripts/datagen/genRandData4Multinomial.dml (N 1000 sparsity 0.9, 5 categories, no
      intercept):
        X = U(1, 5) with 90% non-zeros,  B = U(-1, 1) * 3 / sqrt(1000 * 0.9)  (D x 4),
        P = exp(X B) / (1 + rowSums(exp(X B))),  y = 1 + rowSums(cumsum(P) < r),
        and the last 5 rows take labels 1..5 so every class occurs.
    """
    from systemml_amd.parallel import dist as D
    dev = torch.device("cuda", torch.cuda.current_device())
    s, e = ctx.partition(rows) if ctx is not None else (0, rows)
    n = e - s
    g = torch.Generator(device=dev)
    g.manual_seed(seed + 7919 * s)
    gw = torch.Generator(device=dev)
    gw.manual_seed(seed)
    w = (torch.rand((cols, 1), generator=gw, device=dev) * 2 - 1) * 5.0
    B = (torch.rand((cols, classes - 1), generator=gw, device=dev) * 2 - 1) * (3.0 / math.sqrt(cols * sparsity))
    X1 = torch.empty((n, cols), dtype=dtype, device=dev)
    X2 = torch.empty((n, cols), dtype=dtype, device=dev)
    y1 = torch.empty((n, 1), device=dev)
    y2 = torch.empty((n, 1), device=dev)
    step = 1 << 18
    for a in range(0, n, step):
        b = min(n, a + step)
        m = b - a
        blk = torch.rand((m, cols), generator=g, device=dev).mul_(10.0).sub_(5.0)
        blk.mul_(torch.rand((m, cols), generator=g, device=dev) < sparsity)
        xb = blk.to(dtype)
        X1[a:b] = xb
        prob = torch.sigmoid(xb.float() @ w)
        y1[a:b] = 1.0 + (prob >= torch.rand((m, 1), generator=g, device=dev)).float()
        blk = torch.rand((m, cols), generator=g, device=dev).mul_(4.0).add_(1.0)
        blk.mul_(torch.rand((m, cols), generator=g, device=dev) < sparsity)
        xb = blk.to(dtype)
        X2[a:b] = xb
        E = torch.exp(xb.float() @ B)
        P = torch.cumsum(E / (1.0 + E.sum(1, keepdim=True)), 1)
        y2[a:b] = 1.0 + (P < torch.rand((m, 1), generator=g, device=dev)).float().sum(1, keepdim=True)
        del blk, xb, prob, E, P
    if e == rows and n >= classes:
        y2[n - classes:] = torch.arange(1, classes + 1, device=dev, dtype=torch.float32).reshape(-1, 1)
    if ctx is not None:
        return tuple(D.from_local(ctx, t, rows) for t in (X1, y1, X2, y2))
    return X1, y1, X2, y2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--cols", type=int, default=1000)
    ap.add_argument("--classes", type=int, default=5)
    ap.add_argument("--xdtype", default="bf16", choices=["bf16", "fp32", "fp64"])
    ap.add_argument("--maxi", type=int, default=20)
    ap.add_argument("--moi", type=int, default=20)
    ap.add_argument("--mii", type=int, default=5)
    ap.add_argument("--icpt", type=int, default=0, choices=[0, 1, 2],
                    help="intercept mode of both scripts (perftest runs 0, 1 and 2; the headline is 0)")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--stats", action="store_true")
    ap.add_argument("--gpu-min-cells", type=int, default=None,
                    help="host-placement threshold for small matrices (default: config default)")
    ap.add_argument("--lazy", action="store_true",
                    help="HBM-resident lazy scalars (all matrices in HBM) instead of host scalars + hybrid "
                         "placement (measured slower on this benchmark: 511 vs 486 ms)")
    ap.add_argument("--sample-profile", default="",
                    help="wall-clock stack samples of the timed steps (tools/stack_sampler.py) written here")
    ap.add_argument("--host-profile", default="",
                    help="cProfile the timed steps (host time) and write the top functions to this file")
    ap.add_argument("--reuse-plans", action="store_true",
                    help="diagnostic only (not the headline metric): compile both scripts once and re-execute "
                         "the plans every step, to separate compilation from execution cost")
    ap.add_argument("--no-overlap", action="store_true",
                    help="compile MultiLogReg after LinregCG ran instead of overlapping the two")
    ap.add_argument("--compiler", default="process", choices=["process", "thread"],
                    help="where the next step's scripts compile while this step executes: a compiler "
                         "process (api/compile_service.py, off the executor's interpreter lock) or a thread")
    a = ap.parse_args()

    # the compiler service is started before anything touches the GPU (its process is spawned)
    svc = None
    if a.compiler == "process" and not a.no_overlap and not a.reuse_plans:
        from systemml_amd.api.compile_service import CompileService
        svc = CompileService()

    from systemml_amd.parallel import dist as D
    from systemml_amd.conf import DMLConfig
    from systemml_amd.api import executor as EX
    from systemml_amd.api.mlcontext import SCRIPTS_DIR
    from systemml_amd.ops import kernels
    from systemml_amd.utils.stats import Statistics

    world = int(os.environ.get("WORLD_SIZE", "1"))
    # SYSML_DIST_FORCE=1 runs the SPMD plan as one RCCL rank on one GPU (DIST overhead check)
    ctx = D.init() if world > 1 or os.environ.get("SYSML_DIST_FORCE") == "1" else None
    rank = ctx.rank if ctx else 0
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    if ctx is None:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))

    cfg = DMLConfig(precision="single", dist_min_rows=100_000, lazy_scalars=a.lazy)
    if a.gpu_min_cells is not None:
        cfg.gpu_min_cells = a.gpu_min_cells
    from systemml_amd.ops.backend import backend
    backend.configure(cfg)
    xdt = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp64": torch.float64}[a.xdtype]
    if a.xdtype == "fp64":
        cfg.precision = "double"
        backend.configure(cfg)

    t0 = time.perf_counter()
    X1, y1, X2, lab = gen_data(ctx, a.rows, a.cols, a.classes, xdt)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0

    with open(os.path.join(SCRIPTS_DIR, "algorithms", "LinearRegCG.dml")) as f:
        src_lr = f.read()
    with open(os.path.join(SCRIPTS_DIR, "algorithms", "MultiLogReg.dml")) as f:
        src_mlr = f.read()
    args_lr = dict(X="X", Y="y", B="B", icpt=a.icpt, maxi=a.maxi, tol=0.0001, reg=0.01, fmt="csv")
    args_mlr = dict(X="X", Y="Y", B="B", icpt=a.icpt, reg=0.01, tol=0.0001, moi=a.moi, mii=a.mii)
    log = []
    out = (lambda s: log.append(s)) if not a.verbose else (lambda s: print(s, file=sys.stderr))

    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(1)
    # the compile thread and the executing thread share the GIL: a short switch interval lets
    # the executor take it back promptly after each device wait (the 5 ms default leaves the
    # GPU idle while the compiler runs)
    sys.setswitchinterval(0.0005)

    def compile_lr():
        return EX.compile_script(src_lr, args_lr, inputs={"X": X1, "y": y1}, outputs=["B_out"], config=cfg)

    def compile_mlr():
        return EX.compile_script(src_mlr, args_mlr, inputs={"X": X2, "Y_vec": lab}, outputs=["B_out"], config=cfg)


    def compile_both():
        return compile_lr(), compile_mlr()

    class _Both:
        """The two compilations of one step, requested from the compiler process; the plans
        are received and hydrated (unpickled, instructions bound) on a host thread while this
        step's MultiLogReg runs, whose host thread mostly waits on the device."""

        def __init__(self):
            import threading
            self.p1 = svc.submit(src_lr, args_lr, {"X": X1, "y": y1}, ["B_out"], cfg, world=world)
            self.p2 = svc.submit(src_mlr, args_mlr, {"X": X2, "Y_vec": lab}, ["B_out"], cfg, world=world)
            self.err = None

            def hydrate():
                try:
                    self.p1.result()
                    self.p2.result()
                except BaseException as e:  # noqa: BLE001 - re-raised by result()
                    self.err = e
            self.th = threading.Thread(target=hydrate, daemon=True)
            self.th.start()

        def result(self):
            self.th.join()
            if self.err is not None:
                raise self.err
            r = self.p1.result(), self.p2.result()
            if a.verbose:
                print("compile service (worker s, wait s, hydrate s):", self.p1.times, self.p2.times, file=sys.stderr)
            return r

    def step(stats=None, cs=None, prefetch_next=False):
        # both scripts are parsed + compiled once per step.  The next step's two compilations
        # run on a host thread while this step's MultiLogReg executes (its ~350 ms of GPU work
        # leaves the host mostly waiting on the device, which releases the GIL), as a
        # pipelined driver would; LinregCG's short run keeps the host to itself
        cs1, cs2 = cs if cs is not None else compile_both()
        nxt = None
        if svc is not None and prefetch_next:
            nxt = _Both()            # compiles in the service process while this step runs
        r1, _ = EX.execute(cs1, {"X": X1, "y": y1}, out=out, dist=ctx, stats=stats)
        if svc is None and prefetch_next and not a.no_overlap:
            nxt = pool.submit(compile_both)
        r2, _ = EX.execute(cs2, {"X": X2, "Y_vec": lab}, out=out, dist=ctx, stats=stats)
        return r1["B_out"], r2["B_out"], (nxt.result() if nxt is not None else None)

    fixed = compile_both() if a.reuse_plans else None

    def run_steps(k, stats=None, cs=None):
        # every step compiles the scripts of the step after it while it executes (the last
        # warmup step compiles the first timed step's, the last timed step one more, awaited
        # before the clock stops): each timed step carries one compilation of both scripts
        cs = fixed if fixed is not None else cs
        for i in range(k):
            _, _, cs = step(stats, cs, prefetch_next=fixed is None and not a.no_overlap)
            cs = fixed if fixed is not None else cs
        return cs

    cs_next = run_steps(a.warmup)
    # compiled programs and the data live for the whole run: move them out of the cyclic
    # collector's generations so gen-2 collections during the steps stay short
    gc.collect()
    gc.freeze()
    if ctx:
        ctx.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    st = Statistics(enabled=True) if a.stats else None
    sampler = None
    if a.sample_profile:
        from tools.stack_sampler import Sampler
        sampler = Sampler().__enter__()
    prof = None
    if a.host_profile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    from systemml_amd.utils import hosttrace as HT
    HT.reset()
    run_steps(a.steps, st, cs_next)
    torch.cuda.synchronize()
    if HT.ON and rank == 0:
        print(HT.summary(), file=sys.stderr)
    if prof is not None:
        prof.disable()
    if sampler is not None:
        sampler.__exit__(None, None, None)
        if rank == 0:
            sampler.report(a.sample_profile)
    if ctx:
        ctx.barrier()
    el = time.perf_counter() - t1
    if ctx:
        el = ctx.allreduce_scalar(el, "max")
    sec = el / a.steps
    # physical GPUs used: distinct devices over the ranks (a gloo rehearsal puts several ranks
    # on one GPU and must not report them as several GPUs)
    n_phys = 1
    if ctx:
        import torch.distributed as tdist
        devs = [None] * world
        tdist.all_gather_object(devs, (os.uname().nodename, torch.cuda.current_device()))
        n_phys = len(set(devs))
        if rank == 0 and a.verbose:
            print(f"collectives per step: { {k: v / max(1, a.steps + a.warmup) for k, v in D.stats.items()} }",
                  file=sys.stderr)
    if prof is not None and rank == 0:
        import io
        import pstats
        buf = io.StringIO()
        ps = pstats.Stats(prof, stream=buf)
        ps.sort_stats("tottime").print_stats(45)
        ps.sort_stats("cumulative").print_stats(60)
        # who waits for the device: the callers of the blocking reads
        for fn in ("tolist", "synchronize", "'cpu'", "'item'", "'to'"):
            ps.print_callers(fn)
        with open(a.host_profile, "w") as f:
            f.write(buf.getvalue())
    if rank == 0:
        if st is not None:
            print(st.report(25), file=sys.stderr)
        if a.verbose:
            from systemml_amd.runtime import program as _PR, graphloop as _GL
            print(f"datagen {t_gen:.2f}s, kernels {kernels.counters}, dist {D.stats}", file=sys.stderr)
            print(f"run-ahead {_PR.runahead_stats}, graph replay {_GL.stats}", file=sys.stderr)
        res = {
            "metric": METRIC, "value": round(sec, 4), "unit": "s", "n_gpus": n_phys, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(sec * 1000, 2), "higher_is_better": False,
            "scaling": "strong", "vs_baseline": None, "dtype": "bf16" if a.xdtype == "bf16" else a.xdtype,
            "data": "synthetic (perftest generators genRandData4LogisticRegression / genRandData4Multinomial, "
                    "sparsity 0.9, generated in HBM)",
            "config": {"model": "LinregCG+MultiLogReg (perftest: maxi=%d; k=%d moi=%d mii=%d%s)%s"
                                % (a.maxi, a.classes, a.moi, a.mii, "" if a.icpt == 0 else f"; icpt={a.icpt}",
                                   " [DIAGNOSTIC: plans reused, compilation excluded]" if a.reuse_plans else ""),
                       "global_batch": a.rows, "seq_len": a.cols, "rows": a.rows, "cols": a.cols,
                       "parallelism": f"dp{world}" if n_phys == world else f"dp{world} ({world} ranks on {n_phys} GPU)", "x_storage": a.xdtype, "accumulate": "fp32"},
        }
        print(json.dumps(res), flush=True)
    if svc is not None:
        svc.close()
    if ctx:
        D.shutdown()


if __name__ == "__main__":
    main()
