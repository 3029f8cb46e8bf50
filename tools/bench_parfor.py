"""parfor on the GPU backend against the sequential for loop: `iters` independent bodies, each a
(n x n) GEMM plus a reduction written into a result row (reference ParForProgramBlock with
GPUContextPool: one device context per worker; here one stream per worker thread, and with
config.parfor_gpus > 1 one GPU per worker).  Prints the best-of-`reps` wall time of each
variant, their ratio and whether the results agree.

    python tools/bench_parfor.py [--n 4096] [--iters 4] [--par 4] [--precision single] [--reps 5]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def run(n, iters, par, precision, reps, gpus):
    from systemml_amd.api import executor as EX
    from systemml_amd.conf import DMLConfig
    g = torch.Generator(device="cuda").manual_seed(5)
    dt = torch.float64 if precision == "double" else torch.float32
    # device-resident inputs: the timed runs measure the loops, not host -> device copies
    ins = {"A": torch.rand((n, n), generator=g, device="cuda", dtype=dt) * 2 - 1,
           "B": torch.rand((n, n), generator=g, device="cuda", dtype=dt) * 2 - 1}
    body = "{\n  C = (A + i) %*% B\n  R[1, i] = sum(C * C)\n}"
    srcs = {"seq": f"R = matrix(0, rows=1, cols={iters})\nfor (i in 1:{iters}) " + body,
            "par": f"R = matrix(0, rows=1, cols={iters})\nparfor (i in 1:{iters}, par={par}) " + body}
    cfg = DMLConfig(gpu=True, precision=precision, gpu_min_cells=0)
    cfg.parfor_gpus = gpus
    times, out, plans = {}, {}, {}
    for k, src in srcs.items():
        cs = EX.compile_script(src, {}, inputs=ins, outputs=["R"], config=cfg)
        best = 1e9
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r, _ = EX.execute(cs, ins)
            v = r["R"].double().cpu().numpy()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        times[k] = best
        out[k] = v
        pf = [b for b in cs.cp.blocks if hasattr(b, "last_plan")]
        plans[k] = repr(pf[0].last_plan) if pf else "-"
    ok = np.allclose(out["par"], out["seq"], rtol=1e-5)
    return times, ok, plans


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--par", type=int, default=4)
    ap.add_argument("--precision", default="single")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--gpus", type=int, default=1)
    a = ap.parse_args()
    times, ok, plans = run(a.n, a.iters, a.par, a.precision, a.reps, a.gpus)
    print(f"n={a.n} iters={a.iters} par={a.par} {a.precision}: seq {times['seq'] * 1e3:.2f} ms, "
          f"parfor {times['par'] * 1e3:.2f} ms, speedup {times['seq'] / times['par']:.2f}x, agree={ok}  "
          f"plan {plans['par']}", flush=True)


if __name__ == "__main__":
    main()
