"""Micro-run of the fused tall-skinny chain kernels on the headline matrix (10M x 1K bf16):
XtPSXv (MultiLogReg Hessian-vector product) and XTSMG (fused softmax gradient), for
rocprofv3 --pmc passes and A/B timing.   python tools/bench_chain.py [--reps 5] [--rows N]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--cols", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--variants", default="")
    a = ap.parse_args()
    from systemml_amd.ops import kernels as K
    from systemml_amd.ops.backend import backend
    from systemml_amd.conf import DMLConfig
    backend.configure(DMLConfig(precision="single"))
    dev = torch.device("cuda")
    X = torch.empty((a.rows, a.cols), dtype=torch.bfloat16, device=dev)
    for s in range(0, a.rows, 1 << 20):
        X[s:s + (1 << 20)] = torch.rand((min(1 << 20, a.rows - s), a.cols), device=dev)
    v4 = torch.randn((a.cols, 4), device=dev) * 0.01
    P = torch.softmax(torch.randn((a.rows, 5), device=dev), 1)[:, :4].contiguous()
    Y = (torch.rand((a.rows, 4), device=dev) < 0.2).float()
    cases = {"XtPSXv": lambda: K.mmchain("XtPSXv", X, v4, P), "smgrad": lambda: K.smgrad(X, v4, Y),
             "XtXv": lambda: K.mmchain("XtXv", X, v4[:, :1])}
    if a.only:
        cases = {k: v for k, v in cases.items() if k in a.only.split(",")}
    res = {}
    variants = [("chain4m", True, True, 1), ("chain4m.v0", True, True, 0), ("chain4", True, False, 0),
                ("rowstream", False, False, 0)]
    if a.variants:
        variants = [v for v in variants if v[0] in a.variants.split(",")]
    for name0, fn in list(cases.items()):
      for vname, flag, mflag, var in variants:
        K.CHAIN4 = flag
        K.C4M = mflag
        K.C4M_VARIANT = var
        name = f"{name0}/{vname}"
        fn()
        ts = []
        for _ in range(a.reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e))
        ts.sort()
        ms = ts[len(ts) // 2]
        res[name] = {"ms": ms, "TBps": X.numel() * 2 / ms / 1e9}
        print(json.dumps({name: res[name]}), flush=True)


if __name__ == "__main__":
    main()
