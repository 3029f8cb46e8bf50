"""Generated Row-template kernels (ops/rowgen.py) on the MI355X: effective HBM bandwidth of
typical row programs over a tall matrix (bytes of the distinct inputs read once + output).

    python tools/bench_rowgen.py [--rows 4000000] [--cols 1000] [--reps 10]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from systemml_amd.conf import DMLConfig  # noqa: E402
from systemml_amd.ops import rowgen as R  # noqa: E402
from systemml_amd.ops.backend import backend  # noqa: E402


def progs():
    return {
        # t(X) %*% (exp(X %*% v) - y)
        "tmv_exp_chain": (R.RowProgram(3, [("dot", None, 0, 1), ("u", "exp", 3, 0), ("b", "-", 4, 2)], 0, "tmv",
                                       extra=5), ["X", "v", "y"]),
        # y - X %*% b (residuals)
        "residual": (R.RowProgram(3, [("dot", None, 0, 1), ("b", "-", 2, 3)], 4, "vec"), ["X", "v", "y"]),
        # X / rowSums(X)
        "row_normalise": (R.RowProgram(1, [("ragg", "sum", 0, 0), ("b", "/", 0, 1)], 2, "vec"), ["X"]),
        # colSums(X * (X %*% v))
        "colsum_scaled": (R.RowProgram(2, [("dot", None, 0, 1), ("b", "*", 0, 2)], 3, "col", oagg="sum"), ["X", "v"]),
        # sum((X - rowMeans(X))^2)
        "centered_sumsq": (R.RowProgram(1, [("ragg", "mean", 0, 0), ("b", "-", 0, 1)], 2, "all", oagg="sumsq"), ["X"]),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4_000_000)
    ap.add_argument("--cols", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--dtypes", default="bf16,fp32")
    a = ap.parse_args()
    backend.configure(DMLConfig(gpu=True, precision="single"))
    dev = torch.device("cuda:0")
    n, d = a.rows, a.cols
    res = []
    for dname in a.dtypes.split(","):
        dt = {"bf16": torch.bfloat16, "fp32": torch.float32}[dname]
        X = (torch.rand((n, d), device=dev) - 0.5).to(dt)
        data = {"X": X, "v": torch.rand((d, 1), device=dev) / d, "y": torch.rand((n, 1), device=dev)}
        for name, (prog, ins) in progs().items():
            if name == "row_normalise" and dname == "bf16":
                pass
            args = [data[k] for k in ins]
            r = R._kernel(prog, args)                      # compile + warm
            assert r is not None, name
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                r = R._kernel(prog, args)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.reps * 1e3
            nbytes = sum(t.numel() * t.element_size() for t in args)
            if isinstance(r, torch.Tensor):
                nbytes += r.numel() * r.element_size()
            res.append({"prog": name, "describe": prog.describe(), "dtype": dname, "rows": n, "cols": d,
                        "ms": round(ms, 3), "TBps": round(nbytes / ms / 1e9, 2)})
            print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
