"""Host-side launch overhead of the generated fused operators (ops/cell.py, ops/rowgen.py)
against the torch operators they replace: wall time per call with the device kept busy
asynchronously (no syncs inside the loop), plus a cProfile breakdown of the fused path.

    python tools/bench_launch.py [--reps 2000] [--profile out.txt]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from systemml_amd.conf import DMLConfig  # noqa: E402
from systemml_amd.ops import cell, rowgen  # noqa: E402
from systemml_amd.ops.backend import backend  # noqa: E402
from systemml_amd.ops.cell import CellProgram  # noqa: E402


def timed(f, reps):
    for _ in range(20):
        f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        f()
    host = (time.perf_counter() - t) / reps * 1e6
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t) / reps * 1e6
    return round(host, 1), round(tot, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2000)
    ap.add_argument("--profile", default="")
    a = ap.parse_args()
    backend.configure(DMLConfig(gpu=True, precision="single", gpu_min_cells=0))
    dev = torch.device("cuda", torch.cuda.current_device())
    res = {}
    for n, m in ((32, 64 * 56 * 56), (1024, 1000), (32, 2048)):
        X = torch.randn((n, m), device=dev)
        Y = torch.randn((n, m), device=dev)
        w = torch.randn((1, m), device=dev)
        # (X - w) * Y + 0.5 (3 ops)
        prog = CellProgram([("b", "-", 4, 0, 2), ("b", "*", 4, 4, 1), ("b", "+", 4, 4, 3)], 4, 4)
        args = [X, Y, w, 0.5]
        res[f"cell3 {n}x{m}"] = timed(lambda: cell._kernel(prog, args), a.reps)
        res[f"torch3 {n}x{m}"] = timed(lambda: (X - w) * Y + 0.5, a.reps)
        rp = rowgen.RowProgram(1, [("ragg", "sum", 0, 0), ("b", "/", 0, 1)], 2, "vec")
        res[f"row {n}x{m}"] = timed(lambda: rowgen._kernel(rp, [X]), a.reps)
        res[f"torch_row {n}x{m}"] = timed(lambda: X / X.sum(1, keepdim=True), a.reps)
    for k, v in res.items():
        print(f"{k:28s} host us/call {v[0]:8.1f}   wall us/call {v[1]:8.1f}")
    if a.profile:
        X = torch.randn((1024, 1000), device=dev)
        Y = torch.randn((1024, 1000), device=dev)
        w = torch.randn((1, 1000), device=dev)
        prog = CellProgram([("b", "-", 4, 0, 2), ("b", "*", 4, 4, 1), ("b", "+", 4, 4, 3)], 4, 4)
        rp = rowgen.RowProgram(1, [("ragg", "sum", 0, 0), ("b", "/", 0, 1)], 2, "vec")
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(a.reps):
            cell._kernel(prog, [X, Y, w, 0.5])
            rowgen._kernel(rp, [X])
        pr.disable()
        torch.cuda.synchronize()
        buf = io.StringIO()
        pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(30)
        with open(a.profile, "w") as f:
            f.write(buf.getvalue())


if __name__ == "__main__":
    main()
