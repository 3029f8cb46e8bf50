"""Fused cellwise kernel (ops/hip/cell.hip) vs the same operators as separate torch kernels.

Usage: python tools/bench_cell.py [--rows N] [--cols M]
Prints one JSON line per case: kernel ms, unfused torch ms, effective GB/s of the fused pass
(bytes of the distinct inputs read + output written, divided by time)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from systemml_amd.conf import DMLConfig  # noqa: E402
from systemml_amd.ops import cell  # noqa: E402
from systemml_amd.ops.backend import backend  # noqa: E402
from systemml_amd.ops.cell import CellProgram  # noqa: E402


def _time(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--cols", type=int, default=5)
    a = ap.parse_args()
    backend.configure(DMLConfig(gpu=True, precision="single"))
    dev = torch.device("cuda:0")
    n, m = a.rows, a.cols
    X = torch.rand(n, m, device=dev)
    Y = torch.rand(n, m, device=dev)
    y = torch.rand(n, 1, device=dev)
    cases = {
        # exp((X - y) * Y): 3 operators, 2 full inputs + a column vector
        "exp3": (CellProgram([("b", "-", 3, 0, 2), ("b", "*", 3, 3, 1), ("u", "exp", 3, 3, 0)], 3, 3),
                  [X, Y, y], lambda: torch.exp((X - y) * Y), 3 * n * m * 4),
        "copy": (CellProgram([("b", "+", 1, 0, 1)], 2, 1), [X, 0.0], lambda: X + 0.0, 2 * n * m * 4),
        "rowsum_exp": (CellProgram([("b", "-", 0, 0, 1), ("u", "exp", 0, 0, 0)], 2, 0, ("sum", "row")),
                       [X, y], lambda: torch.exp(X - y).sum(1, keepdim=True), n * m * 4 + 2 * n * 4),
        "sum_sq_diff": (CellProgram([("b", "-", 0, 0, 1), ("u", "sq", 0, 0, 0)], 2, 0, ("sum", "all")),
                        [X, Y], lambda: ((X - Y) ** 2).sum(), 2 * n * m * 4),
        "colsum_log": (CellProgram([("b", "+", 0, 0, 1), ("u", "log", 0, 0, 0)], 2, 0, ("sum", "col")),
                       [X, 1.0], lambda: torch.log(X + 1.0).sum(0, keepdim=True), n * m * 4),
    }
    for (name, (prog, args, ref, nbytes)), rtc in [(c, r) for r in (True, False) for c in cases.items()]:
        cell.RTC = rtc
        got = cell._kernel(prog, args)
        r = ref()
        torch.cuda.synchronize()
        g = torch.as_tensor(got.value() if hasattr(got, "value") else got)
        err = float((g.double().cpu() - r.double().cpu()).abs().max() / (r.double().abs().max() + 1e-30))
        tk = _time(lambda: cell._kernel(prog, args))
        tt = _time(ref)
        print(json.dumps({"case": name, "path": "generated" if rtc else "interpreter", "rows": n, "cols": m, "kernel_ms": round(tk, 4), "torch_ms": round(tt, 4),
                          "kernel_GBps": round(nbytes / tk / 1e6, 1), "rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
