"""Column-scan kernels (ops/hip/scan.hip) against torch's cumsum / cummax on the same device
matrices: time per call and effective bandwidth (2 reads + 1 write of the matrix: the chunk-total
pass and the rescan both read X).

    python tools/bench_scan.py [--reps 50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from systemml_amd.ops import kernels as Kn  # noqa: E402


def timed(f, reps, warm=3):
    for _ in range(warm):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    Kn.load(required=True)
    print(f"{'shape':>16s} {'dtype':>8s} {'op':>7s} {'hip ms':>8s} {'GB/s':>7s} {'torch ms':>9s} {'GB/s':>7s}")
    for shape in ((10_000_000, 1), (1_000_000, 8), (1_000_000, 100), (100_000, 1000), (10_000, 10_000)):
        for dt in (torch.float32, torch.float64):
            X = torch.rand(shape, device="cuda", dtype=dt)
            nbytes = X.numel() * X.element_size()
            for op, tf in (("cumsum", lambda: torch.cumsum(X, 0)), ("cummax", lambda: torch.cummax(X, 0).values)):
                th = timed(lambda: Kn.cumagg(op, X), a.reps)
                tt = timed(tf, a.reps) if op == "cumsum" else timed(tf, 1, 0)   # torch cummax over dim 0 is slow
                print(f"{str(shape):>16s} {str(dt)[6:]:>8s} {op:>7s} {th:8.3f} {3 * nbytes / th / 1e6:7.0f} "
                      f"{tt:9.3f} {2 * nbytes / tt / 1e6:7.0f}", flush=True)
            del X


if __name__ == "__main__":
    main()
