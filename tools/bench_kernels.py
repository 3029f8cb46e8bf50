"""Micro-benchmark of the row-streaming kernels (interleaved A/B in one process).

    python tools/bench_kernels.py [--rows 10000000] [--cols 1000] [--reps 5]

Reports per-mode time and effective HBM bandwidth (bytes of X / time) for the
rows-per-iteration variants R=1 / R=2, plus hipBLASLt (torch.matmul) on fp32 X
for the same products as a library baseline.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--cols", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from systemml_amd.ops import kernels as K
    from systemml_amd.ops.backend import backend
    from systemml_amd.conf import DMLConfig
    backend.configure(DMLConfig(precision="single"))
    L = K.load(required=True)
    L.sysml_set_rows_per_iter.argtypes = [ctypes.c_int]
    dev = torch.device("cuda")
    results = {}
    for dt in (torch.bfloat16, torch.float32):
        X = torch.rand((a.rows, a.cols), device=dev, dtype=torch.float32).to(dt)
        nbytes = X.numel() * X.element_size()
        v1 = torch.randn((a.cols, 1), device=dev)
        v4 = torch.randn((a.cols, 4), device=dev)
        g4 = torch.randn((a.rows, 4), device=dev)
        P = torch.softmax(torch.randn((a.rows, 5), device=dev), 1)[:, :4].contiguous()
        cases = {
            "xv_k1": lambda: K.xv(X, v1),
            "xv_k4": lambda: K.xv(X, v4),
            "xtg_k4": lambda: K.xtg(X, g4),
            "XtXv_k1": lambda: K.mmchain("XtXv", X, v1),
            "XtPSXv_k4": lambda: K.mmchain("XtPSXv", X, v4, P),
            "XtXv_k4": lambda: K.mmchain("XtXv", X, v4),
            "rowsumsq": lambda: K.sumsq(X, "row"),
        }
        if dt == torch.float32:
            cases["torch_mv_k1"] = lambda: X @ v1
            cases["torch_xtg_k4"] = lambda: X.t() @ g4
        times = {}
        L.sysml_set_variant.argtypes = [ctypes.c_int]
        for rep in range(a.reps + 1):
            for name, fn in cases.items():
                variants = (0,) if name.startswith("torch") else (0, 2, 3, 4, 99) if dt == torch.bfloat16 \
                    else (0, 1, 2, 11)
                for R in variants:
                    # R = prefetch depth (pk kernel) / rows per iteration (generic); 11 = generic
                    # kernel; 99 = MFMA chain kernel (bf16 only)
                    # R = 0: the default dispatch (MFMA where it wins, tuned prefetch depth)
                    K.MFMA = R in (0, 99)
                    K.MFMA_ALL = R == 99
                    L.sysml_set_variant(1 if 10 < R < 99 else 0)
                    L.sysml_set_rows_per_iter(R % 10 if R < 99 else 0)
                    torch.cuda.synchronize()
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    fn()
                    e1.record()
                    torch.cuda.synchronize()
                    if rep > 0:
                        times.setdefault(f"{name}/R{R}", []).append(e0.elapsed_time(e1))
        L.sysml_set_rows_per_iter(0)
        K.MFMA, K.MFMA_ALL = True, False
        for k, ts in times.items():
            med = statistics.median(ts)
            results[f"{str(dt).split('.')[-1]}/{k}"] = {"ms": round(med, 3), "min_ms": round(min(ts), 3),
                                                         "GBps": round(nbytes / med / 1e6, 1)}
        del X
        torch.cuda.empty_cache()
    for k, v in results.items():
        print(f"{k:32s} {v['ms']:8.3f} ms  {v['GBps']:8.1f} GB/s")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
