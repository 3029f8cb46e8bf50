"""Per-channel broadcast operators of the DNN path: the bias_add / bias_multiply kernel
(ops/hip/dnn.hip bias_op / bias_op_v4), a generated CHAN cell kernel (the fused batch-norm
form (X bias+ m) bias* g, ops/cell.py) and torch's broadcast ops, on ResNet activation shapes.

    python tools/bench_bias.py [--reps 50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from systemml_amd.conf import DMLConfig  # noqa: E402
from systemml_amd.ops import cell, kernels as Kn  # noqa: E402
from systemml_amd.ops.backend import backend  # noqa: E402
from systemml_amd.ops.cell import CellProgram  # noqa: E402


def timed(f, reps):
    for _ in range(3):
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
    backend.configure(DMLConfig(gpu=True, precision="single", gpu_min_cells=0))
    Kn.load(required=True)
    prog = CellProgram([("b", "bias+", 3, 0, 1), ("b", "bias*", 3, 3, 2)], 3, 3)
    print(f"{'N x C x HW':>18s} {'bias_op ms':>10s} {'TB/s':>6s} {'cell2 ms':>9s} {'TB/s':>6s} {'torch2 ms':>9s}")
    for N, C, HW in ((64, 64, 112 * 112), (64, 256, 56 * 56), (64, 512, 28 * 28), (64, 1024, 14 * 14),
                     (64, 2048, 7 * 7)):
        X = torch.randn((N, C * HW), device="cuda")
        m = torch.randn((C, 1), device="cuda")
        g = torch.randn((C, 1), device="cuda")
        nb = X.numel() * 4 * 2
        t1 = timed(lambda: Kn.bias_op(X, m), a.reps)
        assert cell._kernel(prog, [X, m, g]) is not None
        t2 = timed(lambda: cell._kernel(prog, [X, m, g]), a.reps)
        x3 = X.view(N, C, HW)
        t3 = timed(lambda: (x3 + m.view(1, C, 1)) * g.view(1, C, 1), a.reps)
        print(f"{f'{N}x{C}x{HW}':>18s} {t1:10.3f} {nb / t1 / 1e9:6.2f} {t2:9.3f} {nb / t2 / 1e9:6.2f} {t3:9.3f}",
              flush=True)
        del X
    # column aggregate of a per-channel cell program (batch-norm variance: colSums((X bias+ m)^2))
    cprog = CellProgram([("b", "bias+", 2, 0, 1), ("b", "*", 2, 2, 2)], 2, 2, ("sum", "col"))
    for N, C, HW in ((256, 64, 56 * 56), (256, 256, 14 * 14), (64, 64, 112 * 112)):
        X = torch.randn((N, C * HW), device="cuda")
        m = torch.randn((C, 1), device="cuda")
        assert cell._kernel(cprog, [X, m]) is not None
        tc = timed(lambda: cell._kernel(cprog, [X, m]), a.reps)
        x3 = X.view(N, C, HW)
        tt = timed(lambda: ((x3 + m.view(1, C, 1)) ** 2).sum(0), a.reps)
        print(f"colagg {N}x{C}x{HW}: cell {tc:.3f} ms ({X.numel() * 4 / tc / 1e9:.2f} TB/s), torch {tt:.3f} ms",
              flush=True)
        del X
    # the ResNet stem's 3x3 / stride-2 max pooling and its backward pass (argmax positions + gather)
    for N in (64, 256):
        C, H, Wd = 64, 112, 112
        X = torch.randn((N, C * H * Wd), device="cuda")
        Ho = (H + 2 - 3) // 2 + 1
        G = torch.randn((N, C * Ho * Ho), device="cuda")
        tf = timed(lambda: Kn.pool2d(False, False, X, None, N, C, H, Wd, 3, 3, 2, 2, 1, 1), a.reps)
        tb = timed(lambda: Kn.pool2d(True, False, X, G, N, C, H, Wd, 3, 3, 2, 2, 1, 1), a.reps)
        print(f"max_pool {N}x{C}x{H}x{Wd} k3 s2: fwd {tf:.3f} ms ({(X.numel() + G.numel()) * 4 / tf / 1e9:.2f} TB/s), "
              f"bwd {tb:.3f} ms ({(2 * X.numel() + G.numel()) * 4 / tb / 1e9:.2f} TB/s)", flush=True)
        del X, G


if __name__ == "__main__":
    main()
