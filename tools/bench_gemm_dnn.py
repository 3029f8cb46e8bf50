"""Image-blocked DNN GEMM (gemm.hip sysml_gemm_dnn via kernels._gemm_img) against the batched
library GEMM (torch.matmul -> hipBLASLt) on the ResNet-50 convolution GEMM shapes at batch 256:
1x1 convolutions forward (W . X[n]) and backward data (t(W) . dY[n]), the small-image im2col
forward GEMMs and the col2im backward-data GEMMs.  Prints one line per shape (ms, TFLOP/s, the
library time and the ratio) and the totals.

    python tools/bench_gemm_dnn.py [--batch 256] [--iters 20] [--only 1x1|im2col|col2im]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

# (kind, M, K, hw): out[n] (M x hw) = A (M x K) . B[n] (K x hw)
SHAPES = [
    ("1x1", 64, 64, 3136), ("1x1", 256, 64, 3136), ("1x1", 64, 256, 3136), ("1x1", 128, 256, 3136),
    ("1x1", 512, 128, 784), ("1x1", 128, 512, 784), ("1x1", 256, 512, 784),
    ("1x1", 1024, 256, 196), ("1x1", 256, 1024, 196), ("1x1", 512, 1024, 196),
    ("1x1", 2048, 512, 49), ("1x1", 512, 2048, 49),
    # backward data of the same convolutions: M and K swapped
    ("1x1T", 64, 256, 3136), ("1x1T", 256, 64, 3136), ("1x1T", 256, 128, 3136),
    ("1x1T", 128, 512, 784), ("1x1T", 512, 128, 784), ("1x1T", 512, 256, 784),
    ("1x1T", 256, 1024, 196), ("1x1T", 1024, 256, 196), ("1x1T", 1024, 512, 196),
    ("1x1T", 512, 2048, 49), ("1x1T", 2048, 512, 49),
    # im2col forward: 3 x 3 convolutions on small images (K = 9 C)
    ("im2col", 256, 2304, 196), ("im2col", 512, 4608, 49), ("im2col", 256, 1152, 196), ("im2col", 512, 2304, 49),
    # col2im backward data: cols (9 C x P) = t(W) (9 C x F) . dY (F x P)
    ("col2im", 2304, 256, 196), ("col2im", 4608, 512, 49), ("col2im", 1152, 256, 196), ("col2im", 576, 128, 784),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    from systemml_amd.ops import kernels as K
    K.load(required=True)
    n = a.batch
    tot_k = tot_l = 0.0
    print(f"{'kind':7s} {'M':>5s} {'K':>5s} {'hw':>5s}  {'sysml ms':>9s} {'TF/s':>6s}  {'lib ms':>8s} {'TF/s':>6s}  ratio")
    for kind, M, Kd, hw in SHAPES:
        if a.only and not kind.startswith(a.only):
            continue
        A = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
        B = torch.randn(n, Kd, hw, device="cuda").to(torch.bfloat16)
        out = torch.empty(n, M, hw, dtype=torch.bfloat16, device="cuda")
        t_k = timeit(lambda: K._gemm_img(A, B, out, M, Kd, n, hw), a.iters)
        t_l = timeit(lambda: torch.matmul(A, B), a.iters)
        fl = 2.0 * M * Kd * hw * n
        tot_k += t_k
        tot_l += t_l
        print(f"{kind:7s} {M:5d} {Kd:5d} {hw:5d}  {t_k:9.3f} {fl / t_k / 1e9:6.0f}  {t_l:8.3f} {fl / t_l / 1e9:6.0f}  "
              f"{t_l / t_k:5.2f}", flush=True)
        del A, B, out
    print(f"total sysml {tot_k:.2f} ms, library {tot_l:.2f} ms, ratio {tot_l / tot_k:.2f}")


if __name__ == "__main__":
    main()
