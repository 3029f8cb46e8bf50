"""Convolution kernels on every ResNet-50 conv shape at batch N (default 256), bf16 operands:
forward / backward-data / backward-filter of ops/hip/dnn.hip (bf16 activation outputs, as the
ResNet-50 bench runs them) per shape and the network total weighted by how often each shape
occurs in one training step, against MIOpen (torch.nn.functional.conv2d and its grads).

    python tools/bench_conv_rn50.py [--batch 256] [--reps 5] [--no-miopen]
Prints one JSON line per shape and a total line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def rn50_shapes():
    """(C, H, F, k, stride, pad) -> occurrences of every conv of ResNet-50 (torchvision layout)."""
    occ = {}

    def add(*s):
        occ[s] = occ.get(s, 0) + 1
    add(3, 224, 64, 7, 2, 3)
    cin, h = 64, 56
    for si, (w, nb) in enumerate(((64, 3), (128, 4), (256, 6), (512, 3))):
        for b in range(nb):
            s = 2 if (b == 0 and si > 0) else 1
            add(cin, h, w, 1, 1, 0)
            add(w, h, w, 3, s, 1)
            ho = (h + 2 - 3) // s + 1
            add(w, ho, 4 * w, 1, 1, 0)
            if b == 0:
                add(cin, h, 4 * w, 1, s, 0)
            cin, h = 4 * w, ho
    return occ


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-miopen", action="store_true")
    a = ap.parse_args()
    from systemml_amd.ops import kernels as K
    from systemml_amd.ops.backend import backend
    backend.act_bf16_min_cells = 1 << 22
    dev = torch.device("cuda:0")
    N = a.batch
    tot = {"flop": 0.0, "ours_ms": 0.0, "miopen_ms": 0.0}
    for (C, H, Fo, k, s, p), n in sorted(rn50_shapes().items()):
        X = torch.randn(N, C * H * H, device=dev, dtype=torch.bfloat16)
        W = torch.randn(Fo, C * k * k, device=dev, dtype=torch.float32) * 0.05
        Ho = (H + 2 * p - k) // s + 1
        G = torch.randn(N, Fo * Ho * Ho, device=dev, dtype=torch.bfloat16)
        flop = 2.0 * N * Fo * Ho * Ho * C * k * k
        r = {"C": C, "H": H, "F": Fo, "k": k, "s": s, "count": n}
        fns = {"fwd": lambda: K.conv2d(0, X, W, None, N, C, H, H, Fo, k, k, s, s, p, p),
               "bwd_filter": lambda: K.conv2d(2, X, None, G, N, C, H, H, Fo, k, k, s, s, p, p)}
        if C > 3:            # the stem's input gradient is not needed for training
            fns["bwd_data"] = lambda: K.conv2d(1, None, W, G, N, C, H, H, Fo, k, k, s, s, p, p)
        if not a.no_miopen:
            Wb = W.to(torch.bfloat16)
            fns["miopen_fwd"] = lambda: F.conv2d(X.view(N, C, H, H), Wb.view(Fo, C, k, k), stride=s, padding=p)
            fns["miopen_bwd_filter"] = lambda: torch.nn.grad.conv2d_weight(
                X.view(N, C, H, H), (Fo, C, k, k), G.view(N, Fo, Ho, Ho), stride=s, padding=p)
            if C > 3:
                fns["miopen_bwd_data"] = lambda: torch.nn.grad.conv2d_input(
                    (N, C, H, H), Wb.view(Fo, C, k, k), G.view(N, Fo, Ho, Ho), stride=s, padding=p)
        if k == 1 and s == 1:     # 1x1 stride-1: a batched GEMM per image (hipBLASLt via torch.matmul)
            Wb2 = W.to(torch.bfloat16)
            fns["blas_fwd"] = lambda: torch.matmul(Wb2, X.view(N, C, H * H))
            fns["blas_bwd_data"] = lambda: torch.matmul(Wb2.t(), G.view(N, Fo, H * H))
        for name, fn in fns.items():
            ms = timeit(fn, a.reps)
            r[name + "_ms"] = round(ms, 3)
            r[name + "_TF"] = round(flop / ms / 1e9, 1)
            if name.startswith("blas"):
                continue
            key = "miopen_ms" if name.startswith("miopen") else "ours_ms"
            tot[key] += ms * n
            if not name.startswith("miopen"):
                tot["flop"] += flop * n
        print(json.dumps(r), flush=True)
        del X, W, G
    out = {"batch": N, "step_conv_tflop": round(tot["flop"] / 1e12, 2), "ours_ms": round(tot["ours_ms"], 2),
           "ours_TF": round(tot["flop"] / tot["ours_ms"] / 1e9, 1)}
    if not a.no_miopen:
        out["miopen_ms"] = round(tot["miopen_ms"], 2)
        out["miopen_TF"] = round(tot["flop"] / max(tot["miopen_ms"], 1e-9) / 1e9, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
