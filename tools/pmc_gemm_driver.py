"""Driver for PMC counter passes over the hand-written GEMM kernels (tools/gpu/pmc_gemm.sh): the
bf16 nt 8192^3 product and tsmm of a 10M x 1000 bf16 matrix on gemm.hip, a few launches each.

    python tools/pmc_gemm_driver.py [--reps 3] [--skip-tsmm]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--skip-tsmm", action="store_true")
    a = ap.parse_args()
    from systemml_amd.ops import gemm
    dev = torch.device("cuda")
    A = (torch.rand((8192, 8192), device=dev) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand((8192, 8192), device=dev) * 2 - 1).to(torch.bfloat16)
    for _ in range(a.reps):
        gemm.matmul(A, B.t())
    torch.cuda.synchronize()
    del A, B
    if not a.skip_tsmm:
        n, d = 10_000_000, 1000
        X = torch.empty((n, d), dtype=torch.bfloat16, device=dev)
        for s in range(0, n, 1 << 20):
            X[s:s + (1 << 20)] = (torch.rand((min(1 << 20, n - s), d), device=dev) * 2 - 1).to(torch.bfloat16)
        for _ in range(a.reps):
            gemm.tsmm(X, True)
        torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
