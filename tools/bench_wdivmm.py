"""The fused wdivmm kernel (ops/hip/sddmm.hip) alone on ALS-shaped input: an m x n CSR pattern
with `per-row` sorted random columns, rank-K factors, mode 1 (w * (<u, v> - x)) right form, and
the sampled product (sddmm) over the same pattern for comparison.  Prints ms per call and
non-zeros per second; SYSML_WD_WAVES / SYSML_WD_UNROLL select the launch shape (read once per
process, so sweep them over processes).

    python tools/bench_wdivmm.py [--rows 10000000] [--cols 10000000] [--per-row 100] [--rank 10]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--cols", type=int, default=10_000_000)
    ap.add_argument("--per-row", type=int, default=100)
    ap.add_argument("--rank", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from bench_als import ratings
    from systemml_amd.ops import kernels
    kernels.load(required=True)
    X = ratings(a.rows, a.cols, a.per_row)
    g = torch.Generator(device="cuda").manual_seed(1)
    U = torch.rand(a.rows, a.rank, generator=g, device="cuda")
    V = torch.rand(a.cols, a.rank, generator=g, device="cuda")
    crow, col, xv = X.crow_indices(), kernels.idx32_of(X.col_indices()), X.values()
    wv = (xv != 0).float()
    nnz = col.numel()
    res = {}
    for name, fn in (("wdivmm", lambda: kernels.wdivmm(crow, col, wv, xv, U, V, 1)),
                     ("sddmm", lambda: kernels.sddmm(crow, col, U, V))):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / a.reps
    ref = None
    if a.rows * a.per_row <= 20_000_000:
        uv = (U[X.to_sparse_coo().indices()[0]] * V[X.col_indices()]).sum(1)
        q = wv * (uv - xv)
        ref = torch.sparse_csr_tensor(crow, X.col_indices(), q, X.shape) @ V
        err = (kernels.wdivmm(crow, col, wv, xv, U, V, 1) - ref).abs().max().item()
    print(f"m={a.rows} n={a.cols} nnz={nnz} K={a.rank} waves={os.environ.get('SYSML_WD_WAVES', '32')} "
          f"unroll={os.environ.get('SYSML_WD_UNROLL', '4')}: wdivmm {res['wdivmm']:.2f} ms "
          f"({nnz / res['wdivmm'] / 1e6:.1f} Gnnz/s), sddmm {res['sddmm']:.2f} ms"
          + (f", max err {err:.2e}" if ref is not None else ""), flush=True)


if __name__ == "__main__":
    main()
