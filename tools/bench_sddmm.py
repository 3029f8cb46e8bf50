"""SDDMM (ops/hip/sddmm.hip) vs. the torch gather formulation on an ALS-shaped sampled product:
m=n=1M, nnz=50M (0.005%), rank r in {16, 64}, fp32 and fp64.  Prints one JSON line per rank."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from systemml_amd.ops import kernels


def main():
    dev = torch.device("cuda:0")
    m = n = 1_000_000
    nnz = 50_000_000
    g = torch.Generator(device=dev).manual_seed(0)
    row = torch.sort(torch.randint(0, m, (nnz,), device=dev, generator=g)).values
    col = torch.randint(0, n, (nnz,), device=dev, generator=g)
    crow = torch.searchsorted(row, torch.arange(m + 1, device=dev))
    for r, dt in ((16, torch.float32), (64, torch.float32), (16, torch.float64), (64, torch.float64)):
        U = torch.randn(m, r, device=dev, generator=g, dtype=dt)
        V = torch.randn(n, r, device=dev, generator=g, dtype=dt)
        res = {}
        for name, fn in (("hip", lambda: kernels.sddmm(crow, col, U, V, dt)),
                         ("torch_gather", lambda: (U.index_select(0, row) * V.index_select(0, col)).sum(1))):
            out = fn()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(10):
                out = fn()
            torch.cuda.synchronize()
            res[name] = (time.perf_counter() - t) / 10 * 1e3
            res[name + "_out"] = out
        err = float((res["hip_out"] - res["torch_gather_out"]).abs().max())
        es = U.element_size()
        gbytes = nnz * (r * es + 8 + es) / 1e9        # V row gather + col index + output
        print(json.dumps({"r": r, "dtype": str(dt), "nnz": nnz, "hip_ms": round(res["hip"], 3),
                          "torch_gather_ms": round(res["torch_gather"], 3),
                          "hip_effective_TBps": round(gbytes / res["hip"], 2), "max_abs_diff": err}), flush=True)


if __name__ == "__main__":
    main()
