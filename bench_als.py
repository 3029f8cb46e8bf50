#!/usr/bin/env python
"""ALS-CG benchmark (BASELINE.json config #4: ALS-CG on a sparse ratings matrix; the
reference names 10M x 10M at 0.01 density over 8 GPUs -- this driver runs the same script at a
size chosen on the command line, default 1M x 1M with 100 ratings per row = 100M non-zeros on
one GPU).

    python bench_als.py [--rows R] [--cols C] [--per-row K] [--rank 10] [--maxi 5] [--steps 2]

The ratings matrix is generated directly in HBM as canonical CSR (K distinct random columns
per row, values 1..5), then scripts/algorithms/ALS-CG.dml (L2 regularisation, rank r, maxi
outer iterations, loss check on) runs end to end: the weighted quaternary operators run as
sampled products at the non-zeros (SDDMM kernel), the products with the ratings matrix as CSR
SpMM.  One step = compile + execute of the script; the time of K steps after W warmup steps
is reported as seconds per run.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402


def ratings(rows, cols, per_row, seed=5):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    # distinct sorted columns per row: sorted draws from [0, cols - per_row] plus their rank
    # (canonical CSR: no duplicate cells)
    u = torch.randint(0, cols - per_row + 1, (rows, per_row), generator=g, device=dev).sort(dim=1).values
    colidx = u + torch.arange(per_row, device=dev)
    vals = torch.randint(1, 6, (rows * per_row,), generator=g, device=dev).to(torch.float32)
    crow = torch.arange(0, rows * per_row + 1, per_row, device=dev, dtype=torch.int64)
    return torch.sparse_csr_tensor(crow, colidx.reshape(-1), vals, (rows, cols), device=dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--cols", type=int, default=1_000_000)
    ap.add_argument("--per-row", type=int, default=100)
    ap.add_argument("--rank", type=int, default=10)
    ap.add_argument("--maxi", type=int, default=5)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    if not torch.cuda.is_available():
        raise SystemExit("bench_als.py needs a GPU")
    from systemml_amd.api import executor as EX
    from systemml_amd.api.mlcontext import SCRIPTS_DIR
    from systemml_amd.conf import DMLConfig
    from systemml_amd.ops import kernels
    cfg = DMLConfig(precision="single")
    X = ratings(a.rows, a.cols, a.per_row)
    torch.cuda.synchronize()
    with open(os.path.join(SCRIPTS_DIR, "algorithms", "ALS-CG.dml")) as f:
        src = f.read()
    args = dict(X="X", U="U", V="V", rank=a.rank, reg="L2", **{"lambda": 0.000001}, maxi=a.maxi, check="TRUE",
                thr=0.0001, fmt="csv")
    log = []

    def step():
        cs = EX.compile_script(src, args, inputs={"X": X}, outputs=["U", "V"], config=cfg)
        r, _ = EX.execute(cs, {"X": X}, out=log.append)
        return r

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        r = step()
    torch.cuda.synchronize()
    sec = (time.perf_counter() - t0) / a.steps
    U, V = r["U"], r["V"]
    print(json.dumps({
        "metric": "ALS-CG seconds per run (sparse ratings, rank %d, maxi %d)" % (a.rank, a.maxi),
        "value": round(sec, 4), "unit": "s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "higher_is_better": False, "dtype": "fp32", "data": "synthetic CSR ratings generated in HBM",
        "config": {"rows": a.rows, "cols": a.cols, "nnz": a.rows * a.per_row, "rank": a.rank,
                   "U": list(U.shape), "V": list(V.shape)},
        "kernels": {k: v for k, v in kernels.counters.items() if v},
        "last_loss_lines": [s for s in log if "loss" in s.lower()][-2:],
    }), flush=True)


if __name__ == "__main__":
    main()
