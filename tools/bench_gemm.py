"""Microbenchmark of the hand-written MFMA GEMM / tsmm (ops/hip/gemm.hip) vs torch (hipBLASLt).

    python tools/bench_gemm.py [--out profiles/gemm_kbench.json]

Random uniform [-1, 1) operands (cdna_hip_programming.md §5.4 rule 25: never zero-filled).
Interleaves ours / torch per shape in one process and reports the median of the rounds.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, iters, rounds=5):
    res = []
    for _ in range(rounds):
        fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / iters)
    res.sort()
    return res[len(res) // 2], res[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    from systemml_amd.ops import gemm
    dev = torch.device("cuda")
    rows = []

    def rnd(shape, dt):
        return (torch.rand(shape, device=dev) * 2 - 1).to(dt)

    cases = [("bf16", 8192, 8192, 8192, "nn"), ("bf16", 4096, 4096, 4096, "nn"), ("bf16", 8192, 8192, 8192, "tn"),
             ("bf16", 8192, 8192, 8192, "nt"), ("fp32", 4096, 4096, 4096, "nn"), ("fp64", 4096, 4096, 4096, "nn"),
             ("bf16", 1000, 10_000_000 // 10, 1000, "tn")]
    if a.quick:
        cases = cases[:2]
    for dts, M, K, N, lay in cases:
        dt = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp64": torch.float64}[dts]
        A = rnd((K, M) if lay[0] == "t" else (M, K), dt)
        B = rnd((N, K) if lay[1] == "t" else (K, N), dt)
        P = A.t() if lay[0] == "t" else A
        Q = B.t() if lay[1] == "t" else B
        flop = 2.0 * M * N * K
        it = max(1, int(2e12 / flop * (1 if dt == torch.bfloat16 else 0.1)))
        res = {}
        ref0 = (P.float() @ Q.float())
        for bk in ((0, 32, 64, "64nopf") if dt == torch.bfloat16 else (0,)):
            gemm.set_bk(64 if bk == "64nopf" else bk)
            gemm.set_pf(bk != "64nopf")
            out = gemm.matmul(P, Q)
            err = float((out.float() - ref0).abs().max()) / max(1.0, float(ref0.abs().max()))
            assert err < 1e-2, (bk, err)
            res[bk] = timeit(lambda: gemm.matmul(P, Q), it)
        gemm.set_bk(0)
        gemm.set_pf(True)
        del ref0
        ref = timeit(lambda: P @ Q, it)
        rows.append({"case": f"{dts} {lay} M={M} N={N} K={K}", "ours_ms": res[0][0], "torch_ms": ref[0],
                     "ours_tflops": flop / res[0][0] / 1e9, "torch_tflops": flop / ref[0] / 1e9})
        for bk in (32, 64, "64nopf"):
            if bk in res:
                rows[-1][f"bk{bk}_tflops"] = flop / res[bk][0] / 1e9
        print(json.dumps(rows[-1]), flush=True)
        del A, B, P, Q
    # tsmm on the headline matrix: 10M x 1000 bf16 (20 GB)
    if not a.quick:
        n, d = 10_000_000, 1000
        X = torch.empty((n, d), dtype=torch.bfloat16, device=dev)
        for s in range(0, n, 1 << 20):
            X[s:s + (1 << 20)] = rnd((min(1 << 20, n - s), d), torch.bfloat16)
        flop_tri = 2.0 * d * d * n / 2
        ours = timeit(lambda: gemm.tsmm(X, True), 3, 3)
        hbm_ms = X.numel() * 2 / 6.3e12 * 1e3
        ref = timeit(lambda: X[: n // 10].t() @ X[: n // 10], 3, 3)
        rows.append({"case": "tsmm bf16 t(X)%*%X 10Mx1000", "ours_ms": ours[0], "ours_tflops_tri": flop_tri / ours[0] / 1e9,
                     "one_pass_hbm_ms_at_6.3TBs": hbm_ms, "torch_ms_extrapolated_x10": ref[0] * 10})
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
