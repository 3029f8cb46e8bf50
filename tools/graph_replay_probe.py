"""Host and device cost of a HIP-graph replay vs the same launches issued one by one.

    python tools/graph_replay_probe.py [--nodes 12] [--reps 500]

A run-ahead loop iteration replayed as a graph (runtime/graphloop.py) only pays off when one
hipGraphLaunch costs the host less than the iteration's launches did; this measures both."""
import argparse
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=12)
    ap.add_argument("--reps", type=int, default=500)
    a = ap.parse_args()
    x = torch.rand(1000, 5, device="cuda")
    y = torch.rand(1000, 5, device="cuda")

    def body():
        z = x
        for _ in range(a.nodes):
            z = z * 1.0001 + y
        y.copy_(z * 0.5)

    for _ in range(3):
        body()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.reps):
        body()
    th = time.perf_counter() - t
    torch.cuda.synchronize()
    te = time.perf_counter() - t
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        g.capture_begin()
        body()
        g.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.reps):
        g.replay()
    gh = time.perf_counter() - t
    torch.cuda.synchronize()
    ge = time.perf_counter() - t
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(a.reps):
        g.replay()
    ev1.record()
    torch.cuda.synchronize()
    gd = ev0.elapsed_time(ev1) / a.reps
    n = 2 * a.nodes + 2
    print(f"{n} kernels per iteration: eager host {th / a.reps * 1e6:.1f} us/iter (end-to-end {te / a.reps * 1e6:.1f}); "
          f"graph host {gh / a.reps * 1e6:.1f} us/replay (end-to-end {ge / a.reps * 1e6:.1f}, device {gd * 1e3:.1f})")


if __name__ == "__main__":
    main()
