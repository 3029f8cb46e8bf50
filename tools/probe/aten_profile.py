"""Which framework call sites launch ATen (torch) GPU kernels, weighted by device time: runs
bench.main() (or bench_resnet50.main() with `--target bench_resnet50`) under torch.profiler
with Python stacks and prints, per ATen operator and innermost systemml_amd frames, the call
count and the device time of the kernels it launched.

    python tools/probe/aten_profile.py [--target bench] [--top 40] [bench args]
"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def main():
    args = sys.argv[1:]
    target, top = "bench", 40
    while args[:1] and args[0] in ("--target", "--top"):
        if args[0] == "--target":
            target = args[1]
        else:
            top = int(args[1])
        args = args[2:]
    mod = __import__(target)
    sys.argv = [target + ".py"] + args
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        mod.main()
    rows = []
    for e in prof.key_averages(group_by_stack_n=12):
        if not e.key.startswith("aten::"):
            continue
        dev = getattr(e, "self_device_time_total", None)
        if dev is None:
            dev = getattr(e, "self_cuda_time_total", 0.0)
        if not dev:
            continue
        st = [f for f in (e.stack or []) if "systemml_amd" in f or "bench" in f]
        rows.append((dev, e.count, e.key, [f.split("/")[-1] for f in st[:4]]))
    rows.sort(key=lambda r: -r[0])
    tot = sum(r[0] for r in rows)
    print(f"ATen self device time {tot / 1e3:.1f} ms", file=sys.stderr)
    for dev, n, k, st in rows[:top]:
        print(f"{dev / 1e3:9.2f} ms {n:6d}  {k}  {' < '.join(st)}", file=sys.stderr)


if __name__ == "__main__":
    main()
