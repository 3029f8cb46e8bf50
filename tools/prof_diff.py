"""Difference two rocprofv3 --stats kernel tables: (B - A) / n per kernel name.

    python tools/prof_diff.py DIR_A DIR_B n
Used by tools/gpu/prof_step.sh to isolate the kernels of n timed bench steps.
"""
import csv
import glob
import os
import sys


def load(d):
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True))
    if not f:
        raise SystemExit(f"no kernel_stats.csv under {d}")
    out = {}
    with open(f[0]) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Name") or row.get("KernelName")
            out[name] = (int(row["Calls"]), float(row["TotalDurationNs"]))
    return out


def main():
    a, b, n = load(sys.argv[1]), load(sys.argv[2]), float(sys.argv[3])
    rows = []
    for k in set(a) | set(b):
        ca, ta = a.get(k, (0, 0.0))
        cb, tb = b.get(k, (0, 0.0))
        rows.append(((tb - ta) / n / 1e6, (cb - ca) / n, k))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    own = sum(r[0] for r in rows if "sysml" in r[2])
    print(f"per-step kernel time {tot:.1f} ms; sysml kernels {own:.1f} ms; other {tot - own:.1f} ms")
    for ms, calls, k in rows:
        if abs(ms) < 0.05:
            continue
        print(f"{ms:9.2f} ms  calls/step={calls:7.1f}  {k[:150]}")


if __name__ == "__main__":
    main()
