"""GPU idle-gap analysis of a rocprofv3 kernel trace (`--kernel-trace --output-format csv`).

    python tools/trace_gaps.py <run_kernel_trace.csv> [--from-kernel SUBSTR] [--top 15]

Reports busy time, idle time and the largest idle gaps (with the kernels on either side),
starting at the first dispatch whose name contains --from-kernel (e.g. skip datagen).
Idle time between kernels is host-side time: interpreter work, launches and syncs.
"""
import argparse
import csv
import re
from collections import defaultdict


def short(n):
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"^void ", "", n)
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--from-kernel", default="")
    ap.add_argument("--skip", type=int, default=0, help="skip this many matches of --from-kernel first")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    start = 0
    if a.from_kernel:
        hits = [i for i, r in enumerate(rows) if a.from_kernel in r["Kernel_Name"]]
        start = hits[min(a.skip, len(hits) - 1)]
    rows = rows[start:]
    t0 = int(rows[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in rows)
    busy = 0
    gaps = []
    end = t0
    by_prev = defaultdict(float)
    for i, r in enumerate(rows):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > end:
            g = s - end
            prev = rows[i - 1]["Kernel_Name"] if i else ""
            gaps.append((g, short(prev), short(r["Kernel_Name"])))
            by_prev[short(r["Kernel_Name"])] += g
        busy += max(0, e - max(s, end)) if e > end else 0
        end = max(end, e)
    span = t1 - t0
    idle = sum(g for g, _, _ in gaps)
    print(f"kernels {len(rows)}  span {span / 1e6:.1f} ms  busy {busy / 1e6:.1f} ms  idle {idle / 1e6:.1f} ms "
          f"({100 * idle / span:.1f}%)")
    small = sum(g for g, _, _ in gaps if g < 20_000)
    print(f"  idle in gaps < 20 us: {small / 1e6:.1f} ms over {sum(1 for g, _, _ in gaps if g < 20_000)} gaps")
    print("largest gaps:")
    for g, p, n in sorted(gaps, reverse=True)[:a.top]:
        print(f"  {g / 1e3:9.1f} us  after {p}  before {n}")
    print("idle before kernel (total):")
    for k, v in sorted(by_prev.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"  {v / 1e6:8.2f} ms  {k}")


if __name__ == "__main__":
    main()
