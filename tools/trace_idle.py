"""GPU idle-gap analysis of a rocprofv3 kernel trace: over the last `span` seconds of the
trace, sum the gaps between consecutive kernels and attribute each gap to the kernel that
follows it (what the host was launching when the GPU ran dry).

    python tools/trace_idle.py run_kernel_trace.csv [span_s]
"""
import collections
import csv
import sys


def main():
    rows = []
    with open(sys.argv[1]) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:90]))
    rows.sort()
    span = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    t_end = rows[-1][1]
    t0 = t_end - int(span * 1e9)
    busy = 0
    gaps = collections.Counter()
    ngap = collections.Counter()
    hist = collections.Counter()
    last_end = None
    for s, e, k in rows:
        if e < t0:
            continue
        s = max(s, t0)
        if last_end is not None and s > last_end:
            g = s - last_end
            gaps[k] += g
            ngap[k] += 1
            hist[min(6, len(str(g // 1000)))] += g
        busy += e - s if last_end is None or s >= last_end else max(0, e - last_end)
        last_end = max(last_end or 0, e)
    tot = t_end - t0
    print(f"window {tot / 1e6:.1f} ms: busy {busy / 1e6:.1f} ms, idle {(tot - busy) / 1e6:.1f} ms")
    print("idle by gap size (digits of us):", {k: round(v / 1e6, 1) for k, v in sorted(hist.items())})
    for k, g in gaps.most_common(15):
        print(f"{g / 1e6:8.2f} ms idle before {ngap[k]:5d} x {k}")


if __name__ == "__main__":
    main()
