"""Idle / busy time of a rocprofv3 kernel trace split into solver inner-loop windows (between
consecutive chain4m<2,5,1> Hessian-vector passes less than 1.5 ms apart) and everything else,
over the final W ms of the trace, with the kernels that follow the largest gaps.

    python tools/trace_regions.py run_kernel_trace.csv [W_ms]
"""
import csv, sys
rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
# last 3 steps: use the final 200 ms window
t_end = rows[-1][1]
w = float(sys.argv[2]) * 1e6 if len(sys.argv) > 2 else 200e6
rows = [r for r in rows if r[0] >= t_end - w]
inner = lambda n: "chain4m_kernel<2, 5, 1>" in n
# mark inner windows: between consecutive inner kernels less than 1.5 ms apart
idx = [i for i, r in enumerate(rows) if inner(r[2])]
inwin = [False] * len(rows)
for a, b in zip(idx, idx[1:]):
    if rows[b][0] - rows[a][1] < 1.5e6:
        for i in range(a, b + 1):
            inwin[i] = True
gi = go = bi = bo = 0
for i in range(1, len(rows)):
    g = max(0, rows[i][0] - max(r[1] for r in rows[max(0,i-3):i]))
    if inwin[i] and inwin[i-1]:
        gi += g
    else:
        go += g
for i, r in enumerate(rows):
    if inwin[i]: bi += r[1] - r[0]
    else: bo += r[1] - r[0]
print(f"window {w/1e6:.0f} ms: inner-loop busy {bi/1e6:.1f} idle {gi/1e6:.1f}; outside busy {bo/1e6:.1f} idle {go/1e6:.1f} ms; inner kernels {len(idx)}")
from collections import defaultdict
agg = defaultdict(lambda: [0, 0])
for i in range(1, len(rows)):
    if not (inwin[i] and inwin[i-1]):
        continue
    g = max(0, rows[i][0] - max(r[1] for r in rows[max(0,i-3):i]))
    k = rows[i][2][:70]
    agg[k][0] += g; agg[k][1] += 1
for k, (g, n) in sorted(agg.items(), key=lambda x: -x[1][0])[:12]:
    print(f"  inner idle {g/1e6:6.2f} ms before {n:4d} x {k}")
bus = defaultdict(lambda: [0, 0])
for i, r in enumerate(rows):
    if inwin[i]:
        bus[r[2][:70]][0] += r[1] - r[0]; bus[r[2][:70]][1] += 1
for k, (g, n) in sorted(bus.items(), key=lambda x: -x[1][0])[:12]:
    print(f"  inner busy {g/1e6:6.2f} ms  {n:4d} x {k}")
out = defaultdict(lambda: [0, 0])
for i in range(1, len(rows)):
    if inwin[i] and inwin[i-1]:
        continue
    g = max(0, rows[i][0] - max(r[1] for r in rows[max(0,i-3):i]))
    k = rows[i][2][:70]
    out[k][0] += g; out[k][1] += 1
for k, (g, n) in sorted(out.items(), key=lambda x: -x[1][0])[:15]:
    print(f"  outer idle {g/1e6:6.2f} ms before {n:4d} x {k}")
