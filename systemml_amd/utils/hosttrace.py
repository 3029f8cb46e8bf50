"""Host-side event timestamps for the latency between a device synchronisation and the next
kernel launch (SYSML_HOSTTRACE=1).  `mark(name)` appends (name, ns) when enabled and is a
single global test otherwise; `summary()` averages the time between consecutive marks by
(previous, next) pair -- e.g. vprog-sync -> block-start -> chain-launch of a solver loop."""
import collections
import os
import time

ON = os.environ.get("SYSML_HOSTTRACE", "0") == "1"
_ev = []
_ns = time.perf_counter_ns


def mark(name):
    if ON:
        _ev.append((name, _ns()))


def reset():
    _ev.clear()


def summary(top=30):
    acc = collections.defaultdict(lambda: [0, 0])
    for (a, ta), (b, tb) in zip(_ev, _ev[1:]):
        e = acc[(a, b)]
        e[0] += 1
        e[1] += tb - ta
    rows = sorted(acc.items(), key=lambda kv: -kv[1][1])[:top]
    out = [f"{len(_ev)} events"]
    for (a, b), (n, t) in rows:
        out.append(f"{t / 1e6:9.2f} ms  {n:6d} x  {t / max(n, 1) / 1e3:8.1f} us  {a} -> {b}")
    return "\n".join(out)
