"""Runtime statistics (`-stats`), reference: utils/Statistics.java + GPUStatistics.java.

Records per-opcode counts and wall time (heavy hitters), compile/execute time,
and GPU kernel-library usage counters."""
from __future__ import annotations

import time


class Statistics:
    def __init__(self, enabled=False, sync=False):
        self.enabled = enabled
        self.sync = sync
        self.ops = {}
        self.t_start = time.perf_counter()
        self.t_parse = 0.0
        self.t_compile = 0.0
        self.t_exec = 0.0
        self.counters = {}

    def record(self, opcode, dt):
        c = self.ops.get(opcode)
        if c is None:
            self.ops[opcode] = [1, dt]
        else:
            c[0] += 1
            c[1] += dt

    def count(self, name, n=1):
        self.counters[name] = self.counters.get(name, 0) + n

    def report(self, k=10):
        lines = ["SystemML-AMD Statistics:",
                 f"Total elapsed time:\t\t{time.perf_counter() - self.t_start:.3f} sec.",
                 f"Total compilation time:\t\t{self.t_parse + self.t_compile:.3f} sec.",
                 f"Total execution time:\t\t{self.t_exec:.3f} sec."]
        if self.counters:
            for k_, v in sorted(self.counters.items()):
                lines.append(f"{k_}:\t{v}")
        if self.ops:
            lines.append(f"Heavy hitter instructions:")
            lines.append("  #  Instruction        Time(s)   Count")
            top = sorted(self.ops.items(), key=lambda kv: -kv[1][1])[:k]
            for i, (op, (n, t)) in enumerate(top, 1):
                lines.append(f"{i:3d}  {op:<18s} {t:8.3f} {n:7d}")
        return "\n".join(lines)
