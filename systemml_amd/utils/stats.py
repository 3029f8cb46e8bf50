"""Runtime statistics (`-stats`), reference: utils/Statistics.java + GPUStatistics.java.

Records per-opcode counts and wall time (heavy hitters; on a GPU backend every instruction
is synchronised before it is timed, so the times are execution and not launch times unless
sync=False is requested), compile / execute time, dynamic-recompilation and buffer-pool
counters, host<->HBM transfers made by the CP/GPU placement (count, bytes, time), the
caching allocator's HBM statistics, the generated (codegen) operators' launch and hipRTC
compile / cache counts and the invocation counts of the in-tree HIP kernels."""
from __future__ import annotations

import time


class Statistics:
    def __init__(self, enabled=False, sync=None):
        self.enabled = enabled
        if sync is None:                       # default: time executions, not launches, on a GPU
            import torch
            sync = torch.cuda.is_available()
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
        lines += gpu_report()
        if self.ops:
            lines.append(f"Heavy hitter instructions:")
            lines.append("  #  Instruction        Time(s)   Count")
            top = sorted(self.ops.items(), key=lambda kv: -kv[1][1])[:k]
            for i, (op, (n, t)) in enumerate(top, 1):
                lines.append(f"{i:3d}  {op:<18s} {t:8.3f} {n:7d}")
        return "\n".join(lines)


def gpu_report():
    """GPUStatistics-style section: transfers made by the placement, HBM allocator state and
    HIP kernel invocations (empty without a GPU)."""
    import torch
    out = []
    from ..runtime import instructions as I
    t = I.transfer_stats
    if t["h2d"] or t["d2h"]:
        out.append(f"Host->HBM transfers (count/MB):\t{t['h2d']}/{t['h2d_bytes'] / 1e6:.1f}")
        out.append(f"HBM->host transfers (count/MB):\t{t['d2h']}/{t['d2h_bytes'] / 1e6:.1f}")
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        ms = torch.cuda.memory_stats()
        out.append(f"HBM allocated / peak / reserved (GB):\t{ms.get('allocated_bytes.all.current', 0) / 1e9:.2f} / "
                   f"{ms.get('allocated_bytes.all.peak', 0) / 1e9:.2f} / {ms.get('reserved_bytes.all.current', 0) / 1e9:.2f}")
        out.append(f"HBM allocations / frees / alloc retries:\t{ms.get('allocation.all.allocated', 0)} / "
                   f"{ms.get('allocation.all.freed', 0)} / {ms.get('num_alloc_retries', 0)}")
    from ..ops import cell, outer, rowgen
    cg = [f"{name}.{k}={round(v, 3) if isinstance(v, float) else v}"
          for name, st in (("cell", cell.stats), ("row", rowgen.stats), ("outer", outer.stats))
          for k, v in sorted(st.items()) if v]
    if cg:                                      # Statistics.java "Codegen compile / class cache" lines
        out.append("Codegen operators (launches, hipRTC compiles / cache hits):\t" + ", ".join(cg))
    from ..ops import kernels as K
    if K.counters:
        out.append("HIP kernel invocations:\t" + ", ".join(f"{k}={v}" for k, v in sorted(K.counters.items())))
    return out
