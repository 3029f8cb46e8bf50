"""Buffer pool: HBM-resident live variables with eviction to pinned host memory and
spill to local disk (reference: runtime/controlprogram/caching/{CacheableData,
LazyWriteBuffer,CacheStatistics}.java — the JVM buffer pool evicts MatrixBlocks to the
local file system when the heap budget is exceeded and restores them on the next acquire).

MI355X design: the device (288 GB HBM) is the "memory" tier, pinned host RAM the
first eviction tier and a local spill directory the second.

* Variables of all live frames (the main program and every active function call) are
  candidates; the ones the current basic block reads are pinned.
* Eviction is least-recently-used by `tread` access time.
* Triggers: (1) proactive, after a basic block, when allocated HBM exceeds
  `bufferpool_hbm_fraction` of the device; (2) reactive, when an instruction raises
  `torch.OutOfMemoryError`: evict, empty the caching allocator, retry the instruction.
* An evicted variable is an `Evicted` handle in its frame; `tread` restores it to the
  device transparently (pinned H2D copy, non-blocking on the current stream).
"""
from __future__ import annotations

import itertools
import os
import tempfile
import time

import torch


_SIDE = {}


def _side_stream(dev):
    """One copy stream per device: evictions / restores overlap the compute stream."""
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(device=dev)
    return s


class Evicted:
    """Handle of an evicted device tensor.  Host tier: pinned buffer filled by an async D2H copy
    on the device's side stream (ordered after the producing stream by an event; the device
    block is released to the caching allocator only after the copy, via record_stream).
    Disk tier: a synchronous torch.save of our own spill file."""
    __slots__ = ("cpu", "path", "device", "dtype", "shape", "nbytes", "done")

    def __init__(self, t: torch.Tensor, spill_dir=None):
        self.device = t.device
        self.dtype = t.dtype
        self.shape = tuple(t.shape)
        self.nbytes = t.numel() * t.element_size()
        self.path = None
        self.cpu = None
        self.done = None
        if spill_dir is not None:
            fd, self.path = tempfile.mkstemp(prefix="sysml_spill_", suffix=".pt", dir=spill_dir)
            os.close(fd)
            torch.save(t.detach().cpu(), self.path)
        elif t.is_cuda:
            host = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            side = _side_stream(t.device)
            side.wait_stream(torch.cuda.current_stream(t.device))
            with torch.cuda.stream(side):
                host.copy_(t, non_blocking=True)
                t.record_stream(side)
                self.done = torch.cuda.Event()
                self.done.record(side)
            self.cpu = host
        else:
            self.cpu = t.clone()

    def restore(self) -> torch.Tensor:
        if self.path is not None:
            t = torch.load(self.path, weights_only=True)   # our own spill file
            try:
                os.remove(self.path)
            except OSError:
                pass
            return t.to(self.device, non_blocking=True)
        if self.device.type != "cuda":
            return self.cpu
        cur = torch.cuda.current_stream(self.device)
        side = _side_stream(self.device)
        with torch.cuda.stream(side):
            if self.done is not None:
                side.wait_event(self.done)
            d = torch.empty(self.shape, dtype=self.dtype, device=self.device)
            d.copy_(self.cpu, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(side)
        cur.wait_event(ev)
        d.record_stream(cur)
        return d

    def __repr__(self):
        where = "disk" if self.path else "host"
        return f"Evicted({self.shape}, {self.dtype}, on {where})"


class BufferPool:
    def __init__(self, config=None):
        self.frac = float(getattr(config, "bufferpool_hbm_fraction", 0.85) if config else 0.85)
        self.host_budget = int(getattr(config, "bufferpool_host_bytes", 64 << 30) if config else 64 << 30)
        self.spill_dir = (getattr(config, "bufferpool_spill_dir", "") if config else "") or None
        self.enabled = bool(getattr(config, "bufferpool", True) if config else True)
        self.clock = itertools.count()
        self.last_use = {}          # id(frame), name -> tick
        self.host_bytes = 0
        self.stats = {"evict_host": 0, "evict_disk": 0, "restore": 0, "oom_retries": 0,
                      "bytes_evicted": 0, "time_evict": 0.0, "time_restore": 0.0}
        self.min_bytes = 1 << 20          # smaller variables are never worth evicting
        self.host_tensors = False         # tests: treat host tensors as the "device" tier
        self._total = None
        self._next_check = 0.0
        self.check_interval = 0.05        # s between proactive HBM-usage checks (the query costs ~0.1 ms)

    # ------------------------------------------------------------------ access
    def touch(self, frame, name):
        self.last_use[(id(frame), name)] = next(self.clock)

    def restore(self, frame, name, v):
        t0 = time.perf_counter()
        t = v.restore()
        if v.path is None:
            self.host_bytes -= v.nbytes
        frame[name] = t
        self.stats["restore"] += 1
        self.stats["time_restore"] += time.perf_counter() - t0
        return t

    # ------------------------------------------------------------------ eviction
    def _candidates(self, frames, keep):
        out = []
        for fr in frames:
            for name, v in fr.items():
                if name in keep and fr is frames[-1]:
                    continue
                if isinstance(v, torch.Tensor) and (v.is_cuda or self.host_tensors) and \
                        v.numel() * v.element_size() >= self.min_bytes:
                    out.append((self.last_use.get((id(fr), name), -1), fr, name, v))
        out.sort(key=lambda x: x[0])
        return out

    def evict(self, frames, keep=(), need_bytes=None):
        """Evict LRU device variables until `need_bytes` are released (all candidates if None)."""
        t0 = time.perf_counter()
        freed = 0
        for _, fr, name, v in self._candidates(frames, set(keep)):
            # a tensor may be shared by several variables: evict all its aliases together
            nb = v.numel() * v.element_size()
            to_disk = self.spill_dir is not None and self.host_bytes + nb > self.host_budget
            h = Evicted(v, spill_dir=self.spill_dir if to_disk else None)
            for fr2 in frames:
                for n2, v2 in list(fr2.items()):
                    if v2 is v:
                        fr2[n2] = h
            if to_disk:
                self.stats["evict_disk"] += 1
            else:
                self.host_bytes += nb
                self.stats["evict_host"] += 1
            self.stats["bytes_evicted"] += nb
            freed += nb
            if need_bytes is not None and freed >= need_bytes:
                break
        if freed and torch.cuda.is_available():
            torch.cuda.empty_cache()
        self.stats["time_evict"] += time.perf_counter() - t0
        return freed

    def maybe_evict(self, frames, keep=()):
        if not self.enabled:
            return 0
        now = time.perf_counter()
        if now < self._next_check and self.frac > 0:
            return 0
        self._next_check = now + self.check_interval
        if not torch.cuda.is_available():
            self._next_check = float("inf")
            return 0
        dev = torch.cuda.current_device()
        if self._total is None:
            self._total = torch.cuda.get_device_properties(dev).total_memory
        total = self._total
        used = torch.cuda.memory_allocated(dev)
        budget = self.frac * total
        if used <= budget:
            return 0
        return self.evict(frames, keep, need_bytes=int(used - budget))

    def on_oom(self, frames, keep=()):
        self.stats["oom_retries"] += 1
        return self.evict(frames, keep, need_bytes=None)

    def report(self):
        s = self.stats
        return (f"Buffer pool: evicted {s['evict_host']} to host, {s['evict_disk']} to disk "
                f"({s['bytes_evicted'] / 2**20:.1f} MiB), restored {s['restore']}, OOM retries "
                f"{s['oom_retries']}, evict {s['time_evict']:.3f}s / restore {s['time_restore']:.3f}s")
