"""Process-wide compute backend state: device, compute dtype, kernel library.

The CP backend runs on host tensors in fp64 (reference LibMatrix* semantics);
the GPU backend keeps matrices resident in MI355X HBM in the configured
precision and routes the hot operators to the in-tree HIP kernels
(`systemml_amd/ops/hip/*.hip` → `libsysml_hip.so`).
"""
from __future__ import annotations

import os
import torch


import threading

_TLS = threading.local()


class Backend:
    def __init__(self):
        self._device = torch.device("cpu")
        self.dtype = torch.float64
        self.use_kernels = False
        self.bf16_min_cells = 0
        self.act_bf16_min_cells = 0  # >0: fused cellwise results / conv outputs this large stored bf16
        self.stream_sync = False
        self.small_cells = 0        # GPU backend: matrices below this many cells live on the host
        self.lazy = False           # GPU backend: HBM-resident scalars (runtime/scalars.DevScalar)

    @property
    def device(self):
        # a parfor worker thread on another GPU sees its own device (runtime/parfor.py)
        d = getattr(_TLS, "device", None)
        return self._device if d is None else d

    @device.setter
    def device(self, d):
        self._device = d

    def set_thread_device(self, d):
        _TLS.device = d

    # run-ahead loop state of the executing thread (runtime/program.py _exec_while_runahead):
    # `defer` -- vector programs return their scalars as device-resident values instead of
    # reading them back; `live` -- device address of the fp64 flag (the previous iteration's
    # loop predicate) that the streaming kernels of a speculatively queued iteration read
    # first: 0.0 means the iteration is dead and they return at once (0 = no flag)
    @property
    def defer(self):
        return getattr(_TLS, "defer", False)

    @property
    def live(self):
        return getattr(_TLS, "live", 0)

    def set_runahead(self, defer, live=0):
        _TLS.defer = defer
        if live != getattr(_TLS, "live", 0):
            _TLS.live = live
            if self.use_kernels:
                from . import kernels
                kernels.load(required=True).sysml_set_live(live or None)

    @property
    def on_gpu(self):
        return self._device.type == "cuda"

    def configure(self, config=None):
        want_gpu = True if config is None else (config.gpu and not config.force_cpu)
        if os.environ.get("SYSTEMML_AMD_FORCE_CPU") == "1":
            want_gpu = False
        if want_gpu and torch.cuda.is_available():
            idx = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
            torch.cuda.set_device(idx)
            self.device = torch.device("cuda", idx)
            prec = "double" if config is None else config.precision
            self.dtype = torch.float32 if prec in ("single", "float", "fp32", "bf16") else torch.float64
            self.bf16_min_cells = 0 if config is None else config.bf16_storage_min_cells
            self.act_bf16_min_cells = 0 if config is None else int(getattr(config, "act_bf16_min_cells", 0))
            self.small_cells = 16384 if config is None else int(config.gpu_min_cells)
            self.lazy = bool(config is not None and getattr(config, "lazy_scalars", False))
            if self.lazy:
                self.small_cells = 0
            want_k = True if config is None else config.hip_kernels
            if want_k:
                from . import kernels
                kernels.load(required=True)
                self.use_kernels = True
            else:
                self.use_kernels = False
        else:
            self.device = torch.device("cpu")
            self.dtype = torch.float64
            self.use_kernels = False
            self.bf16_min_cells = 0
            self.act_bf16_min_cells = 0
            self.small_cells = 0
            self.lazy = False
        return self


backend = Backend()


def home(numel: int) -> torch.device:
    """Where a matrix of `numel` cells lives: HBM, or host memory for small matrices on a GPU
    backend (hybrid CP / GPU placement, runtime/instructions.py:_placed)."""
    if backend.small_cells > 0 and numel < backend.small_cells:
        return _CPU
    return backend.device


_CPU = torch.device("cpu")


def place(t: torch.Tensor) -> torch.Tensor:
    """Move a freshly created/loaded matrix into the backend's memory + dtype."""
    if t.dtype == torch.bfloat16:
        return t.to(backend.device)
    dev = home(t.numel())
    if t.device != dev or t.dtype != backend.dtype:
        t = t.to(device=dev, dtype=backend.dtype)
    return t


def maybe_bf16(t: torch.Tensor) -> torch.Tensor:
    """Store large read-only inputs in bf16 (fp32 accumulate in every kernel)."""
    if backend.on_gpu and backend.bf16_min_cells > 0 and t.numel() >= backend.bf16_min_cells \
            and t.dtype != torch.bfloat16:
        return t.to(torch.bfloat16)
    return t
