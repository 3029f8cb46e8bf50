"""Configuration (reference: conf/DMLConfig.java, conf/CompilerConfig.java,
conf/SystemML-config.xml.template).

Keys keep the reference names where one exists (e.g. `sysml.gpu.availableGPUs`,
`sysml.floating.point.precision`, `sysml.parallel.ops`, `sysml.stats.maxWrapLength`)
and add the MI355X-specific ones (`sysml.gpu.storage.bf16.mincells`,
`sysml.dist.minrows`).  A config can be loaded from the reference's XML format.
"""
from __future__ import annotations

import os
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field


@dataclass
class DMLConfig:
    # execution
    gpu: bool = True                    # use the MI355X backend when a GPU is visible
    force_cpu: bool = False
    precision: str = "double"           # 'double' | 'single' : compute dtype of matrices on GPU
    bf16_storage_min_cells: int = 0     # >0: large read-only inputs stored bf16 (fp32 accumulate)
    act_bf16_min_cells: int = 0         # >0: fused cellwise results and convolution outputs with at least
                                        # this many cells stored bf16 (DL activations / gradients; fp32 math)
    dist_min_rows: int = 100_000        # row-partition matrices with >= rows across ranks (SPMD)
    gpu_min_cells: int = 16384          # GPU backend: smaller matrices (and their operators) stay on host
    lazy_scalars: bool = False          # GPU backend: aggregates return HBM-resident scalars (runtime/scalars.DevScalar);
                                        # implies every matrix lives in HBM (gpu_min_cells ignored)
    parallelism: int = 8                # parfor local workers
    parfor_gpu_streams: int = 1         # parfor on the GPU backend without par=: worker streams per device
                                        # (1 = one worker per GPU, as the reference's rule-based optimizer;
                                        # 4 streams on one MI355X measured 0.26-0.86x of the serial loop,
                                        # profiles/parfor_gpu_r5*.txt)
    parfor_gpus: int = 1                # parfor on the GPU backend: devices used by one process's workers
    # compiler
    rewrites: bool = True
    fusion: bool = True
    const_propagation: bool = True
    # output / diagnostics
    stats: bool = False
    stats_count: int = 10
    explain: str = ""                   # '' | hops | runtime | recompile_hops
    print_rank0_only: bool = True
    scratch: str = "scratch_space"
    seed: int = -1                      # >= 0: rand/sample without a seed draw a repeatable sequence
    hip_kernels: bool = True            # use in-tree HIP kernels for the hot ops on GPU
    hip_graphs: bool = False
    # compressed linear algebra (ops/compress.py): "false" | "true" | "auto" (auto: ratio >= 3)
    compressed_linalg: str = "false"
    # buffer pool (runtime/bufferpool.py): HBM -> pinned host -> local disk
    bufferpool: bool = True
    bufferpool_hbm_fraction: float = 0.85
    bufferpool_host_bytes: int = 64 << 30
    bufferpool_spill_dir: str = ""
    extra: dict = field(default_factory=dict)

    _XML_KEYS = {
        "sysml.floating.point.precision": ("precision", str),
        "sysml.gpu.storage.bf16.mincells": ("bf16_storage_min_cells", int),
        "sysml.gpu.activation.bf16.mincells": ("act_bf16_min_cells", int),
        "sysml.dist.minrows": ("dist_min_rows", int),
        "sysml.gpu.mincells": ("gpu_min_cells", int),
        "sysml.gpu.lazy.scalars": ("lazy_scalars", lambda v: str(v).lower() == "true"),
        "sysml.parallel.ops": ("parallelism", lambda v: 8 if str(v).lower() == "true" else 1),
        "sysml.random.seed": ("seed", int),
        "sysml.localtmpdir": ("scratch", str),
        "sysml.scratch": ("scratch", str),
        "sysml.stats.maxHeavyHitters": ("stats_count", int),
        "sysml.codegen.enabled": ("fusion", lambda v: str(v).lower() == "true"),
        "sysml.gpu.hip.kernels": ("hip_kernels", lambda v: str(v).lower() == "true"),
        "sysml.bufferpool.hbm.fraction": ("bufferpool_hbm_fraction", float),
        "sysml.compressed.linalg": ("compressed_linalg", lambda v: str(v).lower()),
        "sysml.bufferpool.spill.dir": ("bufferpool_spill_dir", str),
    }

    def set(self, key, value):
        if key in self._XML_KEYS:
            attr, conv = self._XML_KEYS[key]
            setattr(self, attr, conv(value))
        elif hasattr(self, key) and not key.startswith("_"):
            cur = getattr(self, key)
            if isinstance(cur, bool):
                value = value if isinstance(value, bool) else str(value).lower() in ("1", "true", "yes")
            elif isinstance(cur, int):
                value = int(value)
            setattr(self, key, value)
        else:
            self.extra[key] = value

    @classmethod
    def from_xml(cls, path):
        cfg = cls()
        root = ET.parse(path).getroot()
        for child in root:
            if child.text is not None:
                cfg.set(child.tag, child.text.strip())
        return cfg

    def copy(self):
        import copy
        return copy.deepcopy(self)


_default = None


def get_default_config():
    global _default
    if _default is None:
        _default = DMLConfig()
        env = os.environ.get("SYSTEMML_AMD_CONFIG")
        if env and os.path.exists(env):
            _default = DMLConfig.from_xml(env)
    return _default
