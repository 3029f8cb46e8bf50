"""Run one convolution kernel repeatedly (for rocprofv3 --pmc / --kernel-trace runs).
    python tools/prof_conv.py [mode] [dtype]   mode 0 fwd / 1 bwd data / 2 bwd filter"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from systemml_amd.ops import kernels as K  # noqa: E402

mode = int(sys.argv[1]) if len(sys.argv) > 1 else 0
dt = {"bf16": torch.bfloat16, "fp32": torch.float32}[sys.argv[2] if len(sys.argv) > 2 else "bf16"]
N, C, H, W, F, k, s, p = 64, 64, 56, 56, 64, 3, 1, 1
dev = torch.device("cuda:0")
X = torch.randn(N, C * H * W, device=dev, dtype=dt)
Wt = torch.randn(F, C * k * k, device=dev, dtype=dt)
G = torch.randn(N, F * H * W, device=dev, dtype=dt)
for _ in range(10):
    K.conv2d(mode, X if mode != 1 else None, Wt if mode != 2 else None, G if mode else None,
             N, C, H, W, F, k, k, s, s, p, p)
torch.cuda.synchronize()
print("done")
