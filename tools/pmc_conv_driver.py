"""Runs each ResNet-50 convolution kernel variant a few times at batch 64 (bf16 activations) for
rocprofv3 --pmc passes (tools/gpu/pmc_conv.sh): the direct 3x3 convolution (conv3.hip, forward and
backward data), the implicit-GEMM backward filter (dnn.hip), the 1x1 filter gradient (wgrad.hip)
and the 1x1 forward on the image-blocked GEMM (gemm.hip)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from systemml_amd.ops import kernels as K
    from systemml_amd.ops.backend import backend
    K.load(required=True)
    backend.act_bf16_min_cells = 1
    dev = torch.device("cuda")
    N = 64
    g = torch.Generator(device=dev).manual_seed(1)
    for (C, H, F, k) in ((64, 56, 64, 3), (256, 14, 256, 3), (256, 14, 1024, 1), (64, 56, 256, 1)):
        p = k // 2
        X = torch.randn(N, C * H * H, generator=g, device=dev).to(torch.bfloat16)
        W = torch.randn(F, C * k * k, generator=g, device=dev) * 0.05
        D = torch.randn(N, F * H * H, generator=g, device=dev).to(torch.bfloat16)
        for _ in range(3):
            K.conv2d(0, X, W, None, N, C, H, H, F, k, k, 1, 1, p, p)
            K.conv2d(1, None, W, D, N, C, H, H, F, k, k, 1, 1, p, p)
            K.conv2d(2, X, None, D, N, C, H, H, F, k, k, 1, 1, p, p)
    torch.cuda.synchronize()
    print("done", {k: v for k, v in K.counters.items() if "conv" in k or "wgrad" in k}, flush=True)


if __name__ == "__main__":
    main()
