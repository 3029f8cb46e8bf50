"""Which framework call sites run torch operators on device tensors during one ResNet-50
training step at the plan-test configuration (tests/test_resnet_plan.py: image 64, batch 16,
bf16 activations from 64K cells): a TorchFunctionMode records each torch function / Tensor
method applied to a CUDA tensor of >= --min elements with its innermost systemml_amd frames.

    python tools/probe/resnet_aten.py [--min 65536] [--image 64] [--batch 16]
"""
import argparse
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
sys.path.insert(0, os.path.join(R, "tools", "probe"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min", type=int, default=65536)
    ap.add_argument("--image", type=int, default=64)
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    import torch
    import aten_modes as AM
    from test_resnet_plan import _compile
    from systemml_amd.api import executor as EX
    from systemml_amd.conf import DMLConfig
    from systemml_amd.runtime.udf import register_udf
    register_udf("sysml.bench.Sync", lambda ctx, A: (0.0,))
    AM.MIN = a.min
    cfg = DMLConfig(precision="single", gpu_min_cells=0, act_bf16_min_cells=1 << 16)
    cs, X, Y = _compile(image=a.image, batch=a.batch, config=cfg)
    EX.execute(cs, {"X": X, "Y": Y}, out=lambda s: None)
    torch.cuda.synchronize()
    with AM.Rec():
        EX.execute(cs, {"X": X, "Y": Y}, out=lambda s: None)
        torch.cuda.synchronize()
    for k, (n, b) in sorted(AM.SITES.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"{b / 1e6:9.2f} MB {n:6d}  {k}")


if __name__ == "__main__":
    main()
