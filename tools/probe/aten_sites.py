"""Where do large ATen elementwise / conversion kernels come from?  Runs bench_resnet50.main()
(or bench.main() with `--target bench`) with torch.Tensor arithmetic / conversion / indexing
methods wrapped: every call on a CUDA tensor of >= 1M elements records the innermost
systemml_amd frames; the histogram goes to stderr.

    python tools/probe/aten_sites.py [--target bench] [bench / bench_resnet50 args]
"""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

SITES = collections.Counter()


def _wrap(name):
    orig = getattr(torch.Tensor, name)

    def f(self, *a, **k):
        if isinstance(self, torch.Tensor) and self.is_cuda and self.numel() >= (1 << 20):
            fr = [x for x in traceback.extract_stack(limit=14)[:-1] if "systemml_amd" in x.filename]
            key = (name, str(self.dtype)) + tuple(f"{os.path.basename(x.filename)}:{x.lineno}" for x in fr[-3:])
            SITES[key] += 1
        return orig(self, *a, **k)
    setattr(torch.Tensor, name, f)


for n in ("__mul__", "__rmul__", "__add__", "__radd__", "__sub__", "__rsub__", "__truediv__", "__neg__", "to",
          "float", "double", "sum", "mul", "add", "clone", "contiguous", "__getitem__", "__setitem__", "copy_",
          "exp", "log", "max", "amax", "masked_fill", "fill_", "zero_", "t", "reshape", "expand"):
    _wrap(n)

args = sys.argv[1:]
target = "bench_resnet50"
if args[:1] == ["--target"]:
    target, args = args[1], args[2:]
mod = __import__(target)
sys.argv = [target + ".py"] + args
try:
    mod.main()
finally:
    for k, v in SITES.most_common(40):
        print(f"{v:6d}  {k}", file=sys.stderr)
