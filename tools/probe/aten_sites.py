"""Where do large ATen elementwise / conversion kernels come from?  Runs bench_resnet50.main()
with torch.Tensor arithmetic / conversion methods wrapped: every call on a CUDA tensor of
>= 1M elements records the innermost systemml_amd frames; the histogram goes to stderr.

    python tools/probe/aten_sites.py [bench_resnet50 args]
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


for n in ("__mul__", "__rmul__", "__add__", "__radd__", "__sub__", "__truediv__", "to", "float", "sum", "mul",
          "add", "clone", "contiguous"):
    _wrap(n)

import bench_resnet50  # noqa: E402

sys.argv = ["bench_resnet50.py"] + sys.argv[1:]
try:
    bench_resnet50.main()
finally:
    for k, v in SITES.most_common(40):
        print(f"{v:6d}  {k}", file=sys.stderr)
