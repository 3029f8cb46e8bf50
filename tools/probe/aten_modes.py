"""Which framework call sites run torch operators on large device tensors: runs bench.main()
(or another module's main with `--target`) under a TorchFunctionMode that records, for every
torch function / Tensor method applied to a CUDA tensor of >= 1M elements, the innermost
systemml_amd frames and the bytes of its tensor arguments; prints the sites by bytes.
Only the timed phase counts when `--after-warmup` is given (bench prints no marker, so the
mode is switched on after the first `--skip` seconds).

    python tools/probe/aten_modes.py [--target bench] [--top 40] [bench args]
"""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
from torch.overrides import TorchFunctionMode  # noqa: E402

SITES = collections.defaultdict(lambda: [0, 0])
MIN = 1 << 20          # smallest tensor (elements) recorded
_SKIP = {"crow_indices", "col_indices", "values", "__get__", "__repr__", "size", "dim", "numel", "is_contiguous", "data_ptr", "stride", "element_size",
         "__len__", "shape", "dtype", "device", "is_cuda", "layout", "storage_offset", "__hash__", "__eq__"}


def _same_storage(r, a):
    if r.layout != torch.strided or a.layout != torch.strided:
        return False                       # sparse results: count them
    return r.untyped_storage().data_ptr() == a.untyped_storage().data_ptr()


class Rec(TorchFunctionMode):
    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = getattr(func, "__name__", str(func))
        r = func(*args, **kwargs)
        if name in _SKIP or not isinstance(r, torch.Tensor) or not r.is_cuda:
            return r
        big = [a for a in list(args) + list(kwargs.values())
               if isinstance(a, torch.Tensor) and a.is_cuda and a.numel() >= MIN]
        # calls that produce new device memory or write in place (views and no-op casts launch nothing)
        if big and (name.endswith("_") or not any(_same_storage(r, a) for a in big)):
            fr = [x for x in traceback.extract_stack(limit=16)[:-1] if "systemml_amd" in x.filename]
            key = (name,) + tuple(f"{os.path.basename(x.filename)}:{x.lineno}" for x in fr[-3:])
            SITES[key][0] += 1
            SITES[key][1] += sum(a.numel() * a.element_size() for a in big)
        return r


def main():
    args = sys.argv[1:]
    target, top = "bench", 40
    while args[:1] and args[0] in ("--target", "--top"):
        if args[0] == "--target":
            target = args[1]
        else:
            top = int(args[1])
        args = args[2:]
    mod = __import__(target)
    sys.argv = [target + ".py"] + args
    with Rec():
        mod.main()
    for k, (n, b) in sorted(SITES.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{b / 1e9:9.2f} GB {n:6d}  {k}", file=sys.stderr)


if __name__ == "__main__":
    main()
