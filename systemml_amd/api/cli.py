"""Command-line driver (reference: api/DMLScript.java, bin/systemml,
bin/systemml-standalone.py).

    python -m systemml_amd -f script.dml [-nvargs k=v ...] [-args v1 v2 ...]
        [-stats [N]] [-explain [hops|runtime]] [-config conf.xml] [-gpu] [-cpu]
        [-python] [-s "inline script"] [-exec singlenode|hybrid|spmd]

For multi-GPU SPMD execution launch one process per GPU:
    python -m torch.distributed.run --nproc-per-node 8 -m systemml_amd -f script.dml ...
"""
from __future__ import annotations

import os
import sys

from ..conf import DMLConfig, get_default_config
from ..parser.errors import DMLException, DMLScriptStop


def parse_args(argv):
    opts = {"file": None, "script": None, "nvargs": {}, "args": [], "stats": 0, "explain": "", "config": None,
            "gpu": None, "pydml": False, "exec": None, "debug": False, "help": False}
    i = 0
    while i < len(argv):
        a = argv[i]
        la = a.lstrip("-")
        if la == "f":
            opts["file"] = argv[i + 1]
            i += 2
        elif la == "s":
            opts["script"] = argv[i + 1]
            i += 2
        elif la == "nvargs":
            i += 1
            while i < len(argv) and not argv[i].startswith("-"):
                k, _, v = argv[i].partition("=")
                opts["nvargs"][k] = v
                i += 1
        elif la == "args":
            i += 1
            while i < len(argv) and not argv[i].startswith("-"):
                opts["args"].append(argv[i])
                i += 1
        elif la == "stats":
            opts["stats"] = 10
            if i + 1 < len(argv) and argv[i + 1].isdigit():
                opts["stats"] = int(argv[i + 1])
                i += 1
            i += 1
        elif la == "explain":
            opts["explain"] = "hops"
            if i + 1 < len(argv) and not argv[i + 1].startswith("-"):
                opts["explain"] = argv[i + 1]
                i += 1
            i += 1
        elif la == "config":
            opts["config"] = argv[i + 1]
            i += 2
        elif la == "gpu":
            opts["gpu"] = True
            if i + 1 < len(argv) and argv[i + 1] == "force":
                i += 1
            i += 1
        elif la == "cpu":
            opts["gpu"] = False
            i += 1
        elif la in ("python", "pydml"):
            opts["pydml"] = True
            i += 1
        elif la == "exec":
            opts["exec"] = argv[i + 1]
            i += 2
        elif la == "debug":
            opts["debug"] = True
            i += 1
        elif la in ("help", "h"):
            opts["help"] = True
            i += 1
        else:
            raise SystemExit(f"unknown option {a}")
    return opts


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    o = parse_args(argv)
    if o["help"] or (o["file"] is None and o["script"] is None):
        print(__doc__)
        return 0
    cfg = DMLConfig.from_xml(o["config"]) if o["config"] else get_default_config().copy()
    if o["gpu"] is not None:
        cfg.gpu = o["gpu"]
    if o["exec"] == "singlenode":
        cfg.dist_min_rows = 1 << 62
    cfg.explain = o["explain"]
    if o["file"]:
        with open(o["file"]) as f:
            src = f.read()
        fname = os.path.abspath(o["file"])
        pydml = o["pydml"] or fname.endswith(".pydml")
    else:
        src, fname, pydml = o["script"], "", o["pydml"]
    args = dict(o["nvargs"])
    for k, v in enumerate(o["args"], 1):
        args[str(k)] = v
    from ..parallel import dist as D
    from ..utils.stats import Statistics
    from . import executor as EX
    world = int(os.environ.get("WORLD_SIZE", "1"))
    ctx = D.init() if world > 1 else None
    stats = Statistics(enabled=o["stats"] > 0) if o["stats"] else None
    rc = 0
    try:
        cs = EX.compile_script(src, args, config=cfg, pydml=pydml, filename=fname)
        if o["debug"]:
            from ..utils.debugger import Debugger
            Debugger(cs).run()
        else:
            _, ectx = EX.execute(cs, {}, stats=stats, dist=ctx)
            if stats is not None:
                from ..ops import kernels
                stats.counters.update(kernels.counters)
                ectx.print(stats.report(o["stats"]))
    except DMLScriptStop as e:
        print(f"An Error Occurred : {e}", file=sys.stderr)
        rc = 1
    except DMLException as e:
        print(f"An Error Occurred : {type(e).__name__} -- {e}", file=sys.stderr)
        rc = 1
    finally:
        if ctx is not None:
            D.shutdown()
    return rc


if __name__ == "__main__":
    sys.exit(main())
