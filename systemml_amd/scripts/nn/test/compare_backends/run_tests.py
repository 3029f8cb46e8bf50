"""CPU-vs-GPU comparison of the DNN builtins (reference: scripts/nn/test/compare_backends/
run_tests.sh and its per-operator test_*.sh drivers, which run each script once in CP mode and
once with `-gpu force` and compare the outputs with compare.dml).

For every operator, sparsity, stride and padding: gen_inputs.dml writes the operands, run_op.dml
runs the operator on the CPU backend (fp64) and on the GPU backend (HIP kernels), and
compare.dml prints MATCH / MISMATCH.  Exit status 1 when anything mismatches.

    python systemml_amd/scripts/nn/test/compare_backends/run_tests.py [--quick] [--precision double|single]
"""
from __future__ import annotations

import argparse
import itertools
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, *[".."] * 5)))      # the repository root
OPS = ["conv2d", "conv2d_backward_filter", "conv2d_backward_data", "max_pool", "max_pool_backward",
       "avg_pool", "avg_pool_backward", "softmax"]


def _run(script, nvargs, config, out):
    from systemml_amd.api import executor as EX
    with open(os.path.join(HERE, script)) as f:
        src = f.read()
    cs = EX.compile_script(src, dict(nvargs), config=config, filename=os.path.join(HERE, script))
    EX.execute(cs, {}, out=out)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="one sparsity / stride / padding per operator")
    ap.add_argument("--precision", default="double", choices=["double", "single"])
    ap.add_argument("--ops", default=",".join(OPS))
    a = ap.parse_args(argv)
    from systemml_amd.conf import DMLConfig
    cpu = DMLConfig(gpu=False)
    gpu = DMLConfig(gpu=True, precision=a.precision, gpu_min_cells=0)
    eps = 1e-6 if a.precision == "double" else 2e-3
    dims = dict(N=5, C=3, H=28, W=28, F=32, Hf=3, Wf=3, pool=2)
    sparsities = [0.2] if a.quick else [0.1, 0.2, 0.5, 0.6, 0.9]
    strides = [1] if a.quick else [1, 2, 3]
    pads = [1] if a.quick else [0, 1, 2]
    lines = []
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            for sp, st, pd in itertools.product(sparsities, strides, pads):
                args = dict(dims, sp=sp, stride=st, pad=pd)
                _run("gen_inputs.dml", args, cpu, lines.append)
                for op in a.ops.split(","):
                    if "pool" in op and pd >= dims["pool"]:
                        continue            # a pooling window must overlap the image: padding < pool size
                    args_op = dict(args, op=op)
                    _run("run_op.dml", dict(args_op, out="out_cp.mtx"), cpu, lines.append)
                    _run("run_op.dml", dict(args_op, out="out_gpu.mtx"), gpu, lines.append)
                    tag = f"{op}: sparsity={sp}, stride={st}, pad={pd}"
                    _run("compare.dml", {"1": "out_cp.mtx", "2": "out_gpu.mtx", "3": tag, "eps": eps}, cpu,
                         lines.append)
        finally:
            os.chdir(cwd)
    res = [ln for ln in lines if ln.startswith(("MATCH", "MISMATCH"))]
    for ln in res:
        print(ln)
    bad = [ln for ln in res if ln.startswith("MISMATCH")]
    print(f"{len(res) - len(bad)} of {len(res)} comparisons match")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
