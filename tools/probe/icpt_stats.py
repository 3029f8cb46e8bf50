"""Heavy-hitter instruction statistics (utils/stats.py, synchronised per instruction) of the
headline MultiLogReg at a given intercept mode, on the bench's synthetic data:

    python tools/probe/icpt_stats.py [--rows 1000000] [--icpt 2]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import bench  # noqa: E402
from systemml_amd.api import executor as EX  # noqa: E402
from systemml_amd.api.mlcontext import SCRIPTS_DIR  # noqa: E402
from systemml_amd.conf import DMLConfig  # noqa: E402
from systemml_amd.ops.backend import backend  # noqa: E402
from systemml_amd.utils.stats import Statistics  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--icpt", type=int, default=2)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    cfg = DMLConfig(precision="single", dist_min_rows=100_000)
    backend.configure(cfg)
    _, _, X2, lab = bench.gen_data(None, a.rows, 1000, 5, torch.bfloat16)
    src = open(os.path.join(SCRIPTS_DIR, "algorithms", "MultiLogReg.dml")).read()
    args = dict(X="X", Y="Y", B="B", icpt=a.icpt, reg=0.01, tol=0.0001, moi=20, mii=5)
    for k in range(2):
        cs = EX.compile_script(src, args, inputs={"X": X2, "Y_vec": lab}, outputs=["B_out"], config=cfg)
        st = Statistics(enabled=True) if k == 1 else None
        EX.execute(cs, {"X": X2, "Y_vec": lab}, out=lambda s: None, stats=st)
        torch.cuda.synchronize()
    print(st.report(25))


if __name__ == "__main__":
    main()
