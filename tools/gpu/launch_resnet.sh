#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_launch.py --profile gpurun_out/launch_prof.txt > gpurun_out/launch.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_codegen.py tests/test_rowgen.py tests/test_outer.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1 || exit $?
bash tools/gpu/resnet2.sh
