#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rowgen.py tests/test_outer.py tests/test_codegen.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1 || exit $?
timeout -k 10 200 python tools/bench_rowgen.py > gpurun_out/bench_rowgen.log 2>&1 || exit $?
timeout -k 10 300 python bench_resnet50.py --batch 32 --steps 5 --warmup 2 > gpurun_out/resnet.log 2>&1
