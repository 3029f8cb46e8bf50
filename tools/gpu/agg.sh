#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_agg_gpu.py tests/test_codegen.py tests/test_dnn_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_agg.log 2>&1 || exit $?
timeout -k 10 300 python bench_resnet50.py --steps 5 --warmup 2 > gpurun_out/resnet256.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
