#!/bin/bash
# GPU suite + smoke, then a short ResNet-50 run listing the fused cell programs that miss the
# generated kernels (SYSML_CELL_TRACE=1).
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/full_gpu_tests.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
SYSML_CELL_TRACE=1 timeout -k 10 300 python bench_resnet50.py --batch 64 --steps 2 --warmup 1 \
    > gpurun_out/rn_trace.log 2>&1
