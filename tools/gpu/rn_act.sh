#!/bin/bash
# bf16-activation kernels' tests, then ResNet-50 b256 with bf16 activations (cell-fallback
# trace on) and with fp32 activations.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_act_bf16.py tests/test_dnn_gpu.py -x -q -m gpu \
    --timeout 200 --timeout-method thread > gpurun_out/act_tests.log 2>&1 || exit $?
SYSML_CELL_TRACE=1 timeout -k 10 400 python bench_resnet50.py --batch 256 --steps 3 --warmup 1 \
    > gpurun_out/rn_act.log 2>&1 || exit $?
timeout -k 10 400 python bench_resnet50.py --batch 256 --steps 3 --warmup 1 --fp32-activations \
    > gpurun_out/rn_fp32.log 2>&1
