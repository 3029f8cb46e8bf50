#!/bin/bash
# ResNet-50 iteration: bf16-activation / DNN GPU tests, the conv-shape benchmark (GEMM paths on,
# stride-1 col2im variant), the ATen call-site probe, then the b256 bench.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_act_bf16.py tests/test_dnn_gpu.py -x -q -m gpu \
    --timeout 200 --timeout-method thread > gpurun_out/it_tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_conv_rn50.py --reps 3 --no-miopen > gpurun_out/it_conv.log 2>&1 || exit $?
SYSML_COL2IM_MAX_HW=3136 timeout -k 10 300 python tools/bench_conv_rn50.py --reps 3 --no-miopen > gpurun_out/it_conv_c2i.log 2>&1 || exit $?
timeout -k 10 300 python tools/probe/aten_sites.py --batch 64 --steps 2 --warmup 1 > gpurun_out/it_sites.log 2>&1 || exit $?
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 3 --warmup 1 > gpurun_out/it_bench.log 2>&1
