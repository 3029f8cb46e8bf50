#!/bin/bash
# ResNet-50 round check: DL / Cell-template GPU tests, the b256 bench, then the per-step kernel
# table (tools/gpu/rn_prof2.sh).
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_act_bf16.py \
    tests/test_dnn_gpu.py tests/test_resnet_plan.py tests/test_codegen.py -m gpu \
    > gpurun_out/rc_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/rc_resnet.log 2>&1 || exit $?
bash tools/gpu/rn_prof2.sh
