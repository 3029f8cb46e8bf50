#!/bin/bash
# Round-5 R: conv3 / wgrad tests (3x3 filter-gradient kernel with register prefetch), conv bench with
# and without the 3x3 filter-gradient kernel, ResNet-50 b256, ATen sites at the plan-test config.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rr_progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dnn_gpu.py \
    -k "conv3_direct or wgrad" > gpurun_out/rr_conv3.log 2>&1
rc=$?; echo "conv3 tests rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_resnet_plan.py \
    tests/test_act_bf16.py tests/test_dl.py > gpurun_out/rr_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
SYSML_WGRAD3=1 timeout -k 10 300 python -u tools/bench_conv_rn50.py --no-miopen > gpurun_out/rr_conv_w3.log 2>&1
rc=$?; echo "conv bench w3 rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/rr_resnet.log 2>&1
rc=$?; echo "resnet rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
SYSML_WGRAD3=1 timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/rr_resnet_w3.log 2>&1
rc=$?; echo "resnet w3 rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/probe/resnet_aten.py > gpurun_out/rr_aten.log 2>&1
rc=$?; echo "aten rc=$rc $(date)" >> $P
echo "done $(date)" >> $P
