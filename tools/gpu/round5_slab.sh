#!/bin/bash
# Round-5 slab: backward-filter split-K into a slab (no atomics) -- DNN tests, conv bench and
# ResNet-50 with SYSML_CONV_SLAB=1 / 0.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rsl_progress.txt
echo "start $(date)" > $P
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_dnn_gpu.py \
    tests/test_act_bf16.py tests/test_dl.py tests/test_resnet_plan.py > gpurun_out/rsl_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
for v in 1 0; do
  SYSML_CONV_SLAB=$v timeout -k 10 300 python -u tools/bench_conv_rn50.py --no-miopen > gpurun_out/rsl_conv_$v.log 2>&1
  rc=$?; echo "conv slab=$v rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
  SYSML_CONV_SLAB=$v timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/rsl_resnet_$v.log 2>&1
  rc=$?; echo "resnet slab=$v rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
done
echo "done $(date)" >> $P
