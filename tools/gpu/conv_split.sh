#!/bin/bash
# Sweep of the implicit-GEMM convolutions' split-K heuristic on the ResNet-50 shapes (b256),
# after the bf16 convolution tests.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_act_bf16.py \
    tests/test_dnn_gpu.py > gpurun_out/cs_tests.log 2>&1 || exit $?
for cfg in "2048 512" "2048 1536" "2048 2048" "2048 3072" "4096 2048"; do
  set -- $cfg
  SYSML_CONV_SPLIT_BLOCKS=$1 SYSML_CONV_SPLIT_MINK=$2 timeout -k 10 300 python -u tools/bench_conv_rn50.py --no-miopen \
      > gpurun_out/cs2_$1_$2.log 2>&1 || exit $?
done
