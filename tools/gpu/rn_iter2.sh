#!/bin/bash
# ResNet-50 iteration 2: compiler / kernel GPU tests, ATen call-site probe, b256 bench.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_act_bf16.py tests/test_dnn_gpu.py tests/test_codegen.py \
    tests/test_vector_template.py tests/test_headline_fusion.py -q -m gpu \
    --timeout 200 --timeout-method thread > gpurun_out/it2_tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/probe/aten_sites.py --batch 64 --steps 2 --warmup 1 > gpurun_out/it2_sites.log 2>&1 || exit $?
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 3 --warmup 1 > gpurun_out/it2_bench.log 2>&1
