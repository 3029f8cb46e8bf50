#!/bin/bash
# ResNet-50 iteration 3: DNN / codegen GPU tests, conv-shape benchmark, b256 per-step profile and bench.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 600 python -u -m pytest tests/test_act_bf16.py tests/test_dnn_gpu.py tests/test_codegen.py \
    tests/test_vector_template.py tests/test_headline_fusion.py tests/test_dl_dataparallel.py -q -m gpu \
    --timeout 200 --timeout-method thread > gpurun_out/it3_tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_conv_rn50.py --reps 3 --no-miopen > gpurun_out/it3_conv.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnr_a -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 1 --warmup 1 > gpurun_out/rnr_a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnr_b -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 4 --warmup 1 > gpurun_out/rnr_b.log 2>&1 || exit $?
python3 tools/prof_diff.py gpurun_out/rnr_a gpurun_out/rnr_b 3 > gpurun_out/rnr_step.txt || exit $?
rm -rf gpurun_out/rnr_a gpurun_out/rnr_b
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/it3_b256.log 2>&1
