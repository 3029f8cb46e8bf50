#!/bin/bash
# Round-5 Q: conv3 / wgrad tests, per-shape conv bench, ResNet-50 b256 (single-plane bf16 FC weights,
# the conv-bias fusion on the 1x1 GEMM path, ATen call sites at the plan-test config.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rq_progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dnn_gpu.py \
    -k "conv3_direct or wgrad" > gpurun_out/rq_conv3.log 2>&1
rc=$?; echo "conv3 tests rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_dnn_gpu.py \
    tests/test_resnet_plan.py tests/test_reorg_gpu.py tests/test_codegen.py tests/test_dl.py > gpurun_out/rq_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/bench_conv_rn50.py --no-miopen > gpurun_out/rq_conv.log 2>&1
rc=$?; echo "conv bench rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/rq_resnet.log 2>&1
rc=$?; echo "resnet rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/probe/resnet_aten.py > gpurun_out/rq_aten.log 2>&1
rc=$?; echo "aten rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnq_a -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 1 --warmup 1 > gpurun_out/rnq_a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnq_b -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 4 --warmup 1 > gpurun_out/rnq_b.log 2>&1 || exit $?
python3 tools/prof_diff.py gpurun_out/rnq_a gpurun_out/rnq_b 3 > gpurun_out/rq_rn_step.txt
rm -rf gpurun_out/rnq_a gpurun_out/rnq_b
echo "done $(date)" >> $P
