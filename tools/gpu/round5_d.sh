#!/bin/bash
# Round-5 D: DNN GEMM shapes after the tile retune, ResNet-50 b256 and its per-step kernel
# table, and the GPU tests touched since C (aggregates, DNN incl. compare_backends).
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rd_progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python -u tools/bench_gemm_dnn.py > gpurun_out/rd_gemm_dnn.txt 2>&1
rc=$?; echo "gemm rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/rd_resnet.log 2>&1
rc=$?; echo "resnet rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_agg_gpu.py tests/test_dnn_gpu.py tests/test_act_bf16.py tests/test_gemm_gpu.py > gpurun_out/rd_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnq_a -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 1 --warmup 1 > gpurun_out/rnq_a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnq_b -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 4 --warmup 1 > gpurun_out/rnq_b.log 2>&1 || exit $?
python3 tools/prof_diff.py gpurun_out/rnq_a gpurun_out/rnq_b 3 > gpurun_out/rd_rn_step.txt
rm -rf gpurun_out/rnq_a gpurun_out/rnq_b
echo "done $(date)" >> $P
