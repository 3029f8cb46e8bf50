#!/bin/bash
# Round-5 U: tests (pixel padding, column aggregates with more row blocks, DNN, sparse), ResNet-50
# b256 + per-step kernels, headline icpt=2 with the reused augmented copy.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/ru_progress.txt
echo "start $(date)" > $P
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm_gpu.py \
    tests/test_codegen.py tests/test_agg_gpu.py tests/test_dnn_gpu.py tests/test_resnet_plan.py tests/test_act_bf16.py \
    tests/test_rowgen.py tests/test_headline_fusion.py > gpurun_out/ru_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/ru_resnet.log 2>&1
rc=$?; echo "resnet rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --icpt 2 --steps 3 --warmup 2 > gpurun_out/ru_icpt2.log 2>&1
rc=$?; echo "icpt2 rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ruq_a -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 1 --warmup 1 > gpurun_out/ruq_a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ruq_b -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 4 --warmup 1 > gpurun_out/ruq_b.log 2>&1 || exit $?
python3 tools/prof_diff.py gpurun_out/ruq_a gpurun_out/ruq_b 3 > gpurun_out/ru_rn_step.txt
rm -rf gpurun_out/ruq_a gpurun_out/ruq_b
echo "done $(date)" >> $P
