#!/bin/bash
# Round-5 M: column MAgg (batch-norm statistics in one pass), Cell plan cost fix, parfor in-place
# fix, RCCL one-rank dist paths; ResNet-50 b256 + per-step kernels, headline 10M / 1.25M.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rm_progress.txt
echo "start $(date)" > $P
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_codegen.py \
    tests/test_dist_rccl_gpu.py tests/test_runtime.py tests/test_rowgen.py tests/test_act_bf16.py tests/test_resnet_plan.py \
    tests/test_dnn_gpu.py tests/test_dl.py > gpurun_out/rm_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/rm_resnet.log 2>&1
rc=$?; echo "resnet rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/rm_10m.log 2>&1
rc=$?; echo "10m rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 10 --warmup 3 > gpurun_out/rm_1250k.log 2>&1
rc=$?; echo "1250k rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnq_a -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 1 --warmup 1 > gpurun_out/rnq_a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnq_b -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 4 --warmup 1 > gpurun_out/rnq_b.log 2>&1 || exit $?
python3 tools/prof_diff.py gpurun_out/rnq_a gpurun_out/rnq_b 3 > gpurun_out/rm_rn_step.txt
rm -rf gpurun_out/rnq_a gpurun_out/rnq_b
echo "done $(date)" >> $P
