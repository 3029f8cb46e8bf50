#!/bin/bash
# Round-5 M+N: tests of this round's kernels (column MAgg, fused wdivmm, device-scalar lix, RCCL
# one-rank dist paths, parfor), ResNet-50 b256, headline 10M / 1.25M, ALS-CG 1M / 10M.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rmn_progress.txt
echo "start $(date)" > $P
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_codegen.py \
    tests/test_dist_rccl_gpu.py tests/test_runtime.py tests/test_rowgen.py tests/test_act_bf16.py tests/test_resnet_plan.py \
    tests/test_dnn_gpu.py tests/test_dl.py tests/test_sparse_gpu.py tests/test_reorg_gpu.py tests/test_gpu_algorithms.py \
    > gpurun_out/rmn_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/rmn_resnet.log 2>&1
rc=$?; echo "resnet rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/rmn_10m.log 2>&1
rc=$?; echo "10m rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 10 --warmup 3 > gpurun_out/rmn_1250k.log 2>&1
rc=$?; echo "1250k rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench_als.py --steps 2 --warmup 1 > gpurun_out/rmn_als_1m.log 2>&1
rc=$?; echo "als 1m rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench_als.py --rows 10000000 --cols 10000000 --per-row 100 --maxi 2 --steps 1 --warmup 1 \
    > gpurun_out/rmn_als_10m.log 2>&1
rc=$?; echo "als 10m rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnq_a -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 1 --warmup 1 > gpurun_out/rnq_a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnq_b -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 4 --warmup 1 > gpurun_out/rnq_b.log 2>&1 || exit $?
python3 tools/prof_diff.py gpurun_out/rnq_a gpurun_out/rnq_b 3 > gpurun_out/rmn_rn_step.txt
rm -rf gpurun_out/rnq_a gpurun_out/rnq_b
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rmn_als_prof -o run --output-format csv -- \
    python3 $R/bench_als.py --rows 10000000 --cols 10000000 --per-row 100 --maxi 2 --steps 1 --warmup 0 \
    > $R/gpurun_out/rmn_als_prof.log 2>&1
rc=$?; echo "als prof rc=$rc $(date)" >> $P
echo "done $(date)" >> $P
