#!/bin/bash
# Round-5 O: fixed tests (device-scalar lix, ResNet no-library plan), wdivmm launch-shape sweep
# on 10M x 10M / 1B non-zeros, ALS-CG 10M, ResNet-50 b256 per-step kernels.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/ro_progress.txt
echo "start $(date)" > $P
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_codegen.py \
    tests/test_resnet_plan.py tests/test_reorg_gpu.py tests/test_sparse_gpu.py tests/test_dnn_gpu.py \
    > gpurun_out/ro_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
for w in 32 64 16; do for u in 4 8; do
  SYSML_WD_WAVES=$w SYSML_WD_UNROLL=$u timeout -k 10 200 python -u tools/bench_wdivmm.py >> gpurun_out/ro_wd.log 2>&1
  rc=$?; echo "wd $w $u rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
done; done
timeout -k 10 100 python -u tools/bench_wdivmm.py --rows 100000 --cols 100000 --per-row 100 >> gpurun_out/ro_wd.log 2>&1
rc=$?; echo "wd small rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench_als.py --rows 10000000 --cols 10000000 --per-row 100 --maxi 2 --steps 1 --warmup 1 \
    > gpurun_out/ro_als_10m.log 2>&1
rc=$?; echo "als 10m rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/ro_resnet.log 2>&1
rc=$?; echo "resnet rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnq_a -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 1 --warmup 1 > gpurun_out/rnq_a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnq_b -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 4 --warmup 1 > gpurun_out/rnq_b.log 2>&1 || exit $?
python3 tools/prof_diff.py gpurun_out/rnq_a gpurun_out/rnq_b 3 > gpurun_out/ro_rn_step.txt
rm -rf gpurun_out/rnq_a gpurun_out/rnq_b
echo "done $(date)" >> $P
