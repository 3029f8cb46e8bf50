#!/bin/bash
# Round-5 E: ResNet plan tests (incl. the no-library-GEMM trace test), icpt=2 at 10M with its
# per-step kernel table, the cold single-step run, disk space and the regression perftest
# family at 1M x 1K (reads + GLM predict).
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/re_progress.txt
echo "start $(date)" > $P
df -h /tmp . >> $P 2>&1
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_resnet_plan.py \
    > gpurun_out/re_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --icpt 2 > gpurun_out/re_icpt2.log 2>&1
rc=$?; echo "icpt2 rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-overlap > gpurun_out/re_cold.log 2>&1
rc=$?; echo "cold rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/prof_step.sh --icpt 2 || exit $?
mv gpurun_out/per_step_kernels.txt gpurun_out/re_icpt2_step.txt
rm -rf gpurun_out/pstep1 gpurun_out/pstep3
echo "prof rc=0 $(date)" >> $P
PT_LIMIT=600 bash tools/gpu/perftest.sh 1M_1k regression
rc=$?; echo "perftest rc=$rc $(date)" >> $P
echo "done $(date)" >> $P
