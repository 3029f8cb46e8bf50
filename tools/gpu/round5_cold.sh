#!/bin/bash
# Round-5 cold: the ResNet plan tests, a cold headline run (no overlap of the next step's
# compilation, one step, no warmup), and the 1.25M-row run.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rc_progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_resnet_plan.py \
    tests/test_cell_batch.py > gpurun_out/rc_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-overlap --steps 1 --warmup 0 > gpurun_out/rc_cold.log 2>&1
rc=$?; echo "cold rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 10 --warmup 3 > gpurun_out/rc_1250k.log 2>&1
rc=$?; echo "1250k rc=$rc $(date)" >> $P
echo "done $(date)" >> $P
