#!/bin/bash
# Vector template / if-conversion: GPU tests, then the headline at the 8-GPU per-rank size
# (1.25M rows) and at 10M rows.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=gpurun_out/vprog_progress.txt
echo "start $(date)" > $P
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_vector_template.py \
    -m gpu > gpurun_out/vprog_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 5 --warmup 2 --verbose > gpurun_out/bench_1250k.log 2>&1
rc=$?; echo "bench 1.25M rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --verbose > gpurun_out/bench_10m.log 2>&1
rc=$?; echo "bench 10M rc=$rc $(date)" >> $P
exit $rc
