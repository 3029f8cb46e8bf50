#!/bin/bash
# Round-5 X: deferred vector-program scalar reads -- GPU tests of the solver paths, headline at
# 1.25M and 10M rows with and without them.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rx_progress.txt
echo "start $(date)" > $P
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_vector_template.py \
    tests/test_gpu_algorithms.py tests/test_headline_fusion.py tests/test_runtime.py tests/test_runahead.py \
    tests/test_cell_batch.py > gpurun_out/rx_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
for d in 1 0 1; do
  SYSML_VPROG_DEFER=$d timeout -k 10 300 python -u bench.py --rows 1250000 --steps 10 --warmup 3 >> gpurun_out/rx_1250k.log 2>&1
  rc=$?; echo "1250k defer=$d rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
done
for d in 1 0; do
  SYSML_VPROG_DEFER=$d timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 >> gpurun_out/rx_10m.log 2>&1
  rc=$?; echo "10m defer=$d rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
done
echo "done $(date)" >> $P
