#!/bin/bash
# Round-5 Z: intercept views -- padded copy only on reuse (and reused across runs), one-pass
# scalar ops on the view's matrix; icpt=2 / icpt=1 / icpt=0 headline, GPU algorithm tests.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rz_progress.txt
echo "start $(date)" > $P
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_algorithms.py \
    tests/test_headline_fusion.py tests/test_runtime.py > gpurun_out/rz_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
for i in 2 1 0; do
  timeout -k 10 300 python -u bench.py --icpt $i --steps 3 --warmup 2 >> gpurun_out/rz_icpt.log 2>&1
  rc=$?; echo "icpt $i rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
done
echo "done $(date)" >> $P
