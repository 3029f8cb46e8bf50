#!/bin/bash
# Round-5 N: fused wdivmm (tests, ALS-CG 1M and 10M x 10M / 1e9 non-zeros, kernel stats of the
# 10M run).
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rn_progress.txt
echo "start $(date)" > $P
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_sparse_gpu.py \
    tests/test_gpu_algorithms.py > gpurun_out/rn_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench_als.py --steps 2 --warmup 1 > gpurun_out/rn_als_1m.log 2>&1
rc=$?; echo "als 1m rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench_als.py --rows 10000000 --cols 10000000 --per-row 100 --maxi 2 --steps 1 --warmup 1 \
    > gpurun_out/rn_als_10m.log 2>&1
rc=$?; echo "als 10m rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rn_als_prof -o run --output-format csv -- \
    python3 $R/bench_als.py --rows 10000000 --cols 10000000 --per-row 100 --maxi 2 --steps 1 --warmup 0 \
    > $R/gpurun_out/rn_als_prof.log 2>&1
rc=$?; echo "als prof rc=$rc $(date)" >> $P
echo "done $(date)" >> $P
