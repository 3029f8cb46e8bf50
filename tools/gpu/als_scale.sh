#!/bin/bash
# ALS-CG (BASELINE config #4): 1M x 1M / 1e8 non-zeros, then 10M x 10M / 1e9 non-zeros on one
# GPU, and a kernel profile of the 10M run.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u bench_als.py --steps 2 --warmup 1 > gpurun_out/als_1m.log 2>&1 || exit $?
timeout -k 10 600 python -u bench_als.py --rows 10000000 --cols 10000000 --per-row 100 --maxi 2 --steps 1 --warmup 1 \
    > gpurun_out/als_10m.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/als_prof -o run --output-format csv -- \
    python3 $R/bench_als.py --rows 10000000 --cols 10000000 --per-row 100 --maxi 2 --steps 1 --warmup 0 \
    > $R/gpurun_out/als_prof.log 2>&1 || exit $?
