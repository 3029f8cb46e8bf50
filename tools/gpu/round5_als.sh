#!/bin/bash
# Round-5 ALS: kernel trace of ALS-CG 10M x 10M (1e9 non-zeros), one cold run (includes the
# one-time transposed-pattern build).
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ras_prof -o run --output-format csv -- \
    python3 $R/bench_als.py --rows 10000000 --cols 10000000 --per-row 100 --maxi 2 --steps 1 --warmup 0 \
    > $R/gpurun_out/ras_prof.log 2>&1
echo "rc=$?" >> $R/gpurun_out/ras_prof.log
