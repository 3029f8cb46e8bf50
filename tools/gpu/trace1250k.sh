#!/bin/bash
# Kernel trace of the per-rank-size headline step (1.25M rows; extra args pass through to
# bench.py), for idle-gap attribution on the host (tools/trace_idle.py, tools/trace_regions.py).
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/t1250k -o run --output-format csv -- \
    python3 $R/bench.py --rows ${ROWS:-1250000} --steps 3 --warmup 2 "$@" > $R/gpurun_out/t1250k.log 2>&1 || exit $?
F=$(find $R/gpurun_out/t1250k -name '*kernel_trace.csv' | head -1)
python3 $R/tools/trace_idle.py $F 0.2 > $R/gpurun_out/t1250k_idle.txt 2>&1
python3 $R/tools/trace_regions.py $F 200 > $R/gpurun_out/t1250k_regions.txt 2>&1
tail -n 3 $R/gpurun_out/t1250k.log
