#!/bin/bash
# Per-rank-size (1.25M rows) headline: timing, kernel trace with idle-gap attribution, and
# host cProfile of the timed steps.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/hostprof_progress.txt
echo "start $(date)" > $P
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vector_template.py -m gpu > gpurun_out/hp_tests.log 2>&1 && timeout -k 10 300 python -u bench.py --rows 1250000 --steps 5 --warmup 2 > gpurun_out/hp_bench.log 2>&1
rc=$?; echo "bench rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 3 --warmup 2 --host-profile gpurun_out/hp_cprofile.txt > gpurun_out/hp_cprof.log 2>&1
rc=$?; echo "cprofile rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/hp_trace -o run --output-format csv -- \
    python3 $R/bench.py --rows 1250000 --steps 3 --warmup 2 > $R/gpurun_out/hp_trace.log 2>&1
rc=$?; echo "trace rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
F=$(find $R/gpurun_out/hp_trace -name '*kernel_trace.csv' | head -1)
python3 $R/tools/trace_idle.py $F 0.2 > $R/gpurun_out/hp_idle.txt 2>&1
S=$(find $R/gpurun_out/hp_trace -name '*kernel_stats.csv' | head -1)
cp $S $R/gpurun_out/hp_kernel_stats.csv
echo "done $(date)" >> $P
