#!/bin/bash
# full GPU test suite, bench, rocprof kernel stats of one bench step
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/ -q -m gpu -x > gpurun_out/pytest_gpu13.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc" > gpurun_out/progress13.txt
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_10m_r13.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/progress13.txt
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof13 -o bench --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 > $R/gpurun_out/prof13_bench.log 2>&1
echo "prof rc=$?" >> $R/gpurun_out/progress13.txt
