#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_kernels.py -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" > gpurun_out/progress2.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o bench --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 > $R/gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc" >> $R/gpurun_out/progress2.txt
[ $rc -ne 0 ] && exit $rc
cd $R
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --xdtype fp32 > gpurun_out/bench_fp32.log 2>&1
echo "fp32 rc=$?" >> gpurun_out/progress2.txt
