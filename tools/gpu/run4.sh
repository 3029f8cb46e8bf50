#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_kernels.py -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" > gpurun_out/progress6.txt
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python tools/bench_kernels.py --out gpurun_out/kbench3.json > gpurun_out/kbench3.log 2>&1
rc=$?; echo "kbench rc=$rc" >> gpurun_out/progress6.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_10m_r6.log 2>&1
echo "bench rc=$?" >> gpurun_out/progress6.txt
