#!/bin/bash
# MFMA chain kernel: numerics first (exact-integer layout tests), then A/B microbench, then bench.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -k "mfma_exact" > gpurun_out/pytest_mfma.log 2>&1
rc=$?; echo "pytest_mfma rc=$rc" > gpurun_out/progress11.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -m pytest tests/ -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc" >> gpurun_out/progress11.txt
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python tools/bench_kernels.py --out gpurun_out/kbench8.json > gpurun_out/kbench8.log 2>&1
rc=$?; echo "kbench rc=$rc" >> gpurun_out/progress11.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_10m_r11.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/progress11.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke11.log 2>&1
echo "smoke rc=$?" >> gpurun_out/progress11.txt
