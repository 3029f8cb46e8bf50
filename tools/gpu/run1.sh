#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo start $(date) > gpurun_out/progress.txt
timeout -k 10 420 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/progress.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/progress.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --rows 1000000 --steps 2 --warmup 1 --verbose --stats > gpurun_out/bench_1m.log 2>&1
rc=$?; echo "bench1m rc=$rc" >> gpurun_out/progress.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --stats > gpurun_out/bench_10m.log 2>&1
rc=$?; echo "bench10m rc=$rc" >> gpurun_out/progress.txt
exit $rc
