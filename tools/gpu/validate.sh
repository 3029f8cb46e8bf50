#!/bin/bash
# Round validation on one GPU box: the GPU test suite, smoke(), and the headline bench.
# Each step has its own time limit; the script stops at the first crash / time-out.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=gpurun_out/validate_progress.txt
echo "start $(date)" > $P
timeout -k 10 ${T_TESTS:-700} python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(date)" >> $P
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(date)" >> $P
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 5 --warmup 2} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc $(date)" >> $P
exit $rc
