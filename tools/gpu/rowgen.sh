#!/bin/bash
# Row-template GPU tests, kernel bandwidth, then the round validation (tests, smoke, bench)
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rowgen.py tests/test_outer.py -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_rowgen.log 2>&1
rc=$?; echo "rowgen tests rc=$rc $(date)" > gpurun_out/rowgen_progress.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/bench_rowgen.py > gpurun_out/bench_rowgen.log 2>&1
rc=$?; echo "rowgen bench rc=$rc $(date)" >> gpurun_out/rowgen_progress.txt
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/validate.sh
