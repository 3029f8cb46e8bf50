#!/bin/bash
# quaternary + sddmm kernel tests first (new HIP kernel), then the full GPU suite and smoke
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_quaternary.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_quat14.log 2>&1
rc=$?; echo "pytest_quat rc=$rc" > gpurun_out/progress14.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu14.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc" >> gpurun_out/progress14.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke14.log 2>&1
echo "smoke rc=$?" >> gpurun_out/progress14.txt
