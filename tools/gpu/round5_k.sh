#!/bin/bash
# Round-5 K: generated row kernels after the column-major LDS side-matrix layout (tests, the
# matcher-off headline), ATen attribution of the icpt=2 headline, PMC passes over gemm.hip.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rk_progress.txt
echo "start $(date)" > $P
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_rowgen.py \
    > gpurun_out/rk_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
SYSML_SOFTMAX_MATCHER=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/rk_10m_nomatch.log 2>&1
rc=$?; echo "10m nomatcher rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/probe/aten_profile.py --target bench --rows 2000000 --steps 1 --warmup 1 --icpt 2 \
    --compiler thread > gpurun_out/rk_aten_icpt2.txt 2>&1
rc=$?; echo "aten rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
bash tools/gpu/pmc_gemm.sh > gpurun_out/rk_pmc.log 2>&1
rc=$?; echo "pmc rc=$rc $(date)" >> $P
echo "done $(date)" >> $P
