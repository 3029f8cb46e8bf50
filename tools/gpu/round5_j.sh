#!/bin/bash
# Round-5 J: partial sums on agg.hip (headline, icpt=2), the generated plan with the softmax
# matcher off after the narrow-size cost fix, and the Row-template / aggregate GPU tests.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rj_progress.txt
echo "start $(date)" > $P
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_rowgen.py \
    tests/test_agg_gpu.py tests/test_headline_fusion.py > gpurun_out/rj_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/rj_10m.log 2>&1
rc=$?; echo "10m rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 10 --warmup 3 > gpurun_out/rj_1250k.log 2>&1
rc=$?; echo "1250k rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --icpt 2 > gpurun_out/rj_icpt2.log 2>&1
rc=$?; echo "icpt2 rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
SYSML_SOFTMAX_MATCHER=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/rj_10m_nomatch.log 2>&1
rc=$?; echo "10m nomatcher rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $R
SYSML_SOFTMAX_MATCHER=0 bash tools/gpu/prof_step.sh || exit $?
mv gpurun_out/per_step_kernels.txt gpurun_out/rj_nomatch_step.txt
rm -rf gpurun_out/pstep1 gpurun_out/pstep3
echo "done $(date)" >> $P
