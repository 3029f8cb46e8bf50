#!/bin/bash
# Round-5 L: the whole GPU test suite, ATen attribution of icpt=2 (stack-grouped), and the
# 1.25M-row host profile with the callers of every blocking read.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rl_progress.txt
echo "start $(date)" > $P
timeout -k 10 1500 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/rl_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python -u tools/probe/aten_profile.py --target bench --rows 2000000 --steps 1 --warmup 1 --icpt 2 \
    --compiler thread > gpurun_out/rl_aten_icpt2.txt 2>&1
rc=$?; echo "aten rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 4 --warmup 3 --host-profile gpurun_out/rl_hprof.txt \
    > gpurun_out/rl_hprof.log 2>&1
rc=$?; echo "hprof rc=$rc $(date)" >> $P

SYSML_SOFTMAX_MATCHER=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/rl_10m_nomatch.log 2>&1
rc=$?; echo "10m nomatcher rc=$rc $(date)" >> $P
SYSML_SOFTMAX_MATCHER=0 timeout -k 10 300 python -u bench.py --rows 1250000 --steps 10 --warmup 3 > gpurun_out/rl_1250k_nomatch.log 2>&1
rc=$?; echo "1250k nomatcher rc=$rc $(date)" >> $P
echo "done $(date)" >> $P
