#!/bin/bash
# Round-5 I: Row template with K-wide vectors / multi-output programs (GPU tests), the headline
# with program merging off / on and with the softmax matcher off (generated plan), the icpt=2
# ATen call sites and bench, and the DNN GEMM split-K fill sweep.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/ri_progress.txt
echo "start $(date)" > $P
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_rowgen.py \
    tests/test_headline_fusion.py tests/test_vector_template.py > gpurun_out/ri_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
for m in 0 1; do
  SYSML_ROW_MERGE=$m timeout -k 10 300 python -u bench.py --rows 1250000 --steps 10 --warmup 3 > gpurun_out/ri_1250k_m$m.log 2>&1
  rc=$?; echo "1250k merge=$m rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
  SYSML_ROW_MERGE=$m timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/ri_10m_m$m.log 2>&1
  rc=$?; echo "10m merge=$m rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
done
SYSML_SOFTMAX_MATCHER=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/ri_10m_nomatch.log 2>&1
rc=$?; echo "10m nomatcher rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/probe/aten_sites.py --target bench --rows 2000000 --steps 2 --warmup 1 --icpt 2 \
    --compiler thread > gpurun_out/ri_aten_icpt2.txt 2>&1
rc=$?; echo "aten rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --icpt 2 > gpurun_out/ri_icpt2.log 2>&1
rc=$?; echo "icpt2 rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
for f in 480 720; do
  SYSML_GEMM_DNN_FILL=$f timeout -k 10 300 python -u tools/bench_gemm_dnn.py > gpurun_out/ri_gemm_fill$f.txt 2>&1
  rc=$?; echo "gemm fill=$f rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
done
echo "done $(date)" >> $P
