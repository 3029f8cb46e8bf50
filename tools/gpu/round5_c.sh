#!/bin/bash
# Round-5 C: GEMM / DNN / run-ahead / aggregate / reorg GPU tests, the DNN GEMM shape benchmark,
# the headline at 1.25M and 10M rows (run-ahead off / on) and ResNet-50 b256.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rc_progress.txt
echo "start $(date)" > $P
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gemm_gpu.py tests/test_act_bf16.py tests/test_dnn_gpu.py tests/test_runahead.py \
    tests/test_vector_template.py tests/test_headline_fusion.py tests/test_agg_gpu.py tests/test_reorg_gpu.py \
    > gpurun_out/rc_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/bench_gemm_dnn.py > gpurun_out/rc_gemm_dnn.txt 2>&1
rc=$?; echo "gemm rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
for ra in 0 1; do
  SYSML_RUNAHEAD=$ra timeout -k 10 300 python -u bench.py --rows 1250000 --steps 10 --warmup 3 > gpurun_out/rc_1250k_$ra.log 2>&1
  rc=$?; echo "1250k ra=$ra rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
  SYSML_RUNAHEAD=$ra timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/rc_10m_$ra.log 2>&1
  rc=$?; echo "10m ra=$ra rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/rc_resnet.log 2>&1
rc=$?; echo "resnet rc=$rc $(date)" >> $P
echo "done $(date)" >> $P
