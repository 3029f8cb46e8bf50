#!/bin/bash
# Round-5 B: DNN GEMM shape benchmark against the library GEMM, host cProfile of the 1.25M-row
# headline with run-ahead on / off, and the aggregate / reorg / bf16-conv GPU tests.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rb_progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python -u tools/bench_gemm_dnn.py > gpurun_out/rb_gemm_dnn.txt 2>&1
rc=$?; echo "gemm rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
for ra in 0 1; do
  SYSML_RUNAHEAD=$ra timeout -k 10 300 python -u bench.py --rows 1250000 --steps 4 --warmup 2 \
      --host-profile gpurun_out/rb_hprof_$ra.txt > gpurun_out/rb_hprof_$ra.log 2>&1
  rc=$?; echo "hprof ra=$ra rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_agg_gpu.py tests/test_reorg_gpu.py tests/test_act_bf16.py > gpurun_out/rb_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P
echo "done $(date)" >> $P
