#!/bin/bash
# Round-5 validation A: new-kernel GPU tests (run-ahead, DNN GEMM, aggregates, reorg), the
# headline at 1.25M / 10M rows with run-ahead off / on, ResNet-50 b256, and a 1.25M-row kernel
# trace with idle-gap attribution.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/ra_progress.txt
echo "start $(date)" > $P
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_runahead.py tests/test_vector_template.py tests/test_headline_fusion.py tests/test_gemm_gpu.py \
    tests/test_act_bf16.py tests/test_sparse_gpu.py tests/test_agg_gpu.py tests/test_reorg_gpu.py \
    > gpurun_out/ra_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P
# keep going after ordinary test failures (rc 1); stop on crashes / timeouts
[ $rc -gt 1 ] && exit $rc
for ra in 0 1; do
  SYSML_RUNAHEAD=$ra timeout -k 10 300 python -u bench.py --rows 1250000 --steps 10 --warmup 3 > gpurun_out/ra_1250k_$ra.log 2>&1
  rc=$?; echo "1250k ra=$ra rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
done
for ra in 0 1; do
  SYSML_RUNAHEAD=$ra timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/ra_10m_$ra.log 2>&1
  rc=$?; echo "10m ra=$ra rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/ra_resnet.log 2>&1
rc=$?; echo "resnet rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ra_trace -o run --output-format csv -- \
    python3 $R/bench.py --rows 1250000 --steps 3 --warmup 2 > $R/gpurun_out/ra_trace.log 2>&1
rc=$?; echo "trace rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
F=$(find $R/gpurun_out/ra_trace -name '*kernel_trace.csv' | head -1)
python3 $R/tools/trace_idle.py $F 0.2 > $R/gpurun_out/ra_idle.txt 2>&1
S=$(find $R/gpurun_out/ra_trace -name '*kernel_stats.csv' | head -1)
cp $S $R/gpurun_out/ra_kernel_stats.csv
rm -rf $R/gpurun_out/ra_trace
echo "done $(date)" >> $P
