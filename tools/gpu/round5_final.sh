#!/bin/bash
# Round-5 final: ALS kernel trace (cold run), ResNet-50 with the 128-row DNN GEMM tiles
# (SYSML_GEMM_DNN_T128 sweep), then the whole GPU suite, smoke() and the default bench.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rf_progress.txt
echo "start $(date)" > $P
for t in 0 512 4096; do
  SYSML_GEMM_DNN_T128=$t timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/rf_resnet_t$t.log 2>&1
  rc=$?; echo "resnet t128=$t rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ras_prof -o run --output-format csv -- \
    python3 $R/bench_als.py --rows 10000000 --cols 10000000 --per-row 100 --maxi 2 --steps 1 --warmup 0 \
    > $R/gpurun_out/ras_prof.log 2>&1
rc=$?; echo "als prof rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1200 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/rf_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/rf_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/rf_bench.log 2>&1
rc=$?; echo "bench rc=$rc $(date)" >> $P
echo "done $(date)" >> $P
