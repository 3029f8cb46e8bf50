#!/bin/bash
# Round-5 G: column-aggregate kernel tests, parfor vs for on device-resident inputs, and the
# ATen call sites of the icpt=2 headline (which operators still run torch kernels).
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rg_progress.txt
echo "start $(date)" > $P
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_agg_gpu.py \
    > gpurun_out/rg_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
for cfg in "--n 4096 --precision single" "--n 4096 --precision double" "--n 1024 --iters 16 --precision single"; do
  timeout -k 10 300 python -u tools/bench_parfor.py $cfg >> gpurun_out/rg_parfor.txt 2>&1
  rc=$?; echo "parfor [$cfg] rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python -u tools/probe/aten_sites.py --target bench --rows 2000000 --steps 2 --warmup 1 --icpt 2 \
    > gpurun_out/rg_aten_icpt2.txt 2>&1
rc=$?; echo "aten rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --icpt 2 > gpurun_out/rg_icpt2.log 2>&1
rc=$?; echo "icpt2 rc=$rc $(date)" >> $P
echo "done $(date)" >> $P
