#!/bin/bash
# Round-5 V: column-aggregate tests with the one-pass partial fold; ResNet-50 b256 at 16 / 32 / 64
# rows per thread for the column aggregates; per-step kernels at the default.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rv_progress.txt
echo "start $(date)" > $P
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_codegen.py \
    tests/test_agg_gpu.py tests/test_resnet_plan.py tests/test_act_bf16.py tests/test_sparse_gpu.py tests/test_cell_batch.py \
    tests/test_dl.py > gpurun_out/rv_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
for r in 16 32 64; do
  SYSML_COL_RPT=$r timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/rv_resnet_$r.log 2>&1
  rc=$?; echo "resnet $r rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rvq_a -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 1 --warmup 1 > gpurun_out/rvq_a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rvq_b -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 4 --warmup 1 > gpurun_out/rvq_b.log 2>&1 || exit $?
python3 tools/prof_diff.py gpurun_out/rvq_a gpurun_out/rvq_b 3 > gpurun_out/rv_rn_step.txt
rm -rf gpurun_out/rvq_a gpurun_out/rvq_b
echo "done $(date)" >> $P
