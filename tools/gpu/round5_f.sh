#!/bin/bash
# Round-5 F: parfor GPU timing (bench_parfor at 4096^2 single / 2048^2 / bf16-class sizes), the
# touched GPU tests (gemm incl. one-pass weight cast, reorg incl. mixed-device append, ResNet
# plan incl. the library-kernel trace test, parfor), and the GLM regression perftest at 100k.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rf_progress.txt
echo "start $(date)" > $P
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm_gpu.py \
    tests/test_reorg_gpu.py tests/test_resnet_plan.py tests/test_runtime.py tests/test_parfor_opt.py > gpurun_out/rf_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
for cfg in "--n 4096 --precision single" "--n 2048 --precision single" "--n 4096 --precision double" "--n 1024 --iters 16 --precision single"; do
  timeout -k 10 300 python -u tools/bench_parfor.py $cfg >> gpurun_out/rf_parfor.txt 2>&1
  rc=$?; echo "parfor [$cfg] rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python3 -m systemml_amd.perftest --dir /tmp/perftest_data --sizes 100k_1k --families regression \
    --out gpurun_out/rf_perftest_100k.jsonl > gpurun_out/rf_perftest.log 2>&1
rc=$?; echo "perftest rc=$rc $(date)" >> $P
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/rf_resnet.log 2>&1
rc=$?; echo "resnet rc=$rc $(date)" >> $P
echo "done $(date)" >> $P
