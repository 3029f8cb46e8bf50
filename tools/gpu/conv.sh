#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=gpurun_out/conv_progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python -u -m pytest tests/test_dnn_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_dnn.log 2>&1
rc=$?; echo "dnn tests rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/bench_conv.py > gpurun_out/conv_kbench.log 2>&1
rc=$?; echo "conv bench rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench_resnet50.py --batch 128 --steps 4 --warmup 2 > gpurun_out/resnet128.log 2>&1
rc=$?; echo "resnet rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab.sh
rc=$?; echo "ab rc=$rc $(date)" >> $P
exit $rc
