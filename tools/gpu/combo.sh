#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=gpurun_out/combo_progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python bench.py --rows 1250000 --steps 5 --warmup 2 > gpurun_out/bench_1250k.log 2>&1
rc=$?; echo "bench1250k rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench_resnet50.py --batch 64 --steps 4 --warmup 2 > gpurun_out/resnet64.log 2>&1
rc=$?; echo "resnet64 rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 250 python bench_resnet50.py --batch 128 --steps 3 --warmup 2 > gpurun_out/resnet128.log 2>&1
rc=$?; echo "resnet128 rc=$rc $(date)" >> $P
exit $rc
