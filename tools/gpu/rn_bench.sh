#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python bench_resnet50.py --steps 5 --warmup 2 > gpurun_out/resnet256.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_b.log 2>&1
