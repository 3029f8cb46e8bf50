#!/bin/bash
# Headline bench at the full size and at the per-rank size of an 8-GPU run
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --rows 1250000 --steps 5 --warmup 2 > gpurun_out/bench_1250k.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
