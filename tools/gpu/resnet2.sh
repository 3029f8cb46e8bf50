#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python bench_resnet50.py --batch 32 --steps 5 --warmup 2 > gpurun_out/resnet.log 2>&1 || exit $?
timeout -k 10 300 python bench_resnet50.py --batch 32 --steps 5 --warmup 2 --no-fusion > gpurun_out/resnet_nofuse.log 2>&1
