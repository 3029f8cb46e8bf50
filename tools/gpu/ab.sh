#!/bin/bash
# A/B of the headline bench: as is, with the Row / Outer templates off, and as is again
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/ab_1.log 2>&1 || exit $?
SYSML_ROWGEN=0 timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/ab_norow.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --verbose > gpurun_out/ab_2.log 2>&1 || exit $?
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 3 --warmup 2 > gpurun_out/resnet256.log 2>&1
