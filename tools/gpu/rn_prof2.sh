#!/bin/bash
# Per-step kernel table of ResNet-50 b256 with bf16 activations (two rocprofv3 runs that differ
# by 3 timed steps, differenced by tools/prof_diff.py), then the bench at b256 / b128.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnq_a -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 1 --warmup 1 > gpurun_out/rnq_a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnq_b -o run --output-format csv -- \
    python3 bench_resnet50.py --batch 256 --steps 4 --warmup 1 > gpurun_out/rnq_b.log 2>&1 || exit $?
python3 tools/prof_diff.py gpurun_out/rnq_a gpurun_out/rnq_b 3 > gpurun_out/rnq_step.txt || exit $?
rm -rf gpurun_out/rnq_a gpurun_out/rnq_b


