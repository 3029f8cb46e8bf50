#!/bin/bash
# ResNet-50 training bench (bf16 conv MFMA) and its per-kernel statistics
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python bench_resnet50.py --steps 4 --warmup 2 > gpurun_out/resnet.log 2>&1
rc=$?; echo "resnet rc=$rc $(date)" > gpurun_out/resnet_progress.txt
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rprof -o run --output-format csv -- \
    python3 $R/bench_resnet50.py --steps 3 --warmup 1 > $R/gpurun_out/resnet_prof.log 2>&1
rc=$?; echo "resnet prof rc=$rc $(date)" >> $R/gpurun_out/resnet_progress.txt
exit $rc
