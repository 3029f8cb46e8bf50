#!/bin/bash
# Host overhead at the per-rank size of an 8-GPU run (1.25M rows per rank): bench timing,
# wall-clock stack samples of the timed steps, and the lazy-scalar (device-resident) variant.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=gpurun_out/host_progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python bench.py --rows 1250000 --steps 5 --warmup 2 --verbose \
    --sample-profile gpurun_out/host_samples_1250k.txt > gpurun_out/bench_1250k.log 2>&1
rc=$?; echo "bench 1.25M rc=$rc $(date)" >> $P
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --rows 1250000 --steps 5 --warmup 2 --lazy > gpurun_out/bench_1250k_lazy.log 2>&1
rc=$?; echo "bench 1.25M lazy rc=$rc $(date)" >> $P
exit $rc
