#!/bin/bash
# Scaling rehearsal on one GPU: the per-rank size of an 8-GPU run (1.25M rows) on one rank,
# then 8 SPMD ranks sharing the GPU over gloo (10M rows, fallback-gather / all-reduce counts).
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=gpurun_out/scale_progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 5 --warmup 2 --verbose > gpurun_out/bench_1250k.log 2>&1
rc=$?; echo "bench 1.25M rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
SYSML_DIST_BACKEND=gloo SYSML_DIST_DEVICE=cuda timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node ${NR:-8} --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --rows ${ROWS:-10000000} \
    --steps 2 --warmup 1 --verbose > gpurun_out/bench_${NR:-8}rank.log 2>&1
rc=$?; echo "bench ${NR:-8}rank rc=$rc $(date)" >> $P
exit $rc
