#!/bin/bash
# Round-5 PF: parfor against the sequential loop on one GPU for GEMM bodies that do not fill the
# chip on their own (n = 512 / 1024 / 2048), 4 workers (one stream each).
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
for n in 512 1024 2048; do
  timeout -k 10 200 python -u tools/bench_parfor.py --n $n --iters 16 --par 4 --reps 5 >> gpurun_out/rpf.log 2>&1 || exit $?
done
timeout -k 10 200 python -u tools/bench_parfor.py --n 1024 --iters 16 --par 8 --reps 5 >> gpurun_out/rpf.log 2>&1
