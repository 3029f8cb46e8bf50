#!/bin/bash
# Headline parity and intercept sweep: one verbose step with X stored bf16 and fp64 (solver
# iteration logs on stderr), then timed runs with icpt 0 / 1 / 2.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --verbose > gpurun_out/par_bf16.json 2> gpurun_out/par_bf16.log || exit $?
timeout -k 10 600 python bench.py --steps 1 --warmup 0 --verbose --xdtype fp64 > gpurun_out/par_fp64.json 2> gpurun_out/par_fp64.log || exit $?
for ic in 0 1 2; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --icpt $ic > gpurun_out/icpt_$ic.json 2> gpurun_out/icpt_$ic.log || exit $?
done
