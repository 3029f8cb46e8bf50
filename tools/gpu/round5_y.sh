#!/bin/bash
# Round-5 Y: ATen call sites (new device memory or in-place writes) of the icpt=2 headline at 10M.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/probe/aten_modes.py --target bench --top 40 --icpt 2 --steps 1 --warmup 1 \
    > gpurun_out/ry_icpt_aten.log 2>&1
echo "rc=$?" >> gpurun_out/ry_icpt_aten.log
