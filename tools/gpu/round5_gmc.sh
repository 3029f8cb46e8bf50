#!/bin/bash
# Round-5 GMC: host-placement threshold sweep (small matrices on the host below it) at 1.25M and 10M rows.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
for g in 16384 0 4096 65536 262144; do
  timeout -k 10 300 python -u bench.py --rows 1250000 --steps 10 --warmup 3 --gpu-min-cells $g > gpurun_out/rg_1250k_$g.log 2>&1 || exit $?
done
for g in 16384 65536; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --gpu-min-cells $g > gpurun_out/rg_10m_$g.log 2>&1 || exit $?
done
