#!/bin/bash
# Headline at 1.25M rows (host event trace) and at 10M rows.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
SYSML_HOSTTRACE=1 timeout -k 10 300 python -u bench.py --rows 1250000 --steps 5 --warmup 2 > gpurun_out/bp_1250k.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bp_10m.log 2>&1 || exit $?
