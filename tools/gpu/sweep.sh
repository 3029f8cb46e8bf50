#!/bin/bash
# Generic A/B sweep of one benchmark over environment / argument variants, back to back on one
# box (replaces the round's one-off A/B scripts).  Each variant is "label|ENV=V ...|args";
# the benchmark script and its common arguments come first:
#
#   bash tools/gpu/sweep.sh bench.py "--rows 1250000 --steps 10 --warmup 3" \
#       "d1|SYSML_RUNAHEAD_DEPTH=1|" "d3|SYSML_RUNAHEAD_DEPTH=3|" "gmc0||--gpu-min-cells 0"
#
# Every run is under its own time limit; the sweep stops at the first failure.  The last JSON
# line of each run is collected in gpurun_out/sweep.txt as "label: {...}".
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
SCRIPT=$1; shift
COMMON=$1; shift
: > gpurun_out/sweep.txt
for v in "$@"; do
  L=${v%%|*}; rest=${v#*|}; E=${rest%%|*}; A=${rest#*|}
  env X_SWEEP=1 $E timeout -k 10 ${SWEEP_LIMIT:-400} python -u $SCRIPT $COMMON $A > gpurun_out/sweep_$L.log 2>&1 || exit $?
  echo "$L: $(grep '^{' gpurun_out/sweep_$L.log | tail -1)" >> gpurun_out/sweep.txt
done
cat gpurun_out/sweep.txt
