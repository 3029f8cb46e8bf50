#!/bin/bash
# Per-step kernel statistics of bench.py: profile 1 and 3 timed steps (same warmup) and
# difference the two kernel-stat tables (tools/prof_diff.py) so data generation and the
# warmup step cancel out.   usage: tools/gpu/prof_step.sh [extra bench.py args]
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
for S in 1 3; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pstep$S -o run --output-format csv -- \
    python3 $R/bench.py --steps $S --warmup 1 "$@" > $R/gpurun_out/pstep$S.log 2>&1 || exit $?
  echo "profiled steps=$S" >> $R/gpurun_out/pstep_progress.txt
done
python3 $R/tools/prof_diff.py $R/gpurun_out/pstep1 $R/gpurun_out/pstep3 2 > $R/gpurun_out/per_step_kernels.txt
