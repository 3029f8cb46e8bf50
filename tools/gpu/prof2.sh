#!/bin/bash
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof2 -o bench --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 > $R/gpurun_out/prof2_bench.log 2>&1
echo "prof rc=$?" > $R/gpurun_out/progress5.txt
