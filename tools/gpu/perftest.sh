#!/bin/bash
# Perftest suite on the GPU box: one family per step, each under its own time limit;
# JSON lines accumulate in gpurun_out/perftest_<size>.jsonl.   usage: tools/gpu/perftest.sh SIZE FAMILIES...
R=$GRAFT_REPO_ROOT
SIZE=$1; shift
mkdir -p $R/gpurun_out
for F in "$@"; do
  timeout -k 10 ${PT_LIMIT:-240} python3 -m systemml_amd.perftest --dir /tmp/perftest_data --sizes $SIZE \
      --families $F --out $R/gpurun_out/perftest_$SIZE.jsonl >> $R/gpurun_out/perftest_$SIZE.log 2>&1
  rc=$?
  echo "family $F rc=$rc" >> $R/gpurun_out/perftest_$SIZE.log
  if [ $rc -ge 124 ]; then exit $rc; fi
done
