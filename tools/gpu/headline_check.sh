#!/bin/bash
# Headline path check: run-ahead / forced-DIST GPU tests, then the headline at 10M rows
# (default), at the 8-GPU per-rank size (1.25M rows, default depth and depth 3), the icpt = 2
# variant, and the forced one-rank RCCL SPMD plan (SYSML_DIST_FORCE=1) at both sizes.  One line
# each (ms/step, parallelism), collected in gpurun_out/headline_check.txt.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
O=gpurun_out/headline_check.txt
: > $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_runahead.py tests/test_dist_rccl_gpu.py -m gpu > gpurun_out/hc_tests.log 2>&1 || exit $?
run() {   # label, env, args
  local L=$1; shift
  local E=$1; shift
  env $E timeout -k 10 300 python -u bench.py "$@" > gpurun_out/hc_$L.log 2>&1 || return $?
  echo "$L $(tail -1 gpurun_out/hc_$L.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["parallelism"])')" >> $O
}
run base10m "X=1" --steps 5 --warmup 2 || exit $?
run r1250k "X=1" --rows 1250000 --steps 10 --warmup 3 || exit $?
run r1250k_d3 "SYSML_RUNAHEAD_DEPTH=3" --rows 1250000 --steps 10 --warmup 3 || exit $?
run icpt2_10m "X=1" --icpt 2 --steps 5 --warmup 2 || exit $?
run dist10m "SYSML_DIST_FORCE=1" --steps 5 --warmup 2 || exit $?
run dist1250k "SYSML_DIST_FORCE=1" --rows 1250000 --steps 10 --warmup 3 || exit $?
cat $O
