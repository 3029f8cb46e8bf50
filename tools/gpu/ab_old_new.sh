#!/bin/bash
# A/B of the current tree against the session-start tree (_old), interleaved on one box
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
O=gpurun_out/ab_old_new.txt
: > $O
one() {  # label dir args
  local L=$1; shift; local D=$1; shift
  (cd $R/$D && timeout -k 10 300 python -u bench.py "$@" > $R/gpurun_out/ab_$L.log 2>&1) || return $?
  echo "$L $(tail -n 1 gpurun_out/ab_$L.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> $O
}
one warm . --rows 1250000 --steps 3 --warmup 1 || exit $?
one new10m . --steps 5 --warmup 2 || exit $?
one old10m _old --steps 5 --warmup 2 || exit $?
one new10m_b . --steps 5 --warmup 2 || exit $?
one old10m_b _old --steps 5 --warmup 2 || exit $?
one new1250k . --rows 1250000 --steps 10 --warmup 3 || exit $?
one old1250k _old --rows 1250000 --steps 10 --warmup 3 || exit $?
one new1250k_b . --rows 1250000 --steps 10 --warmup 3 || exit $?
one old1250k_b _old --rows 1250000 --steps 10 --warmup 3 || exit $?
cat $O
