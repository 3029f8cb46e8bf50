#!/bin/bash
# Round-5 W: the whole GPU test suite, smoke(), the headline at 10M and 1.25M rows (host profile
# with the callers of the blocking reads), ALS-CG 10M.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rw_progress.txt
echo "start $(date)" > $P
timeout -k 10 1200 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/rw_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/rw_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/rw_bench_default.log 2>&1
rc=$?; echo "bench default rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 10 --warmup 3 > gpurun_out/rw_1250k.log 2>&1
rc=$?; echo "1250k rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 5 --warmup 3 --host-profile gpurun_out/rw_host_1250k.txt \
    > gpurun_out/rw_1250k_prof.log 2>&1
rc=$?; echo "1250k prof rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench_als.py --rows 10000000 --cols 10000000 --per-row 100 --maxi 2 --steps 1 --warmup 1 \
    > gpurun_out/rw_als_10m.log 2>&1
rc=$?; echo "als rc=$rc $(date)" >> $P
echo "done $(date)" >> $P
