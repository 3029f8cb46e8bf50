#!/bin/bash
# Round-5 last: the whole GPU suite, smoke() and the default bench on the final tree.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rl_progress.txt
echo "start $(date)" > $P
timeout -k 10 1200 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/rl_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/rl_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/rl_bench.log 2>&1
rc=$?; echo "bench rc=$rc $(date)" >> $P
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/rl_resnet.log 2>&1
rc=$?; echo "resnet rc=$rc $(date)" >> $P
echo "done $(date)" >> $P
