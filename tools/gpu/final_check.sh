#!/bin/bash
# Round check: full GPU suite, smoke, headline bench (default config), per-step headline kernel
# table, 1.25M-row headline, ResNet-50 b256.  Each step under its own limit; stops at a failure.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread \
    > gpurun_out/fc_tests.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fc_smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/fc_bench.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --rows 1250000 --steps 10 --warmup 3 > gpurun_out/fc_bench_1250k.log 2>&1 || exit $?
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/fc_resnet.log 2>&1
