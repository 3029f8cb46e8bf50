#!/bin/bash
# Full round check: GPU tests, smoke, headline bench, 2-rank SPMD rehearsal on one GPU (gloo
# transport, both ranks on cuda:0), ResNet-50 bench.  Stops at the first failure.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=gpurun_out/full_progress.txt
echo "start $(date)" > $P
timeout -k 10 700 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
SYSML_DIST_BACKEND=gloo SYSML_DIST_DEVICE=cuda timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --rows 2000000 --steps 3 \
    --warmup 1 --verbose > gpurun_out/bench_2rank.log 2>&1
rc=$?; echo "bench 2rank rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench_resnet50.py --steps 5 --warmup 2 > gpurun_out/resnet.log 2>&1
rc=$?; echo "resnet rc=$rc $(date)" >> $P
exit $rc
