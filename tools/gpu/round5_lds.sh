#!/bin/bash
# Round-5 LDS: conflict-free 96-B LDS pitch in conv3 / wgrad -- their tests, the conv bench,
# ResNet-50, and the bank-conflict counters of the conv kernels.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rld_progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dnn_gpu.py \
    > gpurun_out/rld_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_conv_rn50.py --no-miopen > gpurun_out/rld_conv.log 2>&1
rc=$?; echo "conv rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench_resnet50.py --batch 256 --steps 5 --warmup 2 > gpurun_out/rld_resnet.log 2>&1
rc=$?; echo "resnet rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmcl
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    -d $R/gpurun_out/pmcl/p1 -o p --output-format csv -- python3 $R/tools/pmc_conv_driver.py > $R/gpurun_out/pmcl/p1.log 2>&1
rc=$?; echo "pmc rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmcl > $R/gpurun_out/pmcl/summary.txt
echo "done $(date)" >> $P
