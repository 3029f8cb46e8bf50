#!/bin/bash
# Round-5 T: sparse GPU tests (counting-sort CSR transpose, dot), ATen call sites of ALS-CG (1M x 1M) and of the headline at icpt=2 (1M rows), and the
# icpt=2 kernel profile.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rt_progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_sparse_gpu.py \
    tests/test_quaternary.py > gpurun_out/rt_sparse.log 2>&1
rc=$?; echo "sparse tests rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench_als.py --rows 10000000 --cols 10000000 --per-row 100 --maxi 2 --steps 1 --warmup 1 \
    > gpurun_out/rt_als_10m.log 2>&1
rc=$?; echo "als 10m rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/probe/aten_modes.py --target bench_als --top 40 --steps 1 --warmup 1 \
    > gpurun_out/rt_als_aten.log 2>&1
rc=$?; echo "als aten rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/probe/aten_modes.py --target bench --top 40 --rows 1000000 --icpt 2 --steps 2 \
    --warmup 1 > gpurun_out/rt_icpt_aten.log 2>&1
rc=$?; echo "icpt aten rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --icpt 2 --steps 3 --warmup 2 > gpurun_out/rt_icpt2.log 2>&1
rc=$?; echo "icpt2 rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 > gpurun_out/rt_icpt0.log 2>&1
rc=$?; echo "icpt0 rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rtq_a -o run --output-format csv -- \
    python3 bench.py --icpt 2 --steps 1 --warmup 2 > gpurun_out/rtq_a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rtq_b -o run --output-format csv -- \
    python3 bench.py --icpt 2 --steps 3 --warmup 2 > gpurun_out/rtq_b.log 2>&1 || exit $?
python3 tools/prof_diff.py gpurun_out/rtq_a gpurun_out/rtq_b 2 > gpurun_out/rt_icpt2_step.txt
rm -rf gpurun_out/rtq_a gpurun_out/rtq_b
echo "done $(date)" >> $P
