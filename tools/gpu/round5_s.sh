#!/bin/bash
# Round-5 S: ATen call sites of ALS-CG (1M x 1M) and of the headline at icpt=2 (1M rows), and the
# icpt=2 kernel profile.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rs_progress.txt
echo "start $(date)" > $P
timeout -k 10 300 python -u tools/probe/aten_modes.py --target bench_als --top 40 --steps 1 --warmup 1 \
    > gpurun_out/rs_als_aten.log 2>&1
rc=$?; echo "als aten rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/probe/aten_modes.py --target bench --top 40 --rows 1000000 --icpt 2 --steps 2 \
    --warmup 1 > gpurun_out/rs_icpt_aten.log 2>&1
rc=$?; echo "icpt aten rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --icpt 2 --steps 3 --warmup 2 > gpurun_out/rs_icpt2.log 2>&1
rc=$?; echo "icpt2 rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 > gpurun_out/rs_icpt0.log 2>&1
rc=$?; echo "icpt0 rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rsq_a -o run --output-format csv -- \
    python3 bench.py --icpt 2 --steps 1 --warmup 2 > gpurun_out/rsq_a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rsq_b -o run --output-format csv -- \
    python3 bench.py --icpt 2 --steps 3 --warmup 2 > gpurun_out/rsq_b.log 2>&1 || exit $?
python3 tools/prof_diff.py gpurun_out/rsq_a gpurun_out/rsq_b 2 > gpurun_out/rs_icpt2_step.txt
rm -rf gpurun_out/rsq_a gpurun_out/rsq_b
echo "done $(date)" >> $P
