#!/bin/bash
# Round-5 H: ATen call sites of the icpt=2 headline (thread compiler: no spawned child), the
# icpt=2 10M bench, and the DNN GEMM split-K fill threshold sweep.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
P=$R/gpurun_out/rh_progress.txt
echo "start $(date)" > $P
timeout -k 10 400 python -u tools/probe/aten_sites.py --target bench --rows 2000000 --steps 2 --warmup 1 --icpt 2 \
    --compiler thread > gpurun_out/rh_aten_icpt2.txt 2>&1
rc=$?; echo "aten rc=$rc $(date)" >> $P; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --icpt 2 > gpurun_out/rh_icpt2.log 2>&1
rc=$?; echo "icpt2 rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
for f in 240 480 720; do
  SYSML_GEMM_DNN_FILL=$f timeout -k 10 300 python -u tools/bench_gemm_dnn.py > gpurun_out/rh_gemm_fill$f.txt 2>&1
  rc=$?; echo "gemm fill=$f rc=$rc $(date)" >> $P; [ $rc -ne 0 ] && exit $rc
done
echo "done $(date)" >> $P
