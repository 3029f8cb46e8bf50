#!/bin/bash
# Per-step kernel table of ResNet-50 b256 (bf16 activations, then fp32 activations): two
# rocprofv3 runs that differ by 3 timed steps, differenced by tools/prof_diff.py.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 600 python -u -m pytest tests/test_codegen.py tests/test_act_bf16.py -x -q -m gpu \
    --timeout 200 --timeout-method thread > gpurun_out/rnp_tests.log 2>&1 || exit $?
for mode in act fp32; do
  extra=""; [ $mode = fp32 ] && extra="--fp32-activations"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnp_${mode}_a -o run --output-format csv -- \
      python3 bench_resnet50.py --batch 256 --steps 1 --warmup 1 $extra > gpurun_out/rnp_${mode}_a.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnp_${mode}_b -o run --output-format csv -- \
      python3 bench_resnet50.py --batch 256 --steps 4 --warmup 1 $extra > gpurun_out/rnp_${mode}_b.log 2>&1 || exit $?
  python3 tools/prof_diff.py gpurun_out/rnp_${mode}_a gpurun_out/rnp_${mode}_b 3 > gpurun_out/rnp_${mode}_step.txt || exit $?
  rm -rf gpurun_out/rnp_${mode}_a gpurun_out/rnp_${mode}_b
done
timeout -k 10 300 python tools/bench_conv_rn50.py --reps 3 > gpurun_out/conv_rn50.log 2>&1 || exit $?
SYSML_CONV1X1_GEMM=0 timeout -k 10 300 python tools/bench_conv_rn50.py --reps 3 --no-miopen > gpurun_out/conv_rn50_nogemm.log 2>&1
