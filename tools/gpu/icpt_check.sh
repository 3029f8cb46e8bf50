#!/bin/bash
# Intercept path: GPU tests of the padded cbind(X, 1) copy, then the headline at icpt 0 / 1 / 2.
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_intercept_gpu.py tests/test_vector_template.py tests/test_resnet_plan.py -q -m gpu \
    --timeout 300 --timeout-method thread > gpurun_out/ic_tests.log 2>&1 || exit $?
for ic in 1 2 0; do
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --icpt $ic > gpurun_out/icpt_$ic.json 2> gpurun_out/icpt_$ic.log || exit $?
done
