#!/bin/bash
# ResNet-50 iteration (tests, conv shapes, per-step profile, bench) then the headline per-step
# kernel table.
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu/rn_iter3.sh || exit $?
bash tools/gpu/prof_step.sh
