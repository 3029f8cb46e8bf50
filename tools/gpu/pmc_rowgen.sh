#!/bin/bash
# PMC counter passes over the generated Row-template kernels (tools/bench_rowgen.py, fp32 and
# bf16 at 1M x 1000); one counter group per run
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmc_row
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU"
P2="FETCH_SIZE GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $R/gpurun_out/pmc_row/p$i -o p --output-format csv -- \
      python3 $R/tools/bench_rowgen.py --rows 1000000 --reps 2 > $R/gpurun_out/pmc_row/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_row > $R/gpurun_out/pmc_row/summary.txt
