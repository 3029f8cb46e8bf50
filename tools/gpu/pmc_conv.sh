#!/bin/bash
# PMC counter passes over the ResNet-50 convolution kernels (tools/pmc_conv_driver.py): one pass per run
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmcc
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
P2="FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
P3="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $P -d $R/gpurun_out/pmcc/p$i -o p --output-format csv -- python3 $R/tools/pmc_conv_driver.py > $R/gpurun_out/pmcc/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmcc > $R/gpurun_out/pmcc/summary.txt
