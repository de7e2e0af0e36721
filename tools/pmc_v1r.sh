#!/bin/bash
# PMC passes over the v_conv1 harness (full variant and compute-only variant)
set -e
ROOT=$(pwd); OUT=$ROOT/gpurun_out/v1pmc; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for mode in full compute; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/${mode}_a -o pmc -- $ROOT/tools/_v1r_ablate $mode > $OUT/${mode}_a.log 2>&1
  timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d $OUT/${mode}_b -o pmc -- $ROOT/tools/_v1r_ablate $mode > $OUT/${mode}_b.log 2>&1
done
