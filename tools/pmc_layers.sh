#!/bin/bash
# PMC passes over the generic k_conv launches of the bf16 forward (B=512), one counter group per pass
# (separate rocprofv3 runs, no traces combined):  bash tools/pmc_layers.sh <regex> <tag>
set -e
RX=${1:-k_conv<}
TAG=${2:-layers}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmcl_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" "TA_BUSY_avr SQ_INSTS_VMEM_RD"; do
    timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "$RX" --output-format csv -d $OUT/p$i -o pmc -- \
        python3 $ROOT/tools/fwd_loop.py > $OUT/p$i.log 2>&1
    i=$((i+1))
done
