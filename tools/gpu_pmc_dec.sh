#!/bin/bash
# PMC passes over the fused decoder tail kernel (k_dec_tail), one counter group per rocprofv3 run
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_dec
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
           "SQC_ICACHE_MISSES SQC_ICACHE_HITS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    AVSE_REPS=2 timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "k_dec_tail" --output-format csv -d $OUT/p$i -o pmc -- \
        python3 $ROOT/tools/fwd_loop.py > $OUT/p$i.log 2>&1 || echo "pass $i failed" >> $OUT/fail.txt
    i=$((i+1))
done
