#!/bin/bash
# Diagnostics: B=512 kernel trace of the concurrent forward (launch gaps), LDS / issue counters of the
# decoder-shaped conv kernels (k_conv and k_conv_win), one counter group per rocprofv3 pass
set -e
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/diag
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
AVSE_B=512 AVSE_REPS=5 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o tr -- \
    python3 $ROOT/tools/fwd_loop.py > $OUT/tr.log 2>&1
python3 $ROOT/tools/trace_gaps.py $OUT/tr > $OUT/gaps.txt
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "FETCH_SIZE"; do
    AVSE_REPS=3 timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_conv" --output-format csv -d $OUT/p$i -o pmc -- \
        python3 $ROOT/tools/fwd_loop.py > $OUT/p$i.log 2>&1
    i=$((i+1))
done
cd $ROOT && python3 tools/pmc_layer_summary.py $OUT > $OUT/pmc.txt
