#!/bin/bash
# K6 ISTFT counters over tools/stft_time.py (in-tree library): LDS bank conflicts against LDS instruction cycles,
# VALU issue, wave waits — the same two passes as tools/pmc_stft.sh, filtered to k_istft_fused afterwards
set -e
ROOT=$(pwd); OUT=$ROOT/gpurun_out/istpmc; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d $OUT/a -o pmc -- python3 $ROOT/tools/stft_time.py > $OUT/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/b -o pmc -- python3 $ROOT/tools/stft_time.py > $OUT/b.log 2>&1
echo done
