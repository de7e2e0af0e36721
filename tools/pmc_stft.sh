#!/bin/bash
# K1 diagnostics on the GPU box: per-step s_memtime stamps (variant library tools/_libavse_sstamp.so), a kernel-trace
# stats pass and two PMC passes over tools/stft_only.py (in-tree library).
set -e
ROOT=$(pwd); OUT=$ROOT/gpurun_out/stftpmc; mkdir -p $OUT
timeout -k 10 120 python tools/stft_stamps.py tools/_libavse_sstamp.so > $OUT/stamps.log 2>&1
cat $OUT/stamps.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 $ROOT/tools/stft_only.py 20 > $OUT/trace.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d $OUT/a -o pmc -- python3 $ROOT/tools/stft_only.py 5 > $OUT/a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/b -o pmc -- python3 $ROOT/tools/stft_only.py 5 > $OUT/b.log 2>&1
echo done
