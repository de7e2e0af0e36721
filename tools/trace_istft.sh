#!/bin/bash
# kernel-trace of the ISTFT timing (resource columns: LDS, VGPR / AGPR, scratch per dispatch)
ROOT=$(pwd); OUT=$ROOT/gpurun_out/trist; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 $ROOT/tools/stft_time.py $ROOT/tools/_libavse_${1:-ist15b}.so > $OUT/log.txt 2>&1
f=$(find $OUT -name "*kernel_trace.csv" | head -1)
head -1 $f
grep -m 3 "k_istft_fused" $f
