#!/bin/bash
# Kernel trace of the forward at a small batch (default 8): per-kernel durations and launch gaps
#   bash tools/trace_b8.sh [B] [tag]
set -e
B=${1:-8}
TAG=${2:-b$B}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/trace_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
AVSE_B=$B AVSE_REPS=20 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT -o tr -- \
    python3 $ROOT/tools/fwd_loop.py > $OUT/run.log 2>&1
cd $ROOT && python3 tools/trace_gaps.py $OUT > $OUT/gaps.txt
