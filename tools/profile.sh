#!/bin/bash
# Round profiling recipe (run on the GPU box from the repo root):
#   bash tools/profile.sh r01
# 1. rocprofv3 --kernel-trace --stats of the bench command          -> gpurun_out/prof_<tag>/
# 2. two separate PMC passes (FETCH_SIZE, WRITE_SIZE: they do not fit one TCC pass) over the
#    dominant kernel (v_conv2 = k_conv_stream<5,16,16,1,...>) at the bench shape
# 3. tools/pmc_summary.py turns them into profiles/<tag>_*.{csv,json}
set -e
TAG=${1:-r01}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
    python3 $ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_${TAG}_bench.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_conv_stream<5, 16, 16, 1" --output-format csv \
    -d $OUT/pmc_${TAG}_fetch -o pmc -- python3 $ROOT/tools/fwd_loop.py > $OUT/pmc_${TAG}_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_conv_stream<5, 16, 16, 1" --output-format csv \
    -d $OUT/pmc_${TAG}_write -o pmc -- python3 $ROOT/tools/fwd_loop.py > $OUT/pmc_${TAG}_write.log 2>&1
cd $ROOT
python3 tools/pmc_summary.py $TAG
