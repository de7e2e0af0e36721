#!/bin/bash
# Kernel-trace a short bench run: the timed steps launch back to back (rocprof shows no idle between kernels); the
# profiled breakdown (forward_profile) records an event between kernels, which shows as ~5.7 us gaps
ROOT=$(pwd); OUT=$ROOT/gpurun_out/gaps; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/direct -o run -- python3 $ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-legs > $OUT/direct.log 2>&1
