#!/bin/bash
# One GPU call: the -m gpu suite, the default bench, the end-to-end bench, then (optionally) the rocprof recipe.
# Each step has its own time limit; a test FAILURE (exit 1) still lets the bench run, anything else (fault, abort,
# timeout) ends the call.
TAG=${1:-r02}
OUT=gpurun_out
mkdir -p $OUT
# -rP: every passing test's captured output (the measured errors each tolerance is set against) stays in the log
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread > $OUT/gputest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit $?
echo bench ok
timeout -k 10 300 python bench.py --e2e --steps 5 --warmup 2 > $OUT/bench_e2e_$TAG.json 2> $OUT/bench_e2e_$TAG.err || exit $?
echo e2e ok
if [ "$2" = "prof" ]; then bash tools/profile.sh $TAG || exit $?; fi
tail -3 $OUT/gputest_$TAG.log
