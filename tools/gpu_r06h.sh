# round 6, call h: kernel trace of the default bench step (per-kernel durations and gaps of one forward)
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; rm -rf $OUT/trace_r06h
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_r06h -o run -- \
    python3 $ROOT/bench.py --steps 10 --warmup 3 --no-legs --no-cpu-baseline --profile-reps 1 > $OUT/trace_r06h.log 2>&1 || exit $?
cd $ROOT && ls -R gpurun_out/trace_r06h | head
