#!/bin/bash
# Whole-step A/B: bench.py under several environment settings (ENVS="A=1|B=2"), plus a kernel trace of the
# default configuration's concurrent forward
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/step_ab.log; : > $O
IFS='|' read -ra CFGS <<< "$ENVS"
for c in "${CFGS[@]}"; do
  echo "== $c" >> $O
  env $c timeout -k 10 180 python bench.py --steps 30 --warmup 5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" >> $O || exit 1
done
if [ -n "$TRACE" ]; then
  ROOT=$(pwd); OUT=$ROOT/gpurun_out/trace_step; mkdir -p $OUT
  cd /tmp && export TMPDIR=/tmp
  AVSE_B=512 AVSE_REPS=5 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT -o tr -- python3 $ROOT/tools/fwd_loop.py > $OUT/run.log 2>&1 || exit 1
  cd $ROOT && python3 tools/trace_timeline.py $OUT 1 > $OUT/timeline.txt
fi
