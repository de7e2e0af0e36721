#!/bin/bash
# Per-stage times under several environment settings: ENVS="A=1 B=2|C=3" (configurations separated by |)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/envab.log; : > $O
IFS='|' read -ra CFGS <<< "$ENVS"
for c in "${CFGS[@]}"; do
  env $c AVSE_REPS=${REPS:-5} timeout -k 10 120 python tools/stage_times.py "$c" >> $O 2>/dev/null || exit 1
done
