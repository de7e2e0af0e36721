#!/bin/bash
# Whole-step A/B of the stream convolutions' 32x32x16 compute waves (AVSE_MFMA32=1) against the default 16x16x32,
# alternated twice on one box (bench.py without legs / CPU baseline).
set -e
mkdir -p gpurun_out
for i in 1 2; do
  for m in 0 1; do
    AVSE_MFMA32=$m timeout -k 10 240 python bench.py --steps 200 --warmup 20 --no-legs --no-cpu-baseline > gpurun_out/m32_${m}_$i.json 2> gpurun_out/m32_${m}_$i.err
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/m32_${m}_$i.json').read().strip().splitlines()[-1]); st=d['breakdown']['stage_ms']; print('mfma32=$m run $i', d['ms_per_step'], {k: st[k] for k in ('v_conv2','v_conv3','v_conv4','v_conv5')})"
  done
done
