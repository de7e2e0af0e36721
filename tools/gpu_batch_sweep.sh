#!/bin/bash
# Per-clip stage times of the bf16 step at several batch sizes (Infinity-Cache residency of the layer-to-layer
# activations: v_conv1's output is 1 MB per clip, 128 clips = 134 MB fits the 256 MiB L3, 512 clips do not).
set -e
mkdir -p gpurun_out
for b in ${BATCHES:-128 512 128 512}; do
  timeout -k 10 240 python bench.py --batch $b --steps 100 --warmup 20 --no-legs --no-cpu-baseline > gpurun_out/bs_$b.json 2> gpurun_out/bs_$b.err
  python3 -c "
import json; d=json.loads(open('gpurun_out/bs_$b.json').read().strip().splitlines()[-1]); st=d['breakdown']['stage_ms']
print('batch $b', 'us/clip step', round(1e3*d['ms_per_step']/$b, 4), {k: round(1e3*st[k]/$b, 4) for k in ('v_conv1','v_conv2','v_conv3','v_conv4','d_deconv1','d_deconv4','audio_prep')})"
done
