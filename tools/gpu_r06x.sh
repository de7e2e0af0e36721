# round 6, call x: split a_conv1 on the vector ALUs, a pixel x 64 channels per thread parity and A/B against audio_prep + k_conv
# (AVSE_NO_A1VALU=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -v -rP --timeout 300 --timeout-method thread \
  -k "valu_aconv1 or bench_batch or zero_video or forward_matches or other_frame" > gpurun_out/r06x_tests.log 2>&1 || { tail -40 gpurun_out/r06x_tests.log; exit 1; }
grep -E "VALU vs|passed|failed" gpurun_out/r06x_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_range.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06x_range.log 2>&1 || { tail -30 gpurun_out/r06x_range.log; exit 1; }
tail -1 gpurun_out/r06x_range.log
for r in 1 2; do
  for v in 1 0; do
    AVSE_NO_A1VALU=$v timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline --steps 40 --warmup 5 > gpurun_out/r06x_bench.json 2>> gpurun_out/r06x_bench.err || exit $?
    python -c "
import json
d=json.loads(open('gpurun_out/r06x_bench.json').read().strip().splitlines()[-1])
st=d.get('breakdown', {}).get('stage_ms', {})
print('no_a1valu=$v r$r', d['value'], d['ms_per_step'], d['window_ms_per_step']['median'], 'audio_prep', st.get('audio_prep'), 'a_conv1', st.get('a_conv1'))
"
  done
done
