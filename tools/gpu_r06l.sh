# round 6, call l: packed split v_conv1 (k_conv_v1p, K 128) parity and A/B against k_conv_v1s (AVSE_NO_V1P=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -v -rP --timeout 300 --timeout-method thread \
  -k "packed_v1 or bench_batch or other_frame or forward_matches or small_act" > gpurun_out/r06l_tests.log 2>&1 || { tail -30 gpurun_out/r06l_tests.log; exit 1; }
grep -E "packed vs|passed|failed" gpurun_out/r06l_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_range.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06l_range.log 2>&1 || { tail -30 gpurun_out/r06l_range.log; exit 1; }
tail -1 gpurun_out/r06l_range.log
for r in 1 2; do
  for v in 1 0; do
    AVSE_NO_V1P=$v timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline --steps 40 --warmup 5 > gpurun_out/r06l_bench.json 2>> gpurun_out/r06l_bench.err || exit $?
    python -c "
import json
d=json.loads(open('gpurun_out/r06l_bench.json').read().strip().splitlines()[-1])
print('no_v1p=$v r$r', d['value'], d['ms_per_step'], d['window_ms_per_step']['median'], 'v_conv1', d.get('breakdown', {}).get('stage_ms', {}).get('v_conv1'))
"
  done
done
