# round 6, call g: does the side-stream audio branch overlap the video encoder?  default vs AVSE_SERIAL=1
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 0 1; do
  AVSE_SERIAL=$v timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline --steps 60 --warmup 5 > gpurun_out/r06g_bench_$v.json 2>> gpurun_out/r06g_bench.err || exit $?
  python -c "
import json
d=json.loads(open('gpurun_out/r06g_bench_$v.json').read().strip().splitlines()[-1])
print('serial=$v', d['value'], d['ms_per_step'], d['window_ms_per_step'])
"
done
