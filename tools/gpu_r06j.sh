# round 6, call j: where the split forward's side-stream audio branch forks (AVSE_AUD_FORK = video layers before it)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in 0 1 2 3; do
    AVSE_AUD_FORK=$v timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline --steps 40 --warmup 5 > gpurun_out/r06j_bench.json 2>> gpurun_out/r06j_bench.err || exit $?
    python -c "
import json
d=json.loads(open('gpurun_out/r06j_bench.json').read().strip().splitlines()[-1])
print('aud_fork=$v r$r', d['value'], d['ms_per_step'], d['window_ms_per_step']['median'])
"
  done
done
