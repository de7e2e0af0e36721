# round 6, call z: audio side-stream priority re-check on the round-6 kernels (AVSE_SIDE_PRIO 0 default, 2 greatest),
# alternated three times on one box; bench.py --no-legs 60 steps
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in 0 2; do
    AVSE_SIDE_PRIO=$v timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline --steps 60 --warmup 5 > gpurun_out/r06z_bench.json 2>> gpurun_out/r06z_bench.err || exit $?
    python -c "
import json
d=json.loads(open('gpurun_out/r06z_bench.json').read().strip().splitlines()[-1])
print('side_prio=$v r$r', d['value'], d['ms_per_step'], d['window_ms_per_step']['median'])
"
  done
done
