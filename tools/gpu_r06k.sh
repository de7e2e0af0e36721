# round 6, call k: priority of the split forward's side-stream audio branch (AVSE_SIDE_PRIO 0 default, 1 least, 2 greatest)
set -o pipefail
mkdir -p gpurun_out
python -c "
import ctypes; h=ctypes.CDLL('libamdhip64.so'); a=ctypes.c_int(); b=ctypes.c_int()
print('priority range rc', h.hipDeviceGetStreamPriorityRange(ctypes.byref(a), ctypes.byref(b)), 'least', a.value, 'greatest', b.value)
" || exit $?
for r in 1 2; do
  for v in 0 1 2; do
    AVSE_SIDE_PRIO=$v timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline --steps 40 --warmup 5 > gpurun_out/r06k_bench.json 2>> gpurun_out/r06k_bench.err || exit $?
    python -c "
import json
d=json.loads(open('gpurun_out/r06k_bench.json').read().strip().splitlines()[-1])
print('side_prio=$v r$r', d['value'], d['ms_per_step'], d['window_ms_per_step']['median'])
"
  done
done
