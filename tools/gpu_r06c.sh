# round 6, call c: timing ablations of the split decoder tail (tools/_ab variant libraries; stage d_deconv4 = the tail)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in cur abl1 abl2 abl4; do
    lib=""; [ $v != cur ] && lib=tools/_ab/libavse_$v.so
    AVSE_LIBRARY=$lib AVSE_DTYPE=float32_split AVSE_REPS=9 timeout -k 10 120 python -u tools/stage_times.py $v > gpurun_out/r06c_$v_$r.json 2> gpurun_out/r06c_err.log || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/r06c_$v_$r.json').read().strip().splitlines()[-1]); print(d['label'], $r, d['stage_ms']['d_deconv4'], d['total_ms'])"
  done
done
