# round 6, call m: timing ablations of the packed split v_conv1 (tools/_ab variant libraries, AVSE_V1S_ABL)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in cur vabl1 vabl2 vabl4; do
    lib=""; [ $v != cur ] && lib=tools/_ab/libavse_$v.so
    AVSE_LIBRARY=$lib AVSE_DTYPE=float32_split AVSE_REPS=9 timeout -k 10 120 python -u tools/stage_times.py $v > gpurun_out/r06m_${v}_$r.json 2> gpurun_out/r06m_err.log || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/r06m_${v}_$r.json').read().strip().splitlines()[-1]); print(d['label'], $r, d['stage_ms']['v_conv1'], d['total_ms'])"
  done
done
