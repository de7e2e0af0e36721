# round 6, call v: timing ablations of the split-pair k_gemm (AVSE_GEMM_ABL variant libraries: 2 = no global loads,
# 4 = no MFMAs); stage_times.py profile mode: label, run, v_conv6 ms, dense ms, forward ms
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in cur gabl2 gabl4; do
    lib=""; [ $v != cur ] && lib=tools/_ab/libavse_$v.so
    AVSE_LIBRARY=$lib AVSE_DTYPE=float32_split AVSE_REPS=9 timeout -k 10 120 python -u tools/stage_times.py $v > gpurun_out/r06v_${v}_$r.json 2> gpurun_out/r06v_err.log || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/r06v_${v}_$r.json').read().strip().splitlines()[-1]); st=d['stage_ms']
print(d['label'], $r, st['v_conv6'], round(st['enc_dense']+st['dec_dense1']+st['dec_dense2'],4), d['total_ms'])"
  done
done
