# round 6, call o: packed split v_conv1 epilogue stores, dword channel pairs (library) vs 2-byte pieces (AVSE_V1P_B16
# variant), and k_conv_v1s (AVSE_NO_V1P=1), alternated on one box
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in cur b16 v1s; do
    lib=""; [ $v = b16 ] && lib=tools/_ab/libavse_b16.so
    nv=0; [ $v = v1s ] && nv=1
    AVSE_NO_V1P=$nv AVSE_LIBRARY=$lib AVSE_DTYPE=float32_split AVSE_REPS=9 timeout -k 10 120 python -u tools/stage_times.py $v > gpurun_out/r06o_${v}_$r.json 2> gpurun_out/r06o_err.log || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/r06o_${v}_$r.json').read().strip().splitlines()[-1]); print(d['label'], $r, d['stage_ms']['v_conv1'], d['total_ms'])"
  done
done
