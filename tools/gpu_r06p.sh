# round 6, call p: k_conv_v1p with the two compute waves of a SIMD taking turns on the epilogue (library) vs both after
# their MFMAs (AVSE_V1P_STAGGER=0 variant), k_conv_v1s for scale; parity of the packed path first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v -rP --timeout 200 --timeout-method thread \
  -k "packed_v1 or bench_batch" > gpurun_out/r06p_tests.log 2>&1 || { tail -30 gpurun_out/r06p_tests.log; exit 1; }
grep -E "packed vs|passed|failed" gpurun_out/r06p_tests.log
for r in 1 2 3; do
  for v in cur nostag v1s; do
    lib=""; [ $v = nostag ] && lib=tools/_ab/libavse_nostag.so
    nv=0; [ $v = v1s ] && nv=1
    AVSE_NO_V1P=$nv AVSE_LIBRARY=$lib AVSE_DTYPE=float32_split AVSE_REPS=9 timeout -k 10 120 python -u tools/stage_times.py $v > gpurun_out/r06p_${v}_$r.json 2> gpurun_out/r06p_err.log || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/r06p_${v}_$r.json').read().strip().splitlines()[-1]); print(d['label'], $r, d['stage_ms']['v_conv1'], d['total_ms'])"
  done
done
