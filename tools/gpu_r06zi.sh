# round 6, call zi: split-pair k_gemm with the Wh MFMAs of every accumulator before the Wl ones (library) vs the two
# MFMAs of an accumulator back to back (AVSE_GEMM_PAIRED=1 variant)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -v -rP --timeout 300 --timeout-method thread \
  -k "gemm_matches" > gpurun_out/r06zi_tests.log 2>&1 || { tail -40 gpurun_out/r06zi_tests.log; exit 1; }
grep -E "k_gemm vs|passed|failed" gpurun_out/r06zi_tests.log
for r in 1 2 3; do
  for v in cur gpair; do
    lib=""; [ $v != cur ] && lib=tools/_ab/libavse_$v.so
    AVSE_LIBRARY=$lib AVSE_DTYPE=float32_split AVSE_REPS=9 timeout -k 10 120 python -u tools/stage_times.py $v > gpurun_out/r06zi_${v}_$r.json 2> gpurun_out/r06zi_err.log || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/r06zi_${v}_$r.json').read().strip().splitlines()[-1]); st=d['stage_ms']
print(d['label'], $r, 'v_conv6', st['v_conv6'], 'dense', round(st['enc_dense']+st['dec_dense1']+st['dec_dense2'],4), d['total_ms'])"
  done
done
