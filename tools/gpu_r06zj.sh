# round 6, call zj: k_conv_v1p with Ah Bh and Ah Bl of an accumulator back to back (AVSE_V1P_CHAIN=1 variant) vs
# the grouped order (library); parity of the variant first
set -o pipefail
mkdir -p gpurun_out
AVSE_LIBRARY=$(pwd)/tools/_ab/libavse_chain.so timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -v -rP --timeout 300 --timeout-method thread \
  -k "packed_v1" > gpurun_out/r06zj_tests.log 2>&1 || { tail -40 gpurun_out/r06zj_tests.log; exit 1; }
grep -E "packed vs|passed|failed" gpurun_out/r06zj_tests.log
for r in 1 2 3; do
  for v in cur chain; do
    lib=""; [ $v != cur ] && lib=tools/_ab/libavse_$v.so
    AVSE_LIBRARY=$lib AVSE_DTYPE=float32_split AVSE_REPS=9 timeout -k 10 120 python -u tools/stage_times.py $v > gpurun_out/r06zj_${v}_$r.json 2> gpurun_out/r06zj_err.log || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/r06zj_${v}_$r.json').read().strip().splitlines()[-1]); st=d['stage_ms']
print(d['label'], $r, 'v_conv1', st['v_conv1'], d['total_ms'])"
  done
done
