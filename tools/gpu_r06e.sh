# round 6, call e: split tail, three products per MAC (P3, in-tree) vs four (tools/_ab/libavse_p4.so)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -rP --timeout 240 --timeout-method thread tests/test_gpu_split.py -k "fused_tail or intermediates or 37" > gpurun_out/r06e_tests.log 2>&1; rc=$?; grep -E "fused tail|split N=37|passed|failed" gpurun_out/r06e_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for v in cur p4; do
    lib=""; [ $v != cur ] && lib=tools/_ab/libavse_$v.so
    AVSE_LIBRARY=$lib AVSE_DTYPE=float32_split AVSE_REPS=9 timeout -k 10 120 python -u tools/stage_times.py $v > gpurun_out/r06e_st.json 2> gpurun_out/r06e_err.log || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/r06e_st.json').read().strip().splitlines()[-1]); print(d['label'], $r, d['stage_ms']['d_deconv4'], d['total_ms'])"
  done
done
