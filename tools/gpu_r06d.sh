# round 6, call d: split tail with late window-piece stores: stage times + tail tests
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  AVSE_DTYPE=float32_split AVSE_REPS=9 timeout -k 10 120 python -u tools/stage_times.py late_pieces > gpurun_out/r06d_st_$r.json 2> gpurun_out/r06d_err.log || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/r06d_st_$r.json').read().strip().splitlines()[-1]); print(d['label'], $r, d['stage_ms']['d_deconv4'], d['total_ms'])"
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_split.py -k "fused_tail or intermediates" > gpurun_out/r06d_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r06d_tests.log; exit $rc
