# round 6, call zh: split decoder tail with the Wh MFMAs of every fragment before the Wl ones (library) vs the two
# MFMAs of a fragment back to back (AVSE_DECTS_PAIRED=1 variant); tail parity first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -v -rP --timeout 300 --timeout-method thread \
  -k "fused_tail or bench_batch" > gpurun_out/r06zh_tests.log 2>&1 || { tail -40 gpurun_out/r06zh_tests.log; exit 1; }
grep -E "fused tail vs|passed|failed" gpurun_out/r06zh_tests.log
for r in 1 2 3; do
  for v in cur paired; do
    lib=""; [ $v != cur ] && lib=tools/_ab/libavse_$v.so
    AVSE_LIBRARY=$lib AVSE_DTYPE=float32_split AVSE_REPS=9 timeout -k 10 120 python -u tools/stage_times.py $v > gpurun_out/r06zh_${v}_$r.json 2> gpurun_out/r06zh_err.log || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/r06zh_${v}_$r.json').read().strip().splitlines()[-1]); st=d['stage_ms']
print(d['label'], $r, 'tail', st['d_deconv4'], d['total_ms'])"
  done
done
