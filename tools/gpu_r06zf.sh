# round 6, call zf: k_gemm loaders one row per lane (64 rows x 16 B per wave-instruction;
# lmap variant) vs 16 rows x 64 B (the library, cur); parity of the library first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_forward.py -x -v -rP --timeout 300 --timeout-method thread \
  -k "gemm_matches or batch_invariant or bench_batch or zero_video" > gpurun_out/r06zf_tests.log 2>&1 || { tail -40 gpurun_out/r06zf_tests.log; exit 1; }
grep -E "k_gemm vs|passed|failed" gpurun_out/r06zf_tests.log
for r in 1 2 3; do
  for v in cur lmap; do
    lib=""; [ $v != cur ] && lib=tools/_ab/libavse_$v.so
    AVSE_LIBRARY=$lib AVSE_DTYPE=float32_split AVSE_REPS=9 timeout -k 10 120 python -u tools/stage_times.py $v > gpurun_out/r06zf_${v}_$r.json 2> gpurun_out/r06zf_err.log || exit $?
    AVSE_LIBRARY=$lib AVSE_DTYPE=bf16 AVSE_REPS=9 timeout -k 10 120 python -u tools/stage_times.py $v > gpurun_out/r06zf_${v}_bf_$r.json 2>> gpurun_out/r06zf_err.log || exit $?
    python -c "
import json
for f, dt in (('gpurun_out/r06zf_${v}_$r.json', 'split'), ('gpurun_out/r06zf_${v}_bf_$r.json', 'bf16')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); st=d['stage_ms']
    print(d['label'], dt, $r, 'v_conv6', st['v_conv6'], 'dense', round(st['enc_dense']+st['dec_dense1']+st['dec_dense2'],4), d['total_ms'])"
  done
done
