# round 6, call s: split-pair k_gemm with the h / l MFMA groups interleaved: parity and A/B against k_conv (AVSE_NO_GEMM=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -v -rP --timeout 300 --timeout-method thread \
  -k "gemm_matches or bench_batch or batch_invariant or zero_video or forward_matches" > gpurun_out/r06s_tests.log 2>&1 || { tail -40 gpurun_out/r06s_tests.log; exit 1; }
grep -E "k_gemm vs|passed|failed" gpurun_out/r06s_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_range.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06s_range.log 2>&1 || { tail -30 gpurun_out/r06s_range.log; exit 1; }
tail -1 gpurun_out/r06s_range.log
for r in 1 2; do
  for v in 1 0; do
    AVSE_NO_GEMM=$v timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline --steps 40 --warmup 5 > gpurun_out/r06s_bench.json 2>> gpurun_out/r06s_bench.err || exit $?
    python -c "
import json
d=json.loads(open('gpurun_out/r06s_bench.json').read().strip().splitlines()[-1])
st=d.get('breakdown', {}).get('stage_ms', {})
print('no_gemm=$v r$r', d['value'], d['ms_per_step'], d['window_ms_per_step']['median'], 'v_conv6', st.get('v_conv6'), 'dense', round(st.get('enc_dense',0)+st.get('dec_dense1',0)+st.get('dec_dense2',0),4))
"
  done
done
