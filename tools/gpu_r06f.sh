# round 6, call f: split fused decoder head (conv_dechs.hip): parity tests + A/B bench (AVSE_NO_DECHEAD)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_range.py > gpurun_out/r06f_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|fused head|fused tail|split N=37 db=True" gpurun_out/r06f_tests.log | tail -20
if [ $rc -ne 0 ]; then exit $rc; fi
for v in 0 1 0 1; do
  AVSE_NO_DECHEAD=$v timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline --steps 40 --warmup 5 > gpurun_out/r06f_bench_$v.json 2>> gpurun_out/r06f_bench.err || exit $?
  python -c "
import json
d=json.loads(open('gpurun_out/r06f_bench_$v.json').read().strip().splitlines()[-1]); st=d['breakdown']['stage_ms']
print('no_dechead=$v', d['value'], d['ms_per_step'], 'd1', st['d_deconv1'], 'd2', st['d_deconv2'], 'd3', st['d_deconv3'], 'tail', st['d_deconv4'], 'frac', d['breakdown']['step_frac_of_peak'])
"
done
