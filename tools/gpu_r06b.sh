# round 6, call b: the split fused decoder tail (conv_dects.hip): probe its new packed form, parity tests, A/B timing
set -o pipefail
mkdir -p gpurun_out
PK_KINDS=5,41 timeout -k 10 120 python -u tools/pk_probe.py 8 > gpurun_out/r06b_pk_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; grep kind gpurun_out/r06b_pk_probe.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 600 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_range.py > gpurun_out/r06b_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|fused tail" gpurun_out/r06b_tests.log | tail -40
if [ $rc -ne 0 ]; then exit $rc; fi
for v in 0 1 0 1; do
  AVSE_NO_DECTAIL=$v timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline --steps 40 --warmup 5 > gpurun_out/r06b_bench_$v.json 2>> gpurun_out/r06b_bench.err || exit $?
  python -c "
import json,sys
d=json.loads(open('gpurun_out/r06b_bench_$v.json').read().strip().splitlines()[-1]); st=d['breakdown']['stage_ms']
print('no_dectail=$v', d['value'], d['ms_per_step'], 'd4', st['d_deconv4'], 'd5', st['d_deconv5'], 'd6', st['d_deconv6'], 'frac', d['breakdown']['step_frac_of_peak'])
"
done
