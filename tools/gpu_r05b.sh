set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 200 --timeout-method thread tests/test_gpu_range.py tests/test_gpu_split.py tests/test_gpu_pipeline.py > gpurun_out/r05b_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05b_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in "" "--unchecked" "--graph" "--graph --unchecked" "" "--graph"; do
  timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline --steps 50 --warmup 5 $v > gpurun_out/r05b_bench.json 2>> gpurun_out/r05b_bench.err || exit $?
  python -c "
import json,sys
d=json.loads(open('gpurun_out/r05b_bench.json').read().strip().splitlines()[-1]); print(sys.argv[1:], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['range_guard']['bits'])
" $v
done
