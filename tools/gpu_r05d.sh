set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -rP --timeout 200 --timeout-method thread tests/test_gpu_range.py tests/test_gpu_pipeline.py tests/test_gpu_cli.py > gpurun_out/r05d_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r05d_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in "" "--checked" "" "--checked"; do
  timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline --steps 60 --warmup 5 $v > gpurun_out/r05d_bench.json 2>> gpurun_out/r05d_bench.err || exit $?
  python -c "
import json,sys
d=json.loads(open('gpurun_out/r05d_bench.json').read().strip().splitlines()[-1]); print(sys.argv[1:], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['range_guard'])
" $v
done
timeout -k 10 300 python bench.py --e2e --steps 5 --warmup 2 > gpurun_out/r05d_e2e.json 2>> gpurun_out/r05d_bench.err || exit $?
python -c "
import json; d=json.loads(open('gpurun_out/r05d_e2e.json').read().strip().splitlines()[-1]); print('e2e', d['value'], d['stage_ms_rank0'])"
