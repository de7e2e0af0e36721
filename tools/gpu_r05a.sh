set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 200 --timeout-method thread tests/test_gpu_range.py tests/test_gpu_split.py > gpurun_out/r05a_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r05a_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/r05a_bench.json 2> gpurun_out/r05a_bench.err || exit $?
timeout -k 10 300 python bench.py --no-legs --no-cpu-baseline --steps 50 --warmup 5 --unchecked > gpurun_out/r05a_bench_unchecked.json 2>> gpurun_out/r05a_bench.err || exit $?
python -c "
import json
for f in ['gpurun_out/r05a_bench.json','gpurun_out/r05a_bench_unchecked.json']:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['range_guard'])
"
