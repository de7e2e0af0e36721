# round-3 check: new frame-rate tests, then the whole -m gpu suite, then a short bench
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_framerates.py -v --timeout 300 --timeout-method thread > gpurun_out/t_fr.log 2>&1; rc=$?
echo "framerates rc=$rc"; tail -3 gpurun_out/t_fr.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputest_r03c.log 2>&1; rc=$?
echo "suite rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/gputest_r03c.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_r03c.json 2> gpurun_out/bench_r03c.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_r03c.json'));print(d['value'],d['ms_per_step'],d['breakdown']['stage_ms']['v_conv1'],d['roofline']['avg_launch_ms'])"
