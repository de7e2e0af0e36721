# round 6, call a: packed-FP32 form probe (every op_sel / neg form of the built library, solo vs beside MFMA), the
# two-rank gloo GPU tests, and the range / split / CLI tests after the checked-default change
set -o pipefail
mkdir -p gpurun_out
PK_KINDS=5,7,$(seq -s, 16 40) timeout -k 10 240 python -u tools/pk_probe.py 8 > gpurun_out/r06a_pk_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -30 gpurun_out/r06a_pk_probe.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -x -v -rP --timeout 600 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_range.py tests/test_gpu_split.py tests/test_keras_h5.py tests/test_gpu_cli.py tests/test_gpu_pipeline.py > gpurun_out/r06a_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r06a_tests.log | tail -60
exit $rc
