set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -rP --timeout 200 --timeout-method thread tests/test_gpu_split.py -k "windowed or intermediates or bench_batch" > gpurun_out/r05c_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "window vs|output abs|passed|failed|Error" gpurun_out/r05c_tests.log | head -30
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
for v in 0 1; do
AVSE_NO_WIN=$v timeout -k 10 120 python -u tools/dtype_time.py 512 float32_split > gpurun_out/r05c_t_${v}_${r}.log 2>&1 || exit $?
echo "no_win=$v $(grep -o 'step *[0-9.]* ms' gpurun_out/r05c_t_${v}_${r}.log) $(grep -o "'[ad]_[a-z]*[0-9]': [0-9.]*" gpurun_out/r05c_t_${v}_${r}.log | tr '\n' ' ')"
done; done
