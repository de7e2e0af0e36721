set -o pipefail
mkdir -p gpurun_out
for v in A B C A B C; do timeout -k 10 60 tools/_v1var/run_$v > gpurun_out/v1var_$v.log 2>&1 || exit $?; echo "== $v"; grep -E "full|only MFMA" gpurun_out/v1var_$v.log; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_r03b.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/t_r03b.log
