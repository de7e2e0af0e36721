# round 6, call za: range-guard tests with the round-6 kernels' layers added (a_conv1 on the vector ALUs, v_conv1 on
# k_conv_v1p, enc_dense on the split-pair k_gemm)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_range.py -x -v -rP --timeout 200 --timeout-method thread > gpurun_out/r06za_range.log 2>&1 || { tail -40 gpurun_out/r06za_range.log; exit 1; }
grep -E "x 2\^|passed|failed" gpurun_out/r06za_range.log
