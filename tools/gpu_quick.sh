#!/bin/bash
# Quick GPU iteration: selected -m gpu test files (arg 1, default the STFT / ISTFT / pipeline tests), then
# tools/stft_time.py.  A test failure (rc 1) still runs the timing; anything else ends the call.
TESTS=${1:-"tests/test_gpu_stft.py tests/test_gpu_istft.py tests/test_gpu_pipeline.py"}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest $TESTS -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/quick.log 2>&1
rc=$?
tail -15 gpurun_out/quick.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/stft_time.py
