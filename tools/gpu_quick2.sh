#!/bin/bash
# tests named in $TESTS on the in-tree library, then tools/stft_time.py for each variant library tag given
mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_gpu_stft.py tests/test_gpu_istft.py tests/test_gpu_pipeline.py tests/test_keras_h5.py"}
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/q2_t.log 2>&1
rc=$?
tail -6 gpurun_out/q2_t.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for tag in "$@"; do
  echo "== $tag"
  timeout -k 10 200 python tools/stft_time.py tools/_libavse_$tag.so || exit $?
done
