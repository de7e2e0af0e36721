#!/bin/bash
# K1 A/B: STFT parity tests on the in-tree library, then tools/stft_ab.py over the variant libraries named on the
# command line (tools/_libavse_<tag>.so), each compared with the first.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stft.py tests/test_gpu_pipeline.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/stftab_t.log 2>&1
rc=$?
tail -5 gpurun_out/stftab_t.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
first=""
for tag in "$@"; do
  timeout -k 10 150 python tools/stft_ab.py run tools/_libavse_$tag.so $tag || exit $?
  if [ -z "$first" ]; then first=$tag; else python tools/stft_ab.py cmp $first $tag; fi
done
