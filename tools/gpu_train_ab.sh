#!/bin/bash
# Training A/B: the training parity tests on the in-tree library, then the batch-16 fit-step timing (bench.py
# leg_train) over the variant libraries named on the command line (tools/_libavse_<tag>.so), alternated.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/trainab_t.log 2>&1 || { tail -30 gpurun_out/trainab_t.log; exit 1; }
tail -2 gpurun_out/trainab_t.log
for r in 1 2; do
  for tag in "$@"; do
    echo -n "$tag run $r: "
    AVSE_LIBRARY=$PWD/tools/_libavse_$tag.so timeout -k 10 120 python tools/train_time.py 20 | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['frac'])"
  done
done
