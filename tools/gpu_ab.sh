#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/ab_t.log 2>&1 || true
timeout -k 10 120 python tools/stage_times.py p3 > gpurun_out/ab_new.log 2>&1
AVSE_B=8 timeout -k 10 120 python tools/stage_times.py p3b8 > gpurun_out/ab_b8.log 2>&1
