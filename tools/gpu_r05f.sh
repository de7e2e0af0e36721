#!/bin/bash
# Round-5 closing GPU call: the suite, both benches and the rocprof recipe on the final tree (tools/gpu_round.sh), then
# a two-rank RCCL probe on the box's one GPU and the per-frame-rate forward / STFT times
bash tools/gpu_round.sh r05f prof || exit $?
timeout -k 10 150 python tools/rccl_probe.py 2 > gpurun_out/rccl_probe.log 2>&1
echo "rccl probe rc=$?"; tail -3 gpurun_out/rccl_probe.log
timeout -k 10 300 python -u tools/fps_time.py 512 float32_split bf16 > gpurun_out/fps_time.log 2>&1 || exit $?
cat gpurun_out/fps_time.log
