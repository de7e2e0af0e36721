#!/bin/bash
# Round profiling recipe (run on the GPU box from the repo root):   bash tools/profile.sh r02
# 1. rocprofv3 --kernel-trace --stats of a short bench run                 -> gpurun_out/prof_<tag>/
# 2. separate PMC passes over tools/fwd_loop.py (B = 512 forward + spectrogram, the headline fp32_split dtype and
#    bf16): FETCH_SIZE, WRITE_SIZE (they do not fit one TCC pass), SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE
# 3. FETCH_SIZE / WRITE_SIZE over the configs[1] STFT (B = 4096, rotated buffers: AVSE_MODE=stft)
# 4. tools/pmc_summary.py -> profiles/<tag>_kernel_stats.csv, profiles/<tag>_pmc.json
# Every step has its own time limit and the chain stops at the first failure.
set -e
TAG=${1:-r02}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p $OUT
rm -rf $OUT/prof_$TAG $OUT/pmc_${TAG}_*
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
    python3 $ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof_${TAG}_bench.log 2>&1
for dt in fp32_split bf16; do
    lib=$dt; [ $dt = fp32_split ] && lib=float32_split
    for pass in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "mfma:SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
        name=${dt}_${pass%%:*}; ctr=${pass#*:}
        AVSE_DTYPE=$lib timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_${TAG}_$name -o pmc -- \
            python3 $ROOT/tools/fwd_loop.py > $OUT/pmc_${TAG}_$name.log 2>&1
    done
done
for pass in "sfetch:FETCH_SIZE" "swrite:WRITE_SIZE"; do
    name=${pass%%:*}; ctr=${pass#*:}
    AVSE_MODE=stft timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_${TAG}_$name -o pmc -- \
        python3 $ROOT/tools/fwd_loop.py > $OUT/pmc_${TAG}_$name.log 2>&1
done
cd $ROOT
python3 tools/pmc_summary.py $TAG
