#!/bin/bash
# v_conv1 split-kernel ablation (k_conv_v1s AVSE_V1S_ABL variants in tools/_v1var): stage times of the split forward
# for each library, one process each.  1 = no epilogue stores, 2 = no window staging, 4 = no MFMAs, 6 = 2 | 4.
OUT=gpurun_out
for v in base 1 2 4 6; do
    lib=""; [ $v != base ] && lib=tools/_v1var/libavse_abl$v.so
    AVSE_LIBRARY=$lib timeout -k 10 120 python -u tools/dtype_time.py 512 float32_split > $OUT/v1ab_$v.log 2>&1 || exit $?
    echo "$v $(grep -o "'v_conv1': [0-9.]*" $OUT/v1ab_$v.log)"
done
AVSE_LIBRARY=tools/_v1var/libavse_k3bp4.so timeout -k 10 120 python -u tools/dtype_time.py 512 float32_split > $OUT/v1ab_k3bp4.log 2>&1 || exit $?
echo "k3bp4 $(grep -o "'v_conv[345]': [0-9.]*" $OUT/v1ab_k3bp4.log | tr '\n' ' ') base $(grep -o "'v_conv[345]': [0-9.]*" $OUT/v1ab_base.log | tr '\n' ' ')"
