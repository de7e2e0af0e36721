#!/bin/bash
# A/B of library builds on one box: tools/dtype_time.py (forward stage times at B = 512), variants alternated twice.
#   bash tools/gpu_ab2.sh [variant ...]   (default: prev cur); "cur" is the in-tree libavse.so, any other name X
#   is tools/_v1var/libavse_X.so; DT=bf16 (or float32) times that dtype instead of float32_split
OUT=gpurun_out
VARS=${@:-prev cur}
DT=${DT:-float32_split}
for r in 1 2; do
  for v in $VARS; do
    lib=""; [ $v != cur ] && lib=tools/_v1var/libavse_$v.so
    log=$OUT/ab2_${DT}_${v}_$r.log
    AVSE_LIBRARY=$lib timeout -k 10 120 python -u tools/dtype_time.py 512 $DT > $log 2>&1 || exit $?
    echo "$DT $v $r $(grep -o 'step *[0-9.]* ms' $log) $(grep -o "'v_conv[12]': [0-9.]*" $log | tr '\n' ' ')"
  done
done
