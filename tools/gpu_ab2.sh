#!/bin/bash
# A/B of library builds on one box: tools/dtype_time.py (split forward stage times), variants alternated twice.
#   bash tools/gpu_ab2.sh [variant ...]   (default: prev cur); "cur" is the in-tree libavse.so, any other name X
#   is tools/_v1var/libavse_X.so
OUT=gpurun_out
VARS=${@:-prev cur}
for r in 1 2; do
  for v in $VARS; do
    lib=""; [ $v != cur ] && lib=tools/_v1var/libavse_$v.so
    AVSE_LIBRARY=$lib timeout -k 10 120 python -u tools/dtype_time.py 512 float32_split > $OUT/ab2_${v}_$r.log 2>&1 || exit $?
    echo "$v $r $(grep -o 'step *[0-9.]* ms' $OUT/ab2_${v}_$r.log) $(grep -o "'v_conv1': [0-9.]*" $OUT/ab2_${v}_$r.log)"
  done
done
