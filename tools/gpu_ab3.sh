#!/bin/bash
# A/B of library builds on one box: forward stage times (tools/dtype_time.py, B = 512) alternated twice, then one
# FETCH_SIZE pass per build (tools/ab_fetch.py): "cur" = the in-tree libavse.so, X = tools/_ab/libavse_X.so
#   bash tools/gpu_ab3.sh TAG variant ...      (DT=bf16 | float32 to time another dtype)
OUT=gpurun_out
TAG=$1; shift
VARS=${@:-cur}
DT=${DT:-float32_split}
for r in 1 2; do
  for v in $VARS; do
    lib=""; [ $v != cur ] && lib=tools/_ab/libavse_$v.so
    log=$OUT/ab3_${TAG}_${DT}_${v}_$r.log
    AVSE_LIBRARY=$lib timeout -k 10 120 python -u tools/dtype_time.py 512 $DT > $log 2>&1 || exit $?
    echo "$DT $v $r $(grep -o 'step *[0-9.]* ms' $log) $(grep -o "'[a-z_0-9]*': [0-9.]*" $log | tr '\n' ' ')"
  done
done
if [ -n "$FETCH" ]; then
  cd /tmp && export TMPDIR=/tmp
  for v in $VARS; do
    lib=""; [ $v != cur ] && lib=$GRAFT_REPO_ROOT/tools/_ab/libavse_$v.so
    d=$GRAFT_REPO_ROOT/$OUT/ab3_${TAG}_fetch_$v
    rm -rf $d
    AVSE_LIBRARY=$lib AVSE_DTYPE=$DT timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d -o pmc -- \
        python3 $GRAFT_REPO_ROOT/tools/fwd_loop.py > $d.log 2>&1 || exit $?
    echo "== $v"; python3 $GRAFT_REPO_ROOT/tools/ab_fetch.py $d
  done
fi
