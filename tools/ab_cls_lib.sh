#!/bin/bash
# Classifier timing A/B of two librtdm.so builds (tools/ab_cls.py --values 1, RTDM_LIB alternating
# between the in-tree library and abtmp/$1).  Usage (gpurun): bash tools/ab_cls_lib.sh OLD_SO TAG ["ab_cls args"]
set -u
OLD=$1; TAG=$2; EXTRA=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for I in 1 2; do
  for L in new old; do
    if [ $L = old ]; then export RTDM_LIB=$R/abtmp/$OLD; else export RTDM_LIB=$R/real-time-disaster-management_amd/rtdm/librtdm.so; fi
    timeout -k 10 200 python tools/ab_cls.py --values 1 --rounds 3 --iters 20 $EXTRA > $OUT/${TAG}_${L}$I.log 2>&1 || { tail -5 $OUT/${TAG}_${L}$I.log; exit 1; }
    echo "$L$I $(grep -v amdgpu.ids $OUT/${TAG}_${L}$I.log | tail -2 | tr '\n' ' ')"
  done
done
