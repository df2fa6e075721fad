#!/bin/bash
# A/B of two builds of librtdm.so on one box: bench.py (and the detector alone) alternating
# RTDM_LIB between the in-tree library and abtmp/$1.
# Usage (gpurun): bash tools/ab_lib.sh OLD_SO_NAME TAG ["extra bench args"]
set -u
OLD=$1; TAG=$2; EXTRA=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for I in 1 2; do
  for L in new old; do
    if [ $L = old ]; then export RTDM_LIB=$R/abtmp/$OLD; else export RTDM_LIB=$R/real-time-disaster-management_amd/rtdm/librtdm.so; fi
    timeout -k 10 200 python bench.py --cpu-baseline 0 --h2d-steps 0 $EXTRA > $OUT/${TAG}_${L}$I.log 2>&1 || { tail -5 $OUT/${TAG}_${L}$I.log; exit 1; }
    echo "$L$I $(grep '^{' $OUT/${TAG}_${L}$I.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['achieved'], d['roofline']['frac'])")"
  done
done
echo "== done"
