#!/bin/bash
# Bench operating-point sweep: one short bench line per "RTDM_TUNE|bench args" case.
# Usage (gpurun): bash tools/bench_sweep.sh TAG "tune|args;tune|args;..."
set -u
TAG=$1; CASES=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
IFS=';' read -ra CS <<< "$CASES"
for C in "${CS[@]}"; do
  T=${C%%|*}; A=${C#*|}
  RTDM_TUNE=$T timeout -k 10 200 python bench.py --steps ${STEPS:-30} --warmup ${WARM:-5} --cpu-baseline 0 --h2d-steps 0 --roofline-steps 0 $A > $OUT/${TAG}_case.log 2>&1 || { tail -3 $OUT/${TAG}_case.log; exit 1; }
  V=$(grep '^{' $OUT/${TAG}_case.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config'].get('inflight'))")
  echo "$T | $A => $V" | tee -a $OUT/${TAG}_sweep.txt
done
