#!/bin/bash
# Config 5 evidence: int8 two-stage bench at the global b128 (one GPU) and the b16 per-rank
# shard of N=8, plus rocprofv3 kernel stats of the b128 run.
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python bench.py --dtype i8 --batch 128 > $OUT/${TAG}_i8_b128.log 2>&1 || { tail -5 $OUT/${TAG}_i8_b128.log; exit 1; }
grep '^{' $OUT/${TAG}_i8_b128.log | cut -c1-200
timeout -k 10 300 python bench.py --dtype i8 --batch 16 --cpu-baseline 0 --h2d-steps 0 > $OUT/${TAG}_i8_b16.log 2>&1 || { tail -5 $OUT/${TAG}_i8_b16.log; exit 1; }
grep '^{' $OUT/${TAG}_i8_b16.log | cut -c1-200
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_${TAG}_i8 -o run -- python3 $R/bench.py --dtype i8 --batch 128 --steps 10 --warmup 3 --cpu-baseline 0 --h2d-steps 0 > $OUT/prof_${TAG}_i8.log 2>&1 || { tail -5 $OUT/prof_${TAG}_i8.log; exit 1; }
echo "== done"
