#!/bin/bash
# Evidence run: the driver's bench command + b8 (the N=8 per-rank shard), rocprofv3 kernel
# stats of the bench, and the two PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic.
# Usage (gpurun): bash tools/r02_evidence.sh TAG ["extra bench args"]
set -u
TAG=$1; EXTRA=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
echo "== bench"
timeout -k 10 400 python bench.py $EXTRA > $OUT/${TAG}_bench.log 2>&1 || { tail -5 $OUT/${TAG}_bench.log; exit 1; }
grep '^{' $OUT/${TAG}_bench.log | cut -c1-300
if [ "${B8:-1}" = 1 ]; then
  echo "== bench b8"
  timeout -k 10 300 python bench.py --batch 8 --cpu-baseline 0 --h2d-steps 0 $EXTRA > $OUT/${TAG}_bench_b8.log 2>&1 || { tail -5 $OUT/${TAG}_bench_b8.log; exit 1; }
  grep '^{' $OUT/${TAG}_bench_b8.log | cut -c1-300
fi
cd /tmp
echo "== prof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run -- python3 $R/bench.py --steps ${PSTEPS:-10} --warmup 3 --cpu-baseline 0 --h2d-steps 0 $EXTRA > $OUT/prof_$TAG.log 2>&1 || { tail -5 $OUT/prof_$TAG.log; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $C"
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_${C}_$TAG -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --h2d-steps 0 --roofline-steps 2 $EXTRA > $OUT/pmc_${C}_$TAG.log 2>&1 || { tail -5 $OUT/pmc_${C}_$TAG.log; exit 1; }
done
echo "== done"
