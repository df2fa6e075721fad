#!/bin/bash
# PMC passes (one counter group per pass) over the detector of record alone.
# Usage (gpurun): bash tools/pmc_detector.sh TAG "CTR1 CTR2 ..." ["CTR ..."] ...
# PMC_CMD overrides the profiled program (default: tools/run_detector.py --iters 2).
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
if [ ! -f $OUT/counters_gfx950.txt ]; then timeout -k 10 120 rocprofv3 -L > $OUT/counters_gfx950.txt 2>&1 || true; fi
i=0
for GRP in "$@"; do
  i=$((i+1))
  echo "== pmc pass $i: $GRP"
  timeout -k 10 300 rocprofv3 --pmc $GRP --kernel-trace -d $OUT/pmcdet_${TAG}_$i -o run -- python3 $R/${PMC_CMD:-tools/run_detector.py --iters 2} > $OUT/pmcdet_${TAG}_$i.log 2>&1
  rc=$?; tail -2 $OUT/pmcdet_${TAG}_$i.log; [ $rc -eq 0 ] || exit $rc
done
