#!/bin/bash
# b8 / b64 operating points against the number of HIP hardware queues per process.
# Usage (gpurun): bash tools/hwq_sweep.sh TAG "Q:args;Q:args;..."
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
IFS=';' read -ra RUNS <<< "$2"
i=0
for r in "${RUNS[@]}"; do
  i=$((i+1)); q=${r%%:*}; a=${r#*:}
  (cd $R && GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --cpu-baseline 0 --h2d-steps 0 --roofline-steps 0 $a) > $OUT/${TAG}_$i.log 2>&1
  rc=$?
  v=$(python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]);print(d['value'],d['ms_per_step'],d['step_latency_ms_median'],d['config']['inflight'])" $OUT/${TAG}_$i.log 2>/dev/null)
  echo "q=$q [$a] rc=$rc -> $v"
  [ $rc -eq 0 ] || exit $rc
done
