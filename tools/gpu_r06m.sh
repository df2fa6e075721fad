#!/bin/bash
# Round-6 session m: isolated-launch kernel stats with the objectness side array on / off,
# then the stream-layout knob sweep (tools/gpu_r06j.sh).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
for v in 1 0; do
  (cd /tmp && RTDM_TUNE="objectness=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_r06m_o$v -o run -- python3 $R/bench.py --steps 1 --warmup 0 --h2d-steps 0 --cpu-baseline 0 --inflight 1 > $OUT/prof_r06m_o$v.log 2>&1) || exit $?
  echo "isolated objectness=$v ok"
done
bash tools/gpu_r06j.sh
