#!/bin/bash
# kernel traces (rocprofv3 --kernel-trace) of a few commands, for timeline gap analysis
# Usage (gpurun): bash tools/r02_trace.sh TAG "cmd1;cmd2;..."   (cmds are python scripts + args)
set -u
TAG=$1; CMDS=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
IFS=';' read -ra CS <<< "$CMDS"
for C in "${CS[@]}"; do
  i=$((i+1))
  echo "== trace $i: $C"
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace_${TAG}_$i -o run -- python3 $R/$C > $OUT/trace_${TAG}_$i.log 2>&1
  rc=$?; grep -v amdgpu.ids $OUT/trace_${TAG}_$i.log | grep -v "^W2026\|rocprofv3\]" | tail -2; [ $rc -eq 0 ] || exit $rc
done
echo "== done"
