#!/bin/bash
# Queue one gpurun call: retry only while the pod has no free slot (exit 3, nothing ran and
# nothing was charged); any other exit code (including a failed GPU step) ends the loop.
#   bash tools/gpurun_q.sh LOG TIMEOUT 'command'
LOG=$1
TO=$2
shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 150
done
exit 3
