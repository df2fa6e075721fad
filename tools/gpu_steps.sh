#!/bin/bash
# One GPU-box session: run the steps of a plan file in order, each under its own time limit,
# stopping at the first failure (a GPU fault, abort or timeout ends the session there).
#   bash tools/gpu_steps.sh PLAN TAG
# PLAN: one step per line, "name|seconds|command" (run from the repo root; blank lines and
# lines starting with # are skipped).  Output of step `name` -> gpurun_out/TAG_name.log.
set -u
PLAN=$1
TAG=${2:-r04}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
while IFS='|' read -r name secs cmd; do
  [ -z "$name" ] && continue
  case "$name" in \#*) continue ;; esac
  echo "== $name ($secs s): $cmd"
  (cd $R && timeout -k 10 "$secs" bash -c "$cmd") > "$OUT/${TAG}_${name}.log" 2>&1
  rc=$?
  tail -c 1500 "$OUT/${TAG}_${name}.log"
  echo "== $name rc $rc"
  if [ $rc -ne 0 ] && [ "${CONT:-0}" != 1 ]; then exit $rc; fi
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done < "$PLAN"
echo "== all steps done"
