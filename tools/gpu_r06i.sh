#!/bin/bash
# Round-6 session i: host enqueue time per eager pipeline call (b8, b64) with cProfile.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
for b in 8 64; do
  timeout -k 10 200 python tools/host_launch.py --batch $b --calls 100 > $OUT/r06i_host_b$b.log 2>&1 || exit $?
  grep 'host enqueue' $OUT/r06i_host_b$b.log
done
echo "== session done"
