#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench run.  Usage (gpurun): bash tools/prof_bench.sh TAG ["bench args"]
set -u
TAG=$1; EXTRA=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-baseline 0 --h2d-steps 0 --roofline-steps 0 $EXTRA > $R/gpurun_out/prof_$TAG.log 2>&1
