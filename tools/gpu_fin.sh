#!/bin/bash
# Final-tree certification: full GPU suite, smoke, bench (driver defaults), isolated-launch
# rocprof, the two PMC traffic passes over the bench, config 3 bench line.  TAG = $1.
set -u
TAG=${1:-r06fin}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
bash tools/gpu_check.sh $TAG "tests smoke bench proflaunch pmc" || exit $?
timeout -k 10 300 python bench.py --classifier none --cfg yolov3-aider-416 --img 416 --batch 16 --cpu-baseline 0 --h2d-steps 0 > $OUT/${TAG}c3_bench.log 2>&1 || exit $?
grep '^{' $OUT/${TAG}c3_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c3', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --batch 8 --cpu-baseline 0 --h2d-steps 0 > $OUT/${TAG}b8_bench.log 2>&1 || exit $?
grep '^{' $OUT/${TAG}b8_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('b8', d['value'], d['ms_per_step'])"
echo "== fin done"
