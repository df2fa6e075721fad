#!/bin/bash
# Round-6 session h: kernel traces of the b8 per-rank shard (4 in flight) for tools/overlap.py
# and its isolated launches (one batch in flight).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_r06h8 -o run -- python3 $R/bench.py --batch 8 --steps 40 --warmup 10 --cpu-baseline 0 --h2d-steps 0 --roofline-steps 0 > $OUT/prof_r06h8.log 2>&1 || exit $?
echo "b8 trace ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_r06h8_rl -o run -- python3 $R/bench.py --batch 8 --steps 1 --warmup 0 --h2d-steps 0 --cpu-baseline 0 --inflight 1 > $OUT/prof_r06h8_rl.log 2>&1 || exit $?
echo "b8 isolated ok"
grep '^{' $OUT/prof_r06h8_rl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])"
echo "== session done"
