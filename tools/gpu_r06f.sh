#!/bin/bash
# Round-6 session f: same-box bench A/B (in-tree library vs ab/base.so), the classifier's SQ
# counters at b64, config 3 (yolov3-aider-416 b16) isolated-launch kernel stats + bench line,
# and a kernel trace of the b64 bench for tools/overlap.py.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 60 ./tools/probe/mfma_rate || exit $?
TAG=r06f OLD=ab/base.so BENCHES="--batch 64;--batch 8" PROF="--batch 64" bash tools/ab_session.sh || exit $?
PMC_CMD="tools/cls_stages.py --key acff_chain --values 1 --iters 2 --batch 64" bash tools/pmc_sq.sh r06fcls || exit $?
C3="--classifier none --cfg yolov3-aider-416 --img 416 --batch 16"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_r06fc3_rl -o run -- python3 $R/bench.py $C3 --steps 1 --warmup 0 --h2d-steps 0 --cpu-baseline 0 --roofline-steps 0 --inflight 1 > $OUT/prof_r06fc3_rl.log 2>&1) || exit $?
echo "c3 isolated prof ok"
timeout -k 10 300 python bench.py $C3 --cpu-baseline 0 --h2d-steps 0 > $OUT/r06fc3_bench.log 2>&1 || exit $?
grep '^{' $OUT/r06fc3_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('c3', d['value'], d['ms_per_step'])"
echo "== session done"
