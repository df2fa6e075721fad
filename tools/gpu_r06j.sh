#!/bin/bash
# Round-6 session j: stream-layout knobs re-checked on this round's kernels, alternating in one
# box session: classifier on a side stream (--overlap 1), stream priorities (--priority 1),
# detector heads on a side stream (--det-streams 2), at b64 and b8.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
for rep in 1 2; do
  for b in 64 8; do
    for k in "" "--overlap 1" "--overlap 1 --priority 1" "--det-streams 2"; do
      f=$OUT/r06j_b${b}_$(echo "$k" | tr -d ' -')_$rep.log
      timeout -k 10 200 python bench.py --batch $b --cpu-baseline 0 --h2d-steps 0 --roofline-steps 0 $k > $f 2>&1 || { tail -3 $f; exit 1; }
      echo "b$b [$k] $rep: $(grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])")"
    done
  done
done
echo "== session done"
