#!/bin/bash
# Round-6 session o: acff_chain phase stamps (mode 16, block 0) after the LDS address fix.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
for b in 64 8; do
  timeout -k 10 200 python tools/cls_stages.py --key acff_chain --values 16 --iters 6 --batch $b > $OUT/r06o_chain_b$b.log 2>&1 || exit $?
  grep -v amdgpu $OUT/r06o_chain_b$b.log | tail -3
done
echo "== session done"
