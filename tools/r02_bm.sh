#!/bin/bash
# conv_pipe tile-row sweep: per-step detector tables at forced BM and the cost model
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for B in 8 16 64; do for BM in 0 256 128 64; do
  echo "== b$B bm$BM"
  timeout -k 10 120 python tools/det_roofline.py --batch $B --bm $BM --iters 10 > $OUT/${TAG}_b${B}_bm$BM.log 2>&1 || exit 1
  grep forward $OUT/${TAG}_b${B}_bm$BM.log
done; done
for BM in 0 256 128 64; do
  echo "== v3 b16 bm$BM"
  timeout -k 10 120 python tools/det_roofline.py --cfg yolov3-aider-416 --img 416 --batch 16 --bm $BM --iters 10 > $OUT/${TAG}_v3b16_bm$BM.log 2>&1 || exit 1
  grep forward $OUT/${TAG}_v3b16_bm$BM.log
done
echo "== done"
