#!/bin/bash
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
for K in 0 1; do
  for B in 64 8; do
    KORDER=$K timeout -k 10 120 python tools/det_roofline.py --batch $B > $OUT/${TAG}_k${K}_b$B.log 2>&1 || exit 1
    echo "k$K b$B $(grep forward $OUT/${TAG}_k${K}_b$B.log)"
  done
  KORDER=$K timeout -k 10 200 python tools/det_roofline.py --cfg yolov3-aider-416 --img 416 --batch 16 > $OUT/${TAG}_k${K}_v3.log 2>&1 || exit 1
  echo "k$K v3b16 $(grep forward $OUT/${TAG}_k${K}_v3.log)"
  KORDER=$K timeout -k 10 300 python tools/det_roofline.py --cfg yolov3-spp-aider --img 608 --batch 64 --iters 5 > $OUT/${TAG}_k${K}_spp.log 2>&1 || exit 1
  echo "k$K spp b64 $(grep forward $OUT/${TAG}_k${K}_spp.log)"
done
cd /tmp
for K in 0 1; do for C in FETCH_SIZE WRITE_SIZE; do
  KORDER=$K timeout -k 10 200 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_${C}_${TAG}k$K -o run -- python3 $R/tools/run_detector.py --iters 2 > $OUT/pmc_${C}_${TAG}k$K.log 2>&1 || exit 1
done; done
echo "== done"
