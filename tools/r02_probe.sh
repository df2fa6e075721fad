#!/bin/bash
# Round-2 probe: small-batch regime (the per-rank workload at N=4/8) and the heavy
# Darknet-53 detectors, per-step event tables + two-stage bench lines.
# Usage (gpurun): bash tools/r02_probe.sh TAG
set -u
TAG=${1:-r02a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 $to "$@" > $OUT/${TAG}_$name.log 2>&1
  local rc=$?
  tail -2 $OUT/${TAG}_$name.log
  [ $rc -eq 0 ] || { echo "FAILED rc=$rc"; exit $rc; }
}
run det_v4_b64 180 python tools/det_roofline.py --batch 64
run det_v4_b16 120 python tools/det_roofline.py --batch 16
run det_v4_b8 120 python tools/det_roofline.py --batch 8
run det_v3_416_b16 180 python tools/det_roofline.py --cfg yolov3-aider-416 --img 416 --batch 16
run det_spp_608_b64 300 python tools/det_roofline.py --cfg yolov3-spp-aider --img 608 --batch 64 --iters 5
run bench_b64 300 python bench.py --cpu-baseline 0
run bench_b16 120 python bench.py --batch 16 --cpu-baseline 0 --steps 50
run bench_b8 120 python bench.py --batch 8 --cpu-baseline 0 --steps 50
run bench_b8_noev 120 python bench.py --batch 8 --cpu-baseline 0 --steps 50 --step-events 0
cd /tmp
run prof_b8 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_${TAG}_b8 -o run -- python3 $R/bench.py --batch 8 --steps 20 --warmup 3 --cpu-baseline 0
echo "== done"
