#!/bin/bash
# Round-6 session zb: nms_scan_kernel stages the bitmask in LDS before the scan: NMS tests,
# split A/B timings, kernel durations under rocprofv3.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -x -v --timeout 120 --timeout-method thread -k "nms or two_stage or pipeline" > $OUT/r06zb_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 $OUT/r06zb_tests.log; [ $rc -eq 0 ] || exit $rc
for b in 64 8; do
  timeout -k 10 180 python tools/nms_split_ab.py --batch $b > $OUT/r06zb_split_b$b.log 2>&1 || { tail -5 $OUT/r06zb_split_b$b.log; exit 1; }
  grep '^b' $OUT/r06zb_split_b$b.log
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_r06zb -o run -- python3 $R/tools/nms_split_ab.py --batch 64 --iters 20 > $OUT/prof_r06zb.log 2>&1) || exit $?
echo "== session done"
