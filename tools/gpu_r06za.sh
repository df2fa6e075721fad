#!/bin/bash
# Round-6 session za: bitonic stages j <= 8 on DPP: NMS / pipeline tests, phases
# (one-launch form with stamps), split A/B timings.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_map.py -m gpu -x -v --timeout 120 --timeout-method thread -k "nms or pipeline or two_stage or config or int8 or map" > $OUT/r06za_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 $OUT/r06za_tests.log; [ $rc -eq 0 ] || exit $rc
for b in 64 8; do
  timeout -k 10 120 python tools/nms_phases.py --batch $b > $OUT/r06za_nms_b$b.log 2>&1 || exit $?
  grep -v amdgpu.ids $OUT/r06za_nms_b$b.log | tail -8
  timeout -k 10 180 python tools/nms_split_ab.py --batch $b > $OUT/r06za_split_b$b.log 2>&1 || { tail -5 $OUT/r06za_split_b$b.log; exit 1; }
  grep '^b' $OUT/r06za_split_b$b.log
done
echo "== session done"
