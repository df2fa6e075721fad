#!/bin/bash
# Round-6 session t: NMS IoU mask with the division-free threshold test
# NMS / pipeline tests, per-phase stamps at b64 / b8.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_map.py -m gpu -x -v --timeout 120 --timeout-method thread -k "nms or pipeline or two_stage or config or int8 or map" > $OUT/r06t_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 $OUT/r06t_tests.log; [ $rc -eq 0 ] || exit $rc
for b in 64 8; do
  timeout -k 10 120 python tools/nms_phases.py --batch $b > $OUT/r06t_nms_b$b.log 2>&1 || exit $?
  tail -9 $OUT/r06t_nms_b$b.log
done
echo "== session done"
