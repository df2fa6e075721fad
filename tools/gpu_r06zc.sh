#!/bin/bash
# Round-6 session zc: nms_scan_kernel with keys and the kept list in LDS: NMS tests, the
# bench's isolated-launch kernel stats (the NMS kernels in the bench's own workload).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -x -v --timeout 120 --timeout-method thread -k "nms or two_stage or pipeline" > $OUT/r06zc_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 $OUT/r06zc_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_check.sh r06zc "proflaunch" || exit $?
