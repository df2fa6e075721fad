#!/bin/bash
# Round-6 session k: objectness side array: NMS / pipeline / head tests, then the bench with
# and without it (RTDM_TUNE objectness=0), alternating, b64 and b8.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_heads.py tests/test_gpu_trt.py -m gpu -x -v --timeout 120 --timeout-method thread -k "nms or objectness or pipeline or head or trt or two_stage or config or int8" > $OUT/r06k_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 $OUT/r06k_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for b in 64 8; do
    for v in 1 0; do
      f=$OUT/r06k_b${b}_o${v}_$rep.log
      RTDM_TUNE="objectness=$v" timeout -k 10 200 python bench.py --batch $b --cpu-baseline 0 --h2d-steps 0 --roofline-steps 0 > $f 2>&1 || { tail -3 $f; exit 1; }
      echo "b$b objectness=$v $rep: $(grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])")"
    done
  done
done
echo "== session done"
