#!/bin/bash
# Round-6 session u: NMS split over three launches (prep / bitmask blocks / scan) vs one launch
# per image: NMS + pipeline tests, event-timed A/B at b64 / b8, then the benches.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_map.py -m gpu -x -v --timeout 120 --timeout-method thread -k "nms or pipeline or two_stage or config or int8 or map" > $OUT/r06u_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 $OUT/r06u_tests.log; [ $rc -eq 0 ] || exit $rc
for b in 64 8; do
  timeout -k 10 180 python tools/nms_split_ab.py --batch $b > $OUT/r06u_nms_b$b.log 2>&1 || { tail -5 $OUT/r06u_nms_b$b.log; exit 1; }
  grep '^b' $OUT/r06u_nms_b$b.log
done
for bargs in "--batch 64" "--batch 8"; do
  for rep in 1 2; do
    for v in 0 1; do
      f=$OUT/r06u_bench_${bargs// /}_v${v}_$rep.log
      RTDM_TUNE="nms_split=$v" timeout -k 10 300 python bench.py --cpu-baseline 0 --h2d-steps 0 --roofline-steps 0 $bargs > $f 2>&1
      rc=$?
      echo "bench ($bargs) nms_split=$v rep$rep rc $rc: $(grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
      [ $rc -eq 0 ] || { tail -5 $f; exit $rc; }
    done
  done
done
echo "== session done"
