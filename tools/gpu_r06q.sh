#!/bin/bash
# Round-6 session q: the classifier's fused front (CLI transform + conv1, cls_front 1) against
# two launches (cls_front 0), same library: bit-identity tests, per-launch stage times, benches.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
TAG=r06q
timeout -k 10 600 python -u -m pytest tests/test_gpu_stem.py tests/test_gpu_parity.py tests/test_gpu_int8.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 $OUT/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for b in 64 8; do
  timeout -k 10 200 python tools/cls_stages.py --key cls_front --values 0,1 --batch $b > $OUT/${TAG}_cls_b$b.log 2>&1 || exit $?
  cat $OUT/${TAG}_cls_b$b.log
done
for bargs in "--batch 64" "--batch 8"; do
  for rep in 1 2; do
    for v in 0 1; do
      f=$OUT/${TAG}_bench_${bargs// /}_v${v}_$rep.log
      RTDM_TUNE="cls_front=$v" timeout -k 10 300 python bench.py --cpu-baseline 0 --h2d-steps 0 --roofline-steps 0 $bargs > $f 2>&1
      rc=$?
      echo "bench ($bargs) cls_front=$v rep$rep rc $rc: $(grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
      [ $rc -eq 0 ] || { tail -5 $f; exit $rc; }
    done
  done
done
echo "== done"
