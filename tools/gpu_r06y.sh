#!/bin/bash
# Round-6 session y: acff_persist resident blocks per CU (acff_per_cu 0 = occupancy, 1, 2) in
# the overlapped benches and the classifier alone.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
timeout -k 10 200 python tools/cls_stages.py --key acff_per_cu --values 0,1,2 --batch 64 > $OUT/r06y_cls_b64.log 2>&1 || exit 1
grep 'acff_per_cu=' $OUT/r06y_cls_b64.log
for bargs in "--batch 64" "--batch 8"; do
  for rep in 1 2; do
    for v in 0 1 2; do
      f=$OUT/r06y_bench_${bargs// /}_v${v}_$rep.log
      RTDM_TUNE="acff_per_cu=$v" timeout -k 10 300 python bench.py --cpu-baseline 0 --h2d-steps 0 --roofline-steps 0 $bargs > $f 2>&1
      rc=$?
      echo "bench ($bargs) acff_per_cu=$v rep$rep rc $rc: $(grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
      [ $rc -eq 0 ] || { tail -5 $f; exit $rc; }
    done
  done
done
echo "== done"
