#!/bin/bash
# Round-6 GPU session: selected tests (TESTS, KEXPR), classifier stage timings (CLS: "key values batch;..."),
# bench lines (BENCHES: ";"-separated arg sets).  Usage (gpurun): TAG=r06b TESTS=... bash tools/gpu_r06.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r06}
cd $R
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TTIME:-600} python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread ${KEXPR:+-k "$KEXPR"} > $OUT/${TAG}_tests.log 2>&1
  rc=$?; echo "tests rc $rc"; tail -4 $OUT/${TAG}_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
i=0
IFS=';' read -ra CL <<< "${CLS:-}"
for c in "${CL[@]}"; do
  i=$((i+1)); set -- $c
  timeout -k 10 200 python tools/cls_stages.py --key $1 --values $2 --batch $3 ${4:+--model $4} > $OUT/${TAG}_cls$i.log 2>&1
  rc=$?; echo "cls $i ($c) rc $rc"; grep "total" $OUT/${TAG}_cls$i.log
  [ $rc -eq 0 ] || exit $rc
done
i=0
IFS=';' read -ra BL <<< "${BENCHES:-}"
for b in "${BL[@]}"; do
  i=$((i+1))
  timeout -k 10 400 python bench.py $b > $OUT/${TAG}_bench$i.log 2>&1
  rc=$?; echo "bench $i ($b) rc $rc"
  python - $OUT/${TAG}_bench$i.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")]
if l:
    d = json.loads(l[-1]); r = d.get("roofline") or {}
    print(d["value"], d["ms_per_step"], r.get("kernel"), r.get("frac"))
PY
  [ $rc -eq 0 ] || exit $rc
done
