#!/bin/bash
# One GPU-box A/B session of the in-tree librtdm.so against an older build (OLD, a path under
# the repo such as ab/base.so):
#   TESTS   pytest selection run first on the new library (-m gpu), e.g. "tests/test_gpu_parity.py"
#   KEXPR   optional -k expression for TESTS
#   CLS     classifier stage timing batches ("64 8"), new and old alternating
#   BENCHES ";"-separated bench.py argument sets, new and old alternating, twice
# Usage (gpurun): TAG=r06e OLD=ab/base.so TESTS=... CLS="64 8" BENCHES="--batch 64;--batch 8" bash tools/ab_session.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-ab}
NEW=$R/real-time-disaster-management_amd/rtdm/librtdm.so
OLDP=${OLD:+$R/$OLD}
cd $R
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TTIME:-600} python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread ${KEXPR:+-k "$KEXPR"} > $OUT/${TAG}_tests.log 2>&1
  rc=$?; echo "tests rc $rc"; tail -3 $OUT/${TAG}_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
libs="new"; [ -n "$OLDP" ] && libs="new old"
for b in ${CLS:-}; do
  for L in $libs; do
    if [ $L = old ]; then export RTDM_LIB=$OLDP; else export RTDM_LIB=$NEW; fi
    timeout -k 10 200 python tools/cls_stages.py --key acff_chain --values 1 --batch $b > $OUT/${TAG}_cls_${L}_b$b.log 2>&1
    rc=$?; echo "cls b$b $L rc $rc: $(grep total $OUT/${TAG}_cls_${L}_b$b.log)"
    [ $rc -eq 0 ] || exit $rc
  done
done
i=0
IFS=';' read -ra BL <<< "${BENCHES:-}"
for bargs in "${BL[@]}"; do
  i=$((i+1))
  for rep in 1 2; do
    for L in $libs; do
      if [ $L = old ]; then export RTDM_LIB=$OLDP; else export RTDM_LIB=$NEW; fi
      f=$OUT/${TAG}_bench${i}_${L}${rep}.log
      timeout -k 10 300 python bench.py --cpu-baseline 0 --h2d-steps 0 --roofline-steps 0 $bargs > $f 2>&1
      rc=$?
      echo "bench$i ($bargs) $L$rep rc $rc: $(grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
      [ $rc -eq 0 ] || { tail -5 $f; exit $rc; }
    done
  done
done
# kernel trace of the new library's bench (overlap analysis: tools/overlap.py), PROF = bench args
if [ -n "${PROF:-}" ]; then
  export RTDM_LIB=$NEW
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_${TAG} -o run -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-baseline 0 --h2d-steps 0 --roofline-steps 0 $PROF > $OUT/prof_${TAG}.log 2>&1)
  rc=$?; echo "prof rc $rc"; [ $rc -eq 0 ] || exit $rc
fi
echo "== done"
