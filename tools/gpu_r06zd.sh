#!/bin/bash
# Round-6 session zd: conv_stem3 pooled stores as buffer stores + pkrtz staging (VALU trim): io bit
# identity against ab/head.so, stem tests, per-layer A/B, bench A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
NEW=$R/real-time-disaster-management_amd/rtdm/librtdm.so; OLD=$R/ab/head.so
for c in "yolov4-tiny-aider-416 608 8" "yolov3-aider-416 416 2" "yolov4-tiny-swish 416 2"; do
  set -- $c
  a=$(RTDM_LIB=$NEW timeout -k 10 120 python tools/io_hash.py --cfg $1 --img $2 --batch $3 2>/dev/null | grep sha256) || exit 1
  b=$(RTDM_LIB=$OLD timeout -k 10 120 python tools/io_hash.py --cfg $1 --img $2 --batch $3 2>/dev/null | grep sha256) || exit 1
  echo "new: $a"; echo "old: $b"; [ "$a" == "$b" ] || { echo "io differs"; exit 1; }
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_stem.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r06zd_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 $OUT/r06zd_tests.log; [ $rc -eq 0 ] || exit $rc
for I in 1 2; do
  for L in new old; do
    if [ $L = old ]; then export RTDM_LIB=$OLD; else export RTDM_LIB=$NEW; fi
    timeout -k 10 200 python tools/det_roofline.py > $OUT/r06zd_det_${L}$I.log 2>&1 || { tail -5 $OUT/r06zd_det_${L}$I.log; exit 1; }
    grep -E '^\s+0 ' $OUT/r06zd_det_${L}$I.log | head -2 | sed "s/^/$L$I /"
  done
done
unset RTDM_LIB
TAG=r06zd OLD=ab/head.so BENCHES="--batch 64;--batch 8" bash tools/ab_session.sh || exit $?
