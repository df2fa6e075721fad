#!/bin/bash
# Round-6 session g: classifier parity tests, classifier stage timing and bench A/B of the
# in-tree library against ab/prev.so (the previous commit), nms_kernel phase stamps at b64 / b8.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
TAG=r06g OLD=ab/prev.so TESTS="tests/test_gpu_parity.py tests/test_gpu_int8.py" KEXPR="classifier or acff or redconv or int8" CLS="64 8" BENCHES="--batch 64" bash tools/ab_session.sh || exit $?
for b in 64 8; do
  timeout -k 10 120 python tools/nms_phases.py --batch $b > $OUT/r06g_nms_b$b.log 2>&1 || exit $?
  tail -4 $OUT/r06g_nms_b$b.log
done
echo "== session done"
