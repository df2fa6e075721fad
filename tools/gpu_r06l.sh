#!/bin/bash
# Round-6 session l: resize LDS sized to the geometry (4 blocks / CU): preprocess / classifier /
# CLI tests, classifier stage A/B against ab/head.so, bench A/B; isolated-launch kernel stats
# with the objectness side array on and off.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
cd $R
TAG=r06l OLD=ab/head.so TESTS="tests/test_gpu_parity.py tests/test_cli.py tests/test_gpu_letterbox.py" KEXPR="preprocess or classifier or acff or redconv or cli or batch_edges or two_stage" CLS="64 8" BENCHES="--batch 64" bash tools/ab_session.sh || exit $?
for v in 1 0; do
  (cd /tmp && RTDM_TUNE="objectness=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_r06l_o$v -o run -- python3 $R/bench.py --steps 1 --warmup 0 --h2d-steps 0 --cpu-baseline 0 --inflight 1 > $OUT/prof_r06l_o$v.log 2>&1) || exit $?
  echo "isolated objectness=$v ok"
done
echo "== session done"
