#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats + HBM counters.
# Usage (from the repo root, via gpurun):  bash tools/gpu_check.sh [tag] [stages]
#   stages: any of "tests smoke bench prof pmc" (default: all)
set -u
TAG=${1:-r01}
STAGES=${2:-"tests smoke bench prof proflaunch pmc"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
has() { [[ " $STAGES " == *" $1 "* ]]; }
if has tests; then
  echo "== tests"; timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests_$TAG.log 2>&1
  rc=$?; tail -3 $OUT/gpu_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if has smoke; then
  echo "== smoke"; (cd $R && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()") > $OUT/smoke_$TAG.log 2>&1
  rc=$?; tail -2 $OUT/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if has bench; then
  echo "== bench"; (cd $R && timeout -k 10 600 python bench.py ${BENCH_ARGS:-}) > $OUT/bench_$TAG.log 2>&1
  rc=$?; tail -1 $OUT/bench_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
cd /tmp
if has prof; then
  echo "== rocprofv3 kernel stats"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-baseline 0 ${BENCH_ARGS:-} > $OUT/prof_$TAG.log 2>&1
  rc=$?; tail -1 $OUT/prof_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if has proflaunch; then
  # the bench's roofline figure is measured on isolated eager launches (per-launch hipEvents
  # after the timed region); this profile times the same kind of launches alone
  echo "== rocprofv3 kernel stats, isolated launches"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_${TAG}_rl -o run -- python3 $R/bench.py --steps 1 --warmup 0 --h2d-steps 0 --cpu-baseline 0 --inflight 1 ${BENCH_ARGS:-} > $OUT/prof_${TAG}_rl.log 2>&1
  rc=$?; tail -1 $OUT/prof_${TAG}_rl.log; [ $rc -eq 0 ] || exit $rc
fi
if has pmc; then
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "== rocprofv3 pmc $C"
    timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace --stats -d $OUT/pmc_${C}_$TAG -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 ${BENCH_ARGS:-} > $OUT/pmc_${C}_$TAG.log 2>&1
    rc=$?; tail -1 $OUT/pmc_${C}_$TAG.log; [ $rc -eq 0 ] || exit $rc
  done
fi
echo "== done"
