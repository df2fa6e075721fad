#!/bin/bash
# Round-2 GPU check: a pytest selection, then bench lines (each step time-limited).
# Usage (gpurun): bash tools/r02_check.sh TAG "pytest targets" "bench arg sets separated by ;"
set -u
TAG=$1; TESTS=${2:-}; BENCHES=${3:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
if [ -n "$TESTS" ]; then
  echo "== tests $TESTS"
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/${TAG}_tests.log | tail -40; [ $rc -eq 0 ] || exit $rc
fi
i=0
IFS=';' read -ra BS <<< "$BENCHES"
for B in "${BS[@]}"; do
  i=$((i+1))
  echo "== bench $i: $B"
  timeout -k 10 400 python bench.py $B > $OUT/${TAG}_bench$i.log 2>&1
  rc=$?; grep -v amdgpu.ids $OUT/${TAG}_bench$i.log | tail -3; [ $rc -eq 0 ] || exit $rc
done
echo "== done"
