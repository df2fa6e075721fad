# GPU session: selected tests (TESTS / KEXPR), then bench lines (BENCHES: ";"-separated arg sets)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r03}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TTIME:-900} python -u -m pytest $TESTS -m gpu -v -s --timeout 300 --timeout-method thread ${KEXPR:+-k "$KEXPR"} > $OUT/${TAG}_tests.log 2>&1
  rc=$?; echo "tests rc $rc"; tail -4 $OUT/${TAG}_tests.log
  [ $rc -eq 0 ] || [ "${CONT:-0}" = 1 ] || exit $rc
fi
i=0
IFS=';' read -ra BL <<< "${BENCHES:-}"
for b in "${BL[@]}"; do
  i=$((i+1))
  (cd $R && timeout -k 10 600 python bench.py $b) > $OUT/${TAG}_bench$i.log 2>&1
  rc=$?; echo "bench $i ($b) rc $rc"; tail -c 600 $OUT/${TAG}_bench$i.log; echo
  [ $rc -eq 0 ] || exit $rc
done
