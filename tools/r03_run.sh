set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_int8.py $R/tests/test_gpu_pipeline.py -m gpu -v -s --timeout 300 --timeout-method thread -k "cond or int8 or bench_config or graph_cache" > $OUT/r03a_tests.log 2>&1
echo "tests rc $?"; tail -15 $OUT/r03a_tests.log
[ "${BENCH:-1}" = 1 ] && cd $R && timeout -k 10 600 python bench.py --steps 30 --warmup 5 --cpu-baseline 0 > $OUT/r03a_bench.log 2>&1; echo "bench rc $?"; tail -c 1500 $OUT/r03a_bench.log
