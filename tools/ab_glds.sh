set -e
R=$GRAFT_REPO_ROOT
cd $R
for V in 256x3 256x2 128x2; do
  RTDM_GLDS=$V timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "detector or pipeline" > gpurun_out/ab_tests_$V.log 2>&1
  tail -1 gpurun_out/ab_tests_$V.log
  RTDM_GLDS=$V timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/ab_bench_$V.log 2>&1
  cp gpurun_out/bench_steps.json gpurun_out/ab_steps_$V.json
  grep -o '"value": [0-9.]*' gpurun_out/ab_bench_$V.log | head -1
done
