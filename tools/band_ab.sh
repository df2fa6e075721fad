# same-box A/B of the classifier paths in the two-stage bench
for rep in 1 2; do
for v in 1 0 2; do
  for b in 64 8; do
    RTDM_TUNE="acff_band=$v" timeout -k 10 300 python bench.py --cpu-baseline 0 --h2d-steps 0 --roofline-steps 0 --batch $b > gpurun_out/${TAG}_ab_${v}_${b}_${rep}.log 2>&1 || exit 1
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('band', sys.argv[2], 'b', sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/${TAG}_ab_${v}_${b}_${rep}.log $v $b
  done
done
done
