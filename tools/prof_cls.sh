set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r02ae_cls -o run -- python3 $R/tools/ab_cls.py --values 1 --rounds 2 --iters 10 > $R/gpurun_out/prof_r02ae_cls.log 2>&1
