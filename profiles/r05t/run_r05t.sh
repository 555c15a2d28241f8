# L2 hit rate per kernel of the batch-1 step (TCC_HIT_sum / TCC_MISS_sum, one PMC pass)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05t; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/tcc -o p -- python3 $R/bench.py --batch 1 --steps 5 --warmup 2 --no-cpu-baseline --no-prof --no-extra --eval-images 0 > $O/tcc.log 2>&1 || exit $?
echo ok
