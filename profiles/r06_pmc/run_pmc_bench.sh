#!/bin/bash
# HBM traffic per kernel of the bench workload: one FETCH_SIZE pass and one WRITE_SIZE pass
# (separate rocprofv3 --pmc runs, counters only), summarised by tools/pmc_summary.py.
# Usage (GPU box, repo root): tools/pmc_bench.sh <outdir>
set -e
R=$(pwd)
OUT=$R/${1:-gpurun_out/pmc_bench}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o p -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prof --no-extra --eval-images 0 > $OUT/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o p -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prof --no-extra --eval-images 0 > $OUT/write.log 2>&1
python3 $R/tools/pmc_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
