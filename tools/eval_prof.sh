set -e
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/evprof -o p -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-prof --eval-images 300 > $R/gpurun_out/evprof.log 2>&1
