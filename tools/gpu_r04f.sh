# round-4 profiling pass: PMC traffic passes (FETCH_SIZE / WRITE_SIZE, separate runs) of the
# headline workload -> profiles/r04_pmc (read by bench.py's roofline), the full bench line, and a
# rocprofv3 kernel-trace + stats profile of the headline workload alone. Each step under its own
# limit, chained with &&.
set -o pipefail
R=$(pwd)
TAG=${1:-r04f}
mkdir -p gpurun_out profiles/r04_pmc
bash tools/pmc_bench.sh gpurun_out/pmc_$TAG > gpurun_out/pmc_$TAG.log 2>&1 && \
cp gpurun_out/pmc_$TAG/traffic.json gpurun_out/pmc_$TAG/summary.txt profiles/r04_pmc/ && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra --eval-images 0 > $R/gpurun_out/prof_$TAG.log 2>&1
rc=$?
echo exit $rc
exit $rc
