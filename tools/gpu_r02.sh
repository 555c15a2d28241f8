# round-2 GPU pass: -m gpu tests, the PMC traffic passes (FETCH_SIZE / WRITE_SIZE, separate
# runs) of the headline workload, one bench line (which reads the fresh traffic.json), and a
# kernel-trace profile of the headline workload alone (no eval / fp32 / batch-1 legs, so the
# per-kernel averages are the train step's).
set -o pipefail
R=$(pwd)
TAG=${1:-r02}
mkdir -p gpurun_out profiles/r02_pmc
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 && \
bash tools/pmc_bench.sh gpurun_out/pmc_$TAG > gpurun_out/pmc_$TAG.log 2>&1 && \
cp gpurun_out/pmc_$TAG/traffic.json gpurun_out/pmc_$TAG/summary.txt profiles/r02_pmc/ && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o p -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra --eval-images 0 > $R/gpurun_out/prof_$TAG.log 2>&1
rc=$?
cd $R
[ $rc -eq 0 ] && [ -n "$YARD" ] && timeout -k 10 300 python -u tools/gemm_yardstick.py --vit > gpurun_out/yard_vit_$TAG.log 2>&1
echo exit $rc $?
