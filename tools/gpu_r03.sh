# round-3 GPU pass: -m gpu tests, smoke(), one default bench line (each step under its own
# time limit; the chain stops at the first failure)
set -o pipefail
TAG=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?
echo exit $rc
exit $rc
