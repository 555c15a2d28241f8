# round-4 final check: the whole -m gpu suite and smoke() on the final build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04zf_gpu_tests.txt 2>&1 && \
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04zf_smoke.txt 2>&1
rc=$?
echo exit $rc
exit $rc
