# round-4 GPU pass: the new tests (RCCL 1-rank, W=768 GEMMs, split GEMM, focal reductions, PREC fp32s
# parity, configs 4/5 at C=1000 vs the oracle) -- each step under its own limit, chained with &&
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
  tests/test_dist_nccl_gpu.py tests/test_kernels_gpu.py -k "nccl or focal or w768 or split" \
  > gpurun_out/r04a_kernels.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest -v -s --timeout 600 --timeout-method thread \
  tests/test_parity_gpu.py -k "fp32s and not config" \
  > gpurun_out/r04a_fp32s.txt 2>&1 ; \
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
  tests/test_parity_gpu.py -k "config4 or config5" tests/test_vision_schedule_gpu.py \
  > gpurun_out/r04a_configs.txt 2>&1
rc=$?
echo exit $rc
exit $rc
