# round-4 GPU pass e: fp32 long-attention forward (kernel tests + fp32 / fp32s parity), the GEMM
# split tail (kernel tests), then the headline bench without the extra lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py -k "attn or attention or split_tail" > gpurun_out/r04e_kernels.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_parity_gpu.py tests/test_deep_gpu.py -k "((fp32s or fp32) and not config) or split_tail" > gpurun_out/r04e_parity.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-extra --no-cpu-baseline --eval-images 5000 --steps 20 --warmup 5 \
  > gpurun_out/r04e_bench.json 2> gpurun_out/r04e_bench.err && \
CLIPK_GEMM_TAIL=0 timeout -k 10 300 python -u bench.py --no-extra --no-cpu-baseline --eval-images 5000 --steps 20 --warmup 5 \
  > gpurun_out/r04e_bench_notail.json 2> gpurun_out/r04e_bench_notail.err
rc=$?
echo exit $rc
exit $rc
