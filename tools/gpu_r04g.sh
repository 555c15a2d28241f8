# round-4 GPU pass g: fp32 attention chunk 16 -> 8 units per wave (parity + fp32s / fp32 bench
# lines), and the batch-1 small-M tile A/B (CLIPK_GEMM_SMALL64), interleaved
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_parity_gpu.py -k "(fp32s or fp32) and not config and not large_rows" > gpurun_out/r04g_parity.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --prec fp32s --no-extra --no-cpu-baseline --eval-images 5000 --steps 10 \
  > gpurun_out/r04g_bench_fp32s.json 2> gpurun_out/r04g_bench_fp32s.err && \
timeout -k 10 120 python -u tools/b1_time.py > gpurun_out/r04g_b1.txt 2>&1 && \
CLIPK_GEMM_SMALL64=1 timeout -k 10 120 python -u tools/b1_time.py >> gpurun_out/r04g_b1.txt 2>&1 && \
timeout -k 10 120 python -u tools/b1_time.py >> gpurun_out/r04g_b1.txt 2>&1 && \
CLIPK_GEMM_SMALL64=1 timeout -k 10 120 python -u tools/b1_time.py >> gpurun_out/r04g_b1.txt 2>&1
rc=$?
echo exit $rc
exit $rc
