# round-4 GPU pass d: the fp32 long-attention forward rewrite (ViT L 50..577, text 64 < L <= 77):
# kernel tests, every fp32 / fp32s parity case incl. deep prompts and zero-shot, then fp32s bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py -k "attn or attention" > gpurun_out/r04d_attn.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_parity_gpu.py tests/test_deep_gpu.py -k "(fp32s or fp32) and not config" > gpurun_out/r04d_parity.txt 2>&1 && \
timeout -k 10 250 python -u bench.py --prec fp32s --no-extra --no-cpu-baseline --eval-images 5000 --steps 10 \
  > gpurun_out/r04d_bench_fp32s.json 2> gpurun_out/r04d_bench_fp32s.err
rc=$?
echo exit $rc
exit $rc
