# round-4 GPU pass s: fp32 prefix attention with the chunk size fitted to one round of resident waves (f32_uc)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k prefix \
  > gpurun_out/r04s_tests.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_parity_gpu.py -k "fp32" \
  >> gpurun_out/r04s_tests.txt 2>&1 && \
SWEEP_DTYPE=fp32 timeout -k 10 120 python -u tools/attn_sweep.py --one > gpurun_out/r04s_attn1.txt 2>&1 && \
SWEEP_DTYPE=fp32 CLIPK_LIB=build_ab/f32v0/libclipk.so timeout -k 10 120 python -u tools/attn_sweep.py --one > gpurun_out/r04s_attn0.txt 2>&1 && \
timeout -k 10 300 python -u tools/site_table.py --prec fp32s > gpurun_out/r04s_s1.txt 2>&1 && \
CLIPK_LIB=build_ab/f32v0/libclipk.so timeout -k 10 300 python -u tools/site_table.py --prec fp32s > gpurun_out/r04s_s0.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --prec fp32s --no-extra --no-cpu-baseline --no-configs --eval-images 5000 --steps 10 > gpurun_out/r04s_b1.json 2>/dev/null && \
CLIPK_LIB=build_ab/f32v0/libclipk.so timeout -k 10 300 python -u bench.py --prec fp32s --no-extra --no-cpu-baseline --no-configs --eval-images 5000 --steps 10 > gpurun_out/r04s_b0.json 2>/dev/null
rc=$?
echo exit $rc
exit $rc
