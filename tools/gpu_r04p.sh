# round-4 GPU pass p: the fp32 prefix-attention kernels with the next unit's rows loaded one unit
# ahead (registers) vs the previous kernels (build_ab/f32pf0): kernel + fp32-class parity tests,
# the fp32s site table and the fp32s / fp32 bench lines, interleaved
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k prefix \
  > gpurun_out/r04p_tests.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_parity_gpu.py -k "fp32" \
  >> gpurun_out/r04p_tests.txt 2>&1 && \
timeout -k 10 300 python -u tools/site_table.py --prec fp32s > gpurun_out/r04p_s1.txt 2>&1 && \
CLIPK_LIB=build_ab/f32pf0/libclipk.so timeout -k 10 300 python -u tools/site_table.py --prec fp32s > gpurun_out/r04p_s0.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --prec fp32s --no-extra --no-cpu-baseline --no-configs --eval-images 5000 --steps 10 > gpurun_out/r04p_b1.json 2>/dev/null && \
CLIPK_LIB=build_ab/f32pf0/libclipk.so timeout -k 10 300 python -u bench.py --prec fp32s --no-extra --no-cpu-baseline --no-configs --eval-images 5000 --steps 10 > gpurun_out/r04p_b0.json 2>/dev/null
rc=$?
echo exit $rc
exit $rc
