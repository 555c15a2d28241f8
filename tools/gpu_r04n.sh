# round-4 GPU pass n: shared-prefix attention with the transposed operand reads issued at the top
# of each tile (and the prefix operand hoisted out of the loop) vs the per-operand reads
# (build_ab/tr0): prefix-attention kernel tests, the isolated kernels, the headline site table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k prefix \
  > gpurun_out/r04n_tests.txt 2>&1 && \
timeout -k 10 120 python -u tools/attn_sweep.py --one > gpurun_out/r04n_attn1.txt 2>&1 && \
CLIPK_LIB=build_ab/tr0/libclipk.so timeout -k 10 120 python -u tools/attn_sweep.py --one > gpurun_out/r04n_attn0.txt 2>&1 && \
timeout -k 10 120 python -u tools/attn_sweep.py --one >> gpurun_out/r04n_attn1.txt 2>&1 && \
CLIPK_LIB=build_ab/tr0/libclipk.so timeout -k 10 120 python -u tools/attn_sweep.py --one >> gpurun_out/r04n_attn0.txt 2>&1 && \
timeout -k 10 300 python -u tools/site_table.py > gpurun_out/r04n_s1.txt 2>&1 && \
CLIPK_LIB=build_ab/tr0/libclipk.so timeout -k 10 300 python -u tools/site_table.py > gpurun_out/r04n_s0.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_parity_gpu.py -k "not config" \
  > gpurun_out/r04n_parity.txt 2>&1
rc=$?
echo exit $rc
exit $rc
