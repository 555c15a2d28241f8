# round-4 GPU pass i: split lo part by mixed-precision FMA (CLIPK_SPLIT_MIX 1) vs the cvt + sub
# form (build_ab/mix0): split GEMM tests, then the fp32s step site table interleaved, ViT timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "split" \
  > gpurun_out/r04i_tests.txt 2>&1 && \
timeout -k 10 300 python -u tools/site_table.py --prec fp32s > gpurun_out/r04i_mix1.txt 2>&1 && \
CLIPK_LIB=build_ab/mix0/libclipk.so timeout -k 10 300 python -u tools/site_table.py --prec fp32s > gpurun_out/r04i_mix0.txt 2>&1 && \
timeout -k 10 300 python -u tools/site_table.py --prec fp32s >> gpurun_out/r04i_mix1.txt 2>&1 && \
CLIPK_LIB=build_ab/mix0/libclipk.so timeout -k 10 300 python -u tools/site_table.py --prec fp32s >> gpurun_out/r04i_mix0.txt 2>&1 && \
timeout -k 10 300 python -u tools/vit_time.py > gpurun_out/r04i_vit.txt 2>&1
rc=$?
echo exit $rc
exit $rc
