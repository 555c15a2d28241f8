# round-4 GPU pass h: fp32 attention waves per block (CLIPK_F32ATTN_WPB 2 / 4 / 8) on the fp32s
# headline, interleaved; fp32 prefix-attention kernel tests first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k prefix \
  > gpurun_out/r04h_tests.txt 2>&1 && \
CLIPK_F32ATTN_WPB=2 timeout -k 10 300 python -u tests/../tools/site_table.py --prec fp32s > gpurun_out/r04h_w2.txt 2>&1 && \
CLIPK_F32ATTN_WPB=4 timeout -k 10 300 python -u tools/site_table.py --prec fp32s > gpurun_out/r04h_w4.txt 2>&1 && \
CLIPK_F32ATTN_WPB=8 timeout -k 10 300 python -u tools/site_table.py --prec fp32s > gpurun_out/r04h_w8.txt 2>&1 && \
CLIPK_F32ATTN_WPB=2 timeout -k 10 300 python -u tools/site_table.py --prec fp32s >> gpurun_out/r04h_w2.txt 2>&1
rc=$?
echo exit $rc
exit $rc
