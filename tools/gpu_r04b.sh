# round-4 GPU pass b: split GEMM kernel tests, every fp32 / fp32s parity fixture (the fp32
# prefix attention kernels were rewritten), then per-site times of PREC fp32s and fp32.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py -k "split" > gpurun_out/r04b_split.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
  tests/test_parity_gpu.py -k "(fp32s or fp32) and not config" > gpurun_out/r04b_fp32.txt 2>&1 && \
timeout -k 10 300 python -u tools/site_table.py --prec fp32s > gpurun_out/r04b_sites_fp32s.txt 2>&1 && \
timeout -k 10 300 python -u tools/site_table.py --prec fp32 > gpurun_out/r04b_sites_fp32.txt 2>&1
rc=$?
echo exit $rc
exit $rc
