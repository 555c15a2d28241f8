# round-4 GPU pass c: split GEMM tests + fp32s headline parity, then the fp32s / fp32 bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py -k "split" tests/test_parity_gpu.py::test_headline_shape_vs_oracle \
  tests/test_parity_gpu.py::test_cocoop_full > gpurun_out/r04c_tests.txt 2>&1 && \
timeout -k 10 250 python -u bench.py --prec fp32s --no-extra --no-cpu-baseline --eval-images 5000 --steps 10 \
  > gpurun_out/r04c_bench_fp32s.json 2> gpurun_out/r04c_bench_fp32s.err && \
timeout -k 10 300 python -u tools/site_table.py --prec fp32s > gpurun_out/r04c_sites_fp32s.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --prec fp32 --no-extra --no-cpu-baseline --eval-images 2000 --steps 10 \
  > gpurun_out/r04c_bench_fp32.json 2> gpurun_out/r04c_bench_fp32.err
rc=$?
echo exit $rc
exit $rc
