#!/bin/bash
# split mode 2 with the LayerNorm fold's gamma on A (clipk_gemm_ln_gamma): GEMM-level and
# end-to-end tests, the fp32s parity cases, then the A/B line
set -o pipefail
mkdir -p gpurun_out/r05w16
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_lnfold_gpu.py \
  tests/test_split_w16_gpu.py > gpurun_out/r05w16/tests_gamma.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py -k fp32s \
  > gpurun_out/r05w16/parity_fp32s.txt 2>&1 &&
timeout -k 10 400 python -u tools/lab/fp32s_w16.py > gpurun_out/r05w16/ab_gamma.txt 2>&1
