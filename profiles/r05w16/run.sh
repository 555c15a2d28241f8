#!/bin/bash
# PREC fp32s on fp16-valued weights (CLIPK_F32S16): MFMA zero-product lab, the per-path diff,
# the bitwise / oracle tests, then the A/B line
set -o pipefail
mkdir -p gpurun_out/r05w16
timeout -k 10 60 ./tools/lab/mfma_zero > gpurun_out/r05w16/mfma_zero.txt 2>&1 &&
timeout -k 10 200 python -u tools/lab/w16_diff.py > gpurun_out/r05w16/diff_fenced.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_split_w16_gpu.py \
  > gpurun_out/r05w16/tests.txt 2>&1 &&
timeout -k 10 400 python -u tools/lab/fp32s_w16.py > gpurun_out/r05w16/ab.txt 2>&1
