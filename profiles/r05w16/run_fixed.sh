#!/bin/bash
# after the split hazard fix (compiler-visible split in the 2- / 4-slot loop; CLIPK_F32S16 on
# every tile path): per-path diff, the split / fold / w16 tests, the fp32s parity cases, A/B line
set -o pipefail
mkdir -p gpurun_out/r05w16
timeout -k 10 200 python -u tools/lab/w16_diff.py > gpurun_out/r05w16/diff_fixed.txt 2>&1 &&
timeout -k 10 700 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_lnfold_gpu.py \
  tests/test_split_w16_gpu.py tests/test_kernels_gpu.py -k "split or w16 or gamma or fold or qgelu" \
  > gpurun_out/r05w16/tests_fixed.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py -k fp32s \
  > gpurun_out/r05w16/parity_fp32s_fixed.txt 2>&1 &&
timeout -k 10 400 python -u tools/lab/fp32s_w16.py > gpurun_out/r05w16/ab_fixed.txt 2>&1
