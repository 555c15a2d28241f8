#!/bin/bash
# the 2-MFMA kernel on every tile path (CLIPK_W16_ALL=1): as built, with the cvt+sub+cvt split
# (no v_fma_mix partial writes), and with s_nop 7 after each split in the 2-/4-slot loop
set -o pipefail
mkdir -p gpurun_out/r05w16
for v in w16all w16mix0 w16nop; do
  echo "== $v" >> gpurun_out/r05w16/hazard.txt
  CLIPK_LIB=$(pwd)/build_ab/$v/libclipk.so timeout -k 10 200 python -u tools/lab/w16_diff.py >> gpurun_out/r05w16/hazard.txt 2>&1 || exit 1
done
