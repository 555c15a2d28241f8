#!/bin/bash
# GEMM loop diagnostics on the GPU box: the text-shape yardstick on the in-tree library and on
# diagnostic variants (tools/build_variant.sh), cold (A rotated through HBM) and hot.
#   tools/gemm_diag.sh tag1 tag2 ...   -> gpurun_out/gemm_diag.log
R=$(pwd)
mkdir -p gpurun_out
for t in "$@"; do
  # cfgN = the in-tree library with CLIPK_GEMM_CFG=N (tile configuration forced)
  case $t in
    base) L=""; CFG="";;
    env:*) L=""; CFG=""; export ${t#env:};;
    cfg*) L=""; CFG=${t#cfg};;
    *) L=$R/build_ab/$t/libclipk.so; CFG="";;
  esac
  for mode in "" ${HOT:+--hot}; do
    echo "== $t $mode" >> gpurun_out/gemm_diag.log
    if [ -n "$CFG" ]; then export CLIPK_GEMM_CFG=$CFG; else unset CLIPK_GEMM_CFG; fi
    CLIPK_LIB=$L timeout -k 10 200 python -u tools/gemm_yardstick.py --no-ref $mode >> gpurun_out/gemm_diag.log 2>&1 || exit 1
  done
done
