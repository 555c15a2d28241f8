#!/bin/bash
# SQ / LDS / MFMA counters of one yardstick shape (default fc_dx) for the in-tree library and
# variants: tools/gemm_pmc.sh <shape> tag ...  -> gpurun_out/gemm_pmc/<tag>/
R=$(pwd)
SHAPE=$1; shift
mkdir -p $R/gpurun_out/gemm_pmc
cd /tmp && export TMPDIR=/tmp
for t in "$@"; do
  case $t in base) L="";; *) L=$R/build_ab/$t/libclipk.so;; esac
  CLIPK_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d $R/gpurun_out/gemm_pmc/$t -o p -- python3 $R/tools/gemm_yardstick.py --no-ref --only $SHAPE \
    > $R/gpurun_out/gemm_pmc/$t.log 2>&1 || exit 1
done
