#!/bin/bash
# s_nop 4 after the ping-pong loop's asm split (CLIPK_PP_SPLIT_NOP=5) vs none: the fp32s line
set -o pipefail
mkdir -p gpurun_out/r05w16
timeout -k 10 300 python -u tools/lab/fp32s_w16.py > gpurun_out/r05w16/ppnop_base.txt 2>&1 &&
CLIPK_LIB=$(pwd)/build_ab/ppnop/libclipk.so timeout -k 10 300 python -u tools/lab/fp32s_w16.py > gpurun_out/r05w16/ppnop_nop.txt 2>&1
