#!/bin/bash
# CLIPK_F32S16 vs CLIPK_F32S across tile paths, with the zero product skipped (base) and kept (w16keep)
set -o pipefail
mkdir -p gpurun_out/r05w16
timeout -k 10 200 python -u tools/lab/w16_diff.py > gpurun_out/r05w16/diff_base.txt 2>&1 &&
CLIPK_LIB=$(pwd)/build_ab/w16keep/libclipk.so timeout -k 10 200 python -u tools/lab/w16_diff.py > gpurun_out/r05w16/diff_keep.txt 2>&1
