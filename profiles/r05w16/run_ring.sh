#!/bin/bash
# 128x128 tiles: the 4-slot ring (CLIPK_GEMM_DEEP=1, default) vs the 2-slot loop on the same inputs
set -o pipefail
mkdir -p gpurun_out/r05w16
timeout -k 10 120 python -u tools/lab/ring_dump.py gpurun_out/r05w16/ring1.pt > gpurun_out/r05w16/ring.txt 2>&1 &&
CLIPK_GEMM_DEEP=0 timeout -k 10 120 python -u tools/lab/ring_dump.py gpurun_out/r05w16/ring0.pt >> gpurun_out/r05w16/ring.txt 2>&1 &&
timeout -k 10 120 python -u tools/lab/ring_dump.py --cmp gpurun_out/r05w16/ring1.pt gpurun_out/r05w16/ring0.pt >> gpurun_out/r05w16/ring.txt 2>&1 &&
rm -f gpurun_out/r05w16/ring*.pt
