# 96-row deep-ring tiles for better-filled one-round grids (CLIPK_GEMM_T96): split-GEMM tests
# incl. 96 vs 128 bitwise, then the batch-1 fp32s step interleaved on / off, and the headline step
set -o pipefail
mkdir -p gpurun_out/r06v
F='^>>\|Loading\|Use \|amdgpu.ids'
timeout -k 10 700 python -u -m pytest tests/test_split_w16_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06v/tests.txt 2>&1 || { tail -30 gpurun_out/r06v/tests.txt; exit 1; }
tail -1 gpurun_out/r06v/tests.txt
for i in 1 2 3; do
  for t in 1 0; do
    echo "=== t96 $t batch 1" >> gpurun_out/r06v/ab.txt
    CLIPK_GEMM_T96=$t BATCH=1 PREC=fp32s MODE=vit timeout -k 10 240 python -u tools/lab/vit_contention.py 100 2>&1 | grep -v "$F" >> gpurun_out/r06v/ab.txt || exit 1
  done
done
for t in 1 0; do
  echo "=== t96 $t batch 8" >> gpurun_out/r06v/ab.txt
  CLIPK_GEMM_T96=$t PREC=fp32s MODE=vit timeout -k 10 240 python -u tools/lab/vit_contention.py 30 2>&1 | grep -v "$F" >> gpurun_out/r06v/ab.txt || exit 1
done
