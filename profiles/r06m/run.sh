# fp32s train step vs CLIPK_GEMM_SKEW (start delay of every other CU in the persistent GEMMs, us), interleaved
set -o pipefail
mkdir -p gpurun_out/r06m
for sk in 0 8 16 0 8 16 24; do
  echo "=== skew $sk" >> gpurun_out/r06m/skew.txt
  CLIPK_GEMM_SKEW=$sk PREC=fp32s MODE=vit timeout -k 10 240 python -u tools/lab/vit_contention.py 30 2>&1 | grep -v "^>>\|Loading\|Use \|amdgpu.ids" >> gpurun_out/r06m/skew.txt || exit 1
done
