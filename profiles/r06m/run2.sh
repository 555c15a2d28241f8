# fp32s train step: per-tile stamps of the persistent GEMM classes (EPI 5 c_fc, 6 dgelu, 4 dx,
# 1 residual producers, 0 qkv), then CLIPK_GEMM_SKEW now reaching the split GEMMs, interleaved
set -o pipefail
mkdir -p gpurun_out/r06m
F='^>>\|Loading\|Use \|amdgpu.ids'
for e in 5 6 4 1 0; do
  CLIPK_GEMM_STAMP=1 CLIPK_GEMM_STAMP_EPI=$e CLIPK_GEMM_STAMP_MINM=40000 PREC=fp32s timeout -k 10 240 python -u tools/lab/step_stamps.py 5 2>&1 | grep -v "$F" >> gpurun_out/r06m/stamps.txt || exit 1
done
for sk in 0 6 12 0 6 12; do
  echo "=== skew $sk" >> gpurun_out/r06m/skew_split.txt
  CLIPK_GEMM_SKEW=$sk PREC=fp32s MODE=vit timeout -k 10 240 python -u tools/lab/vit_contention.py 30 2>&1 | grep -v "$F" >> gpurun_out/r06m/skew_split.txt || exit 1
done
