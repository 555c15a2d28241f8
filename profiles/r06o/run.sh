# fp32s step: the ViT on the side stream (bench default) vs in line on the main stream, interleaved
set -o pipefail
mkdir -p gpurun_out/r06o
F='^>>\|Loading\|Use \|amdgpu.ids'
for i in 1 2 3; do
  for m in vit serial; do
    PREC=fp32s MODE=$m timeout -k 10 240 python -u tools/lab/vit_contention.py 30 2>&1 | grep -v "$F" >> gpurun_out/r06o/serial.txt || exit 1
  done
done
