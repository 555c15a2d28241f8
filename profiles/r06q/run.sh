# fp32s step: the next batch's side-stream ViT started after this step's forward (default) or
# before it (CLIPK_PREFETCH_EARLY=1: an A/B knob in trainers/cocoop.py for this run only, removed
# afterwards), interleaved
set -o pipefail
mkdir -p gpurun_out/r06q
F='^>>\|Loading\|Use \|amdgpu.ids'
for i in 1 2 3; do
  for e in 0 1; do
    echo "=== early $e" >> gpurun_out/r06q/early.txt
    CLIPK_PREFETCH_EARLY=$e PREC=fp32s MODE=vit timeout -k 10 240 python -u tools/lab/vit_contention.py 30 2>&1 | grep -v "$F" >> gpurun_out/r06q/early.txt || exit 1
  done
done
