# the small-M tile configuration (the ViT at 8 images, on the side stream): 64x128 (default) vs 128x128
set -o pipefail
O=gpurun_out/r05zi; mkdir -p $O
for r in 1 2; do
  for v in 7 0; do
    CLIPK_GEMM_SMALLM=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --eval-images 2000 > $O/fp16_s${v}_$r.json 2> $O/err.log || exit $?
    CLIPK_GEMM_SMALLM=$v timeout -k 10 200 python -u bench.py --prec fp32s --steps 10 --warmup 3 --no-extra --no-cpu-baseline --eval-images 1000 > $O/fp32s_s${v}_$r.json 2> $O/err.log || exit $?
  done
done
echo ok
