# round-4 GPU pass: the interleaved lane-column map in the any-L fp32 forward (attn_fwd_f32:
# ViT under PREC fp32 / fp32s, plain text): kernel tests + fp32 parity fixtures on the default
# build, isolated times il1 (default) vs il0 (contiguous map), fp32s bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  > gpurun_out/r04z8_tests.txt 2>&1 && \
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_parity_gpu.py -k "fp32" \
  >> gpurun_out/r04z8_tests.txt 2>&1 && \
for v in il1 il0 il1 il0; do
  if [ $v = il1 ]; then unset CLIPK_LIB; else export CLIPK_LIB=build_ab/$v/libclipk.so; fi
  echo "$v $(timeout -k 10 120 python -u tools/attn_sweep.py --anyl 2>/dev/null | grep vit)" >> gpurun_out/r04z8_attn.txt || exit 1
done
for v in il1 il0 il1 il0; do
  if [ $v = il1 ]; then unset CLIPK_LIB; else export CLIPK_LIB=build_ab/$v/libclipk.so; fi
  timeout -k 10 300 python -u bench.py --prec fp32s --no-extra --no-cpu-baseline --no-configs --eval-images 2000 --steps 10 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['eval_images_per_sec'])" >> gpurun_out/r04z8_bench.txt || exit 1
done
echo exit 0
