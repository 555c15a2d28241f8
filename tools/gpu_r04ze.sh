# round-4 GPU pass: all-fp32 LayerNorm backward at 4 elements per lane (whole-wave contiguous 16-B
# loads) instead of 8: kernel tests + fp32 / fp32s parity fixtures on the default build, then
# fp32s bench lines new (default) vs base (build_ab/base: the previous layernorm.hip), interleaved
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  > gpurun_out/r04ze_tests.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_parity_gpu.py -k "fp32" \
  >> gpurun_out/r04ze_tests.txt 2>&1 && \
for v in new base new base; do
  if [ $v = new ]; then unset CLIPK_LIB; else export CLIPK_LIB=build_ab/$v/libclipk.so; fi
  timeout -k 10 300 python -u bench.py --prec fp32s --no-extra --no-cpu-baseline --no-configs --eval-images 2000 --steps 10 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels', {}); print('$v fp32s', d['value'], d['ms_per_step'], d['eval_images_per_sec'], 'ln_bwd', k.get('ln_bwd', {}).get('ms_per_step'), k.get('ln_bwd', {}).get('roof_frac'))" >> gpurun_out/r04ze_bench.txt || exit 1
done
echo exit 0
