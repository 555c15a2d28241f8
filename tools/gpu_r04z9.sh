# round-4 GPU pass: LayerNorm fold under PREC fp32s (fp32 residual stream, split-packed W'):
# fold tests + fp32s parity fixtures, then fp32s bench lines fold on (default) vs off
# (FSP_LN_FOLD=0: the LayerNorm passes), interleaved
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_lnfold_gpu.py \
  > gpurun_out/r04z9_tests.txt 2>&1 && \
timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_parity_gpu.py -k "fp32s" -s \
  >> gpurun_out/r04z9_tests.txt 2>&1 && \
for v in on off on off; do
  if [ $v = on ]; then unset FSP_LN_FOLD; else export FSP_LN_FOLD=0; fi
  timeout -k 10 300 python -u bench.py --prec fp32s --no-extra --no-cpu-baseline --no-configs --eval-images 2000 --steps 10 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['eval_images_per_sec'], json.dumps({k: v['ms_per_step'] for k, v in d.get('kernels', {}).items()}))" >> gpurun_out/r04z9_bench.txt || exit 1
done
echo exit 0
