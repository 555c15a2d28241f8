# round-4 GPU pass: fp32-gradient text backward without the dX_lp copy (the input-grad GEMMs
# read the fp32 residual gradient dX itself): the whole -m gpu suite on the default build, then
# fp32s / fp32 bench lines new (default) vs base (build_ab/base: the previous encoder), interleaved
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests \
  > gpurun_out/r04za_tests.txt 2>&1 && \
for v in new base new base; do
  if [ $v = new ]; then unset CLIPK_LIB; else export CLIPK_LIB=build_ab/$v/libclipk.so; fi
  timeout -k 10 300 python -u bench.py --prec fp32s --no-extra --no-cpu-baseline --no-configs --eval-images 2000 --steps 10 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v fp32s', d['value'], d['ms_per_step'], d['eval_images_per_sec'], json.dumps({k: v['ms_per_step'] for k, v in d.get('kernels', {}).items()}))" >> gpurun_out/r04za_bench.txt || exit 1
done
for v in new base; do
  if [ $v = new ]; then unset CLIPK_LIB; else export CLIPK_LIB=build_ab/$v/libclipk.so; fi
  timeout -k 10 300 python -u bench.py --prec fp32 --no-extra --no-cpu-baseline --no-configs --eval-images 1000 --steps 5 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v fp32', d['value'], d['ms_per_step'])" >> gpurun_out/r04za_bench.txt || exit 1
done
echo exit 0
