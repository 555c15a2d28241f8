# round-4 GPU pass: fp32 prefix forward keys per wave-uniform bound (1 = previous build, 2 =
# default, 4): prefix tests on the default, isolated kernel times, fp32s bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "prefix" \
  > gpurun_out/r04z6_tests.txt 2>&1 && \
for v in kg2 kg1 kg4 kg2 kg1 kg4; do
  if [ $v = kg2 ]; then unset CLIPK_LIB; else export CLIPK_LIB=build_ab/$v/libclipk.so; fi
  echo "$v $(SWEEP_DTYPE=fp32 timeout -k 10 120 python -u tools/attn_sweep.py --one 2>/dev/null | grep rows)" >> gpurun_out/r04z6_attn.txt || exit 1
done
for v in kg2 kg1 kg4; do
  if [ $v = kg2 ]; then unset CLIPK_LIB; else export CLIPK_LIB=build_ab/$v/libclipk.so; fi
  timeout -k 10 300 python -u bench.py --prec fp32s --no-extra --no-cpu-baseline --no-configs --eval-images 2000 --steps 10 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['eval_images_per_sec'])" >> gpurun_out/r04z6_bench.txt || exit 1
done
echo exit 0
