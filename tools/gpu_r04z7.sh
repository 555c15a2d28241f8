# round-4 GPU pass: fp32 prefix kernels' interleaved lane-column map (il1, default: the 4
# lanes of a row cover 64 contiguous bytes per f32x4 load) vs the contiguous map (il0:
# lane s holds columns 16 s .. 16 s + 15): the GPU suite on the default, isolated kernel
# times, fp32s bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests \
  > gpurun_out/r04z7_tests.txt 2>&1 && \
for v in il1 il0 il1 il0 il1 il0; do
  if [ $v = il1 ]; then unset CLIPK_LIB; else export CLIPK_LIB=build_ab/$v/libclipk.so; fi
  echo "$v $(SWEEP_DTYPE=fp32 timeout -k 10 120 python -u tools/attn_sweep.py --one 2>/dev/null | grep rows)" >> gpurun_out/r04z7_attn.txt || exit 1
done
for v in il1 il0 il1 il0; do
  if [ $v = il1 ]; then unset CLIPK_LIB; else export CLIPK_LIB=build_ab/$v/libclipk.so; fi
  timeout -k 10 300 python -u bench.py --prec fp32s --no-extra --no-cpu-baseline --no-configs --eval-images 2000 --steps 10 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['eval_images_per_sec'])" >> gpurun_out/r04z7_bench.txt || exit 1
done
echo exit 0
