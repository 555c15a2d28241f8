# round-4 GPU pass w: fp32s / fp32 bench lines after r04z2 read 256.8 / 120.5 (r04z: 278.1 / 127.7):
# current fp32 prefix attention vs the r04z one (build_ab/apz) and the prefetch-only one
# (build_ab/app), interleaved on one box
set -o pipefail
mkdir -p gpurun_out
b() { timeout -k 10 300 python -u bench.py --prec $1 --no-extra --no-cpu-baseline --no-configs --eval-images 2000 --steps 10 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', '$1', d['value'], d['ms_per_step'], d['eval_images_per_sec'])" >> gpurun_out/r04w.txt; }
b fp32s cur && CLIPK_LIB=build_ab/apz/libclipk.so b fp32s apz && CLIPK_LIB=build_ab/app/libclipk.so b fp32s app && \
b fp32s cur && CLIPK_LIB=build_ab/apz/libclipk.so b fp32s apz && CLIPK_LIB=build_ab/app/libclipk.so b fp32s app && \
b fp32 cur && CLIPK_LIB=build_ab/apz/libclipk.so b fp32 apz
rc=$?
echo exit $rc
exit $rc
