# split-form epilogue stores by v_fma_mix + the split scale on the LayerNorm fold's rstd:
# whole -m gpu suite on the new build, then same-box A/B of the fp32s step against the
# convert / subtract build (build_ab/cvtsplit, -DCLIPK_EPI_MIXSPLIT=0) and per-tile stamps
set -o pipefail
mkdir -p gpurun_out/r06n
F='^>>\|Loading\|Use \|amdgpu.ids'
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06n/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r06n/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r06n/gpu_tests.txt
OLD=$PWD/build_ab/cvtsplit/libclipk.so
for i in 1 2 3; do
  for v in new old; do
    L=""; [ $v = old ] && L=$OLD
    echo "=== $v" >> gpurun_out/r06n/ab.txt
    CLIPK_LIB=$L PREC=fp32s MODE=vit timeout -k 10 240 python -u tools/lab/vit_contention.py 30 2>&1 | grep -v "$F" >> gpurun_out/r06n/ab.txt || exit 1
  done
done
for v in new old; do
  L=""; [ $v = old ] && L=$OLD
  for e in 5 6 1; do
    echo "=== $v" >> gpurun_out/r06n/stamps.txt
    CLIPK_LIB=$L CLIPK_GEMM_STAMP=1 CLIPK_GEMM_STAMP_EPI=$e CLIPK_GEMM_STAMP_MINM=40000 PREC=fp32s timeout -k 10 240 python -u tools/lab/step_stamps.py 5 2>&1 | grep -v "$F" >> gpurun_out/r06n/stamps.txt || exit 1
  done
done
