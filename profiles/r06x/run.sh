# CLIPK_GEMM_EPI_OVL=1 build (build_ab/epiovl): the next tile's step-1 B0 staged before the
# epilogue, whose stores then drain through two K steps; split-GEMM tests and the headline
# parity under it, then the fp32s step A/B and per-tile stamps against the default build
set -o pipefail
mkdir -p gpurun_out/r06x
F='^>>\|Loading\|Use \|amdgpu.ids'
V=$PWD/build_ab/epiovl/libclipk.so
CLIPK_LIB=$V timeout -k 10 900 python -u -m pytest tests/test_split_w16_gpu.py tests/test_lnfold_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06x/tests.txt 2>&1 || { tail -30 gpurun_out/r06x/tests.txt; exit 1; }
tail -1 gpurun_out/r06x/tests.txt
CLIPK_LIB=$V timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fp32s" > gpurun_out/r06x/tests_parity.txt 2>&1 || { tail -30 gpurun_out/r06x/tests_parity.txt; exit 1; }
tail -1 gpurun_out/r06x/tests_parity.txt
for i in 1 2 3; do
  for v in ovl def; do
    L=""; [ $v = ovl ] && L=$V
    echo "=== $v" >> gpurun_out/r06x/ab.txt
    CLIPK_LIB=$L PREC=fp32s MODE=vit timeout -k 10 240 python -u tools/lab/vit_contention.py 30 2>&1 | grep -v "$F" >> gpurun_out/r06x/ab.txt || exit 1
  done
done
for e in 5 4; do
  echo "=== ovl" >> gpurun_out/r06x/stamps.txt
  CLIPK_LIB=$V CLIPK_GEMM_STAMP=1 CLIPK_GEMM_STAMP_EPI=$e CLIPK_GEMM_STAMP_MINM=40000 PREC=fp32s timeout -k 10 240 python -u tools/lab/step_stamps.py 5 2>&1 | grep -v "$F" >> gpurun_out/r06x/stamps.txt || exit 1
done
