# CLIPK_EPI_NOWAIT=1 build (build_ab/nowait): GEMM epilogue transposes without the two
# lgkmcnt(0) waits per row group; GEMM / split / fold / parity tests under it, then the fp32s and
# fp16 step A/B against the default build
set -o pipefail
mkdir -p gpurun_out/r06y
F='^>>\|Loading\|Use \|amdgpu.ids'
V=$PWD/build_ab/nowait/libclipk.so
CLIPK_LIB=$V timeout -k 10 900 python -u -m pytest tests/test_split_w16_gpu.py tests/test_lnfold_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06y/tests.txt 2>&1 || { tail -30 gpurun_out/r06y/tests.txt; exit 1; }
tail -1 gpurun_out/r06y/tests.txt
CLIPK_LIB=$V timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gemm" > gpurun_out/r06y/tests_gemm.txt 2>&1 || { tail -30 gpurun_out/r06y/tests_gemm.txt; exit 1; }
tail -1 gpurun_out/r06y/tests_gemm.txt
CLIPK_LIB=$V timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "headline" > gpurun_out/r06y/tests_parity.txt 2>&1 || { tail -30 gpurun_out/r06y/tests_parity.txt; exit 1; }
tail -1 gpurun_out/r06y/tests_parity.txt
for i in 1 2 3; do
  for v in nowait def; do
    L=""; [ $v = nowait ] && L=$V
    echo "=== $v" >> gpurun_out/r06y/ab.txt
    CLIPK_LIB=$L PREC=fp32s MODE=vit timeout -k 10 240 python -u tools/lab/vit_contention.py 30 2>&1 | grep -v "$F" >> gpurun_out/r06y/ab.txt || exit 1
  done
done
for v in nowait def; do
  L=""; [ $v = nowait ] && L=$V
  echo "=== $v fp16" >> gpurun_out/r06y/ab.txt
  CLIPK_LIB=$L PREC=fp16 MODE=vit timeout -k 10 240 python -u tools/lab/vit_contention.py 30 2>&1 | grep -v "$F" >> gpurun_out/r06y/ab.txt || exit 1
done
