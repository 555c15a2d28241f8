# round-4 GPU pass j: fp32s bench line with the fma_mix split (after r04i's site A/B)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --prec fp32s --no-extra --no-cpu-baseline --eval-images 5000 --steps 10 \
  > gpurun_out/r04j_bench_fp32s.json 2> gpurun_out/r04j_bench_fp32s.err && \
CLIPK_LIB=build_ab/mix0/libclipk.so timeout -k 10 300 python -u bench.py --prec fp32s --no-extra --no-cpu-baseline --eval-images 5000 --steps 10 \
  > gpurun_out/r04j_bench_fp32s_mix0.json 2>> gpurun_out/r04j_bench_fp32s.err
rc=$?
echo exit $rc
exit $rc
