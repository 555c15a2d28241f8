# round 5: fp32s with the activation operand's lo part dropped (build_ab/terms2: every GEMM;
# terms2bwd: the backward's input-grad GEMMs) -- parity against the reference outputs and speed
set -o pipefail
O=gpurun_out/r05h
mkdir -p $O
for v in base terms2 terms2bwd; do
  L=""; [ $v != base ] && L=$(pwd)/build_ab/$v/libclipk.so
  CLIPK_LIB=$L timeout -k 10 300 python -u -m pytest -s -q -p no:cacheprovider --timeout 250 --timeout-method thread \
    "tests/test_parity_gpu.py::test_headline_batch8_vs_golden[fp32s]" \
    "tests/test_parity_gpu.py::test_cocoop_full[cocoop_vitb16_c4-fp32s-packed]" \
    "tests/test_parity_gpu.py::test_coop_full[coop_vitb16_c6_focal-fp32s-packed]" > $O/parity_$v.txt 2>&1
  rc=$?; [ $rc -gt 1 ] && exit $rc
  CLIPK_LIB=$L timeout -k 10 300 python -u bench.py --prec fp32s --steps 10 --warmup 3 --no-extra --no-cpu-baseline \
    --eval-images 2000 > $O/bench_$v.json 2> $O/bench_$v.err || exit $?
done
echo done
