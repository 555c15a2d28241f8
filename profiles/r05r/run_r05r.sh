# in-kernel LN statistics merge (clipk_gemm_ln_merge): kernel tests, the LN-fold / parity suites,
# then batch-1 and headline bench A/B against CLIPK_LN_MERGE_FUSED=0
set -o pipefail
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_lnfold_gpu.py tests/test_parity_gpu.py tests/test_kernels_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1 || exit $?
for r in 1 2; do
  for f in 1 0; do
    CLIPK_LN_MERGE_FUSED=$f timeout -k 10 200 python -u bench.py --batch 1 --steps 50 --warmup 5 --no-extra --no-cpu-baseline \
      --eval-images 100 > $O/b1_f${f}_$r.json 2> $O/b1_f${f}_$r.err || exit $?
  done
done
echo ok
