# round 6: fp32 prefix attention with its prefix K/V in dynamic LDS sized to P rows (occupancy 8 -> 10 / 12 -> 16
# waves per CU): attention tests, parity, bench (A/B against the previous build is profiles/r06h)
set -o pipefail
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_split_w16_gpu.py -q -k "prefix or split_copy" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_attn.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -q -k "cocoop or headline or prefix_input" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_parity.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --eval-images 5000 > $O/b_$r.json 2> $O/b_$r.err || exit 1
done
echo done
